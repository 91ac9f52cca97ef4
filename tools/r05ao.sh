# dense A/B from its own builds (build/abtest, build/abtestprof): tests, stamps, bench
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05ao}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/abtest/libmpccbf.so
MPCCBF_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_dense_qp.py tests/test_qpcpp_adapter.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_dense.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 1
MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/abtestprof/libmpccbf.so MPCCBF_DENSE_STAMPS=1 timeout -k 10 120 python3 tools/dense_stamps.py 20 1 > $OUT/stamps1.log 2> $OUT/stamps1.err || exit 2
for i in 1 2; do MPCCBF_LIB=$L timeout -k 10 200 python3 bench.py --workload dense --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_dense_$i.json 2> $OUT/bench_dense_$i.err || exit 3; done
