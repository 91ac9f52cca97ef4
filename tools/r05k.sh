# dense path: tests, bench, profile (zero-copy pinned input)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05k}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_dense_qp.py tests/test_qpcpp_adapter.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_dense.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 200 python3 bench.py --workload dense --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_dense.json 2> $OUT/bench_dense.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $OUT/prof_dense -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload dense --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_dense_prof.json 2> $OUT/bench_dense_prof.err || exit 3
