# A/B: HEAD library (build/base) vs the working tree (iteration-1 CBF rows in one pass over the
# (sample, neighbour) pairs), config 3 interleaved twice; parity tests; stamps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05p}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python3 bench.py --no-cpu-baseline --no-trace --steps 400 --warmup 50"
for rep in 1 2; do
  for v in base new; do
    L=mpc-cbf_amd/build/libmpccbf.so; [ $v = base ] && L=mpc-cbf_amd/build/base/libmpccbf.so
    MPCCBF_LIB=$L timeout -k 10 200 $B > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit 1
    MPCCBF_LIB=$L timeout -k 10 200 $B --crowded > $OUT/cr_${v}_$rep.json 2> $OUT/cr_${v}_$rep.err || exit 2
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 3
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 4096 100 0 > $OUT/stamps4096.log 2>&1 || exit 4
