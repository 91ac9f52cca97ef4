# A/B: HEAD library (build/base) vs the working tree (16-lane one-round-trip query, wide staging
# overlap): config 3 and the 8-rank share, interleaved twice; then the GPU tests and stamps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05m
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python3 bench.py --no-cpu-baseline --no-trace --steps 400 --warmup 50"
for rep in 1 2; do
  for v in base new; do
    L=mpc-cbf_amd/build/libmpccbf.so; [ $v = base ] && L=mpc-cbf_amd/build/base/libmpccbf.so
    MPCCBF_LIB=$L timeout -k 10 200 $B > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit 1
    MPCCBF_LIB=$L timeout -k 10 200 $B --rank-share 8 --agents-total 8192 > $OUT/sh_${v}_$rep.json 2> $OUT/sh_${v}_$rep.err || exit 2
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 3
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 4096 100 0 > $OUT/stamps4096.log 2>&1 || exit 4
