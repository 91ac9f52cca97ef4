# A/B of the collision kernel (default build vs build/${1:-nokw}): GPU tests first, then bench lines
# on the driver command and at 300 steps, 2 rounds interleaved. The alternative library is built
# beforehand, e.g. from a stashed tree: make -C mpc-cbf_amd BUILD=build/base build/base/libmpccbf.so
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
ALT=${1:-nokw}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/ab_pytest.log 2>&1
B="python3 bench.py --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 120 $B --steps 20 --warmup 5 > $O/ab_new_drv_$r.json 2> $O/ab_new_drv_$r.err
  MPCCBF_LIB=$PWD/mpc-cbf_amd/build/$ALT/libmpccbf.so timeout -k 10 120 $B --steps 20 --warmup 5 > $O/ab_old_drv_$r.json 2> $O/ab_old_drv_$r.err
  timeout -k 10 120 $B --steps 300 --warmup 20 > $O/ab_new_300_$r.json 2> $O/ab_new_300_$r.err
  MPCCBF_LIB=$PWD/mpc-cbf_amd/build/$ALT/libmpccbf.so timeout -k 10 120 $B --steps 300 --warmup 20 > $O/ab_old_300_$r.json 2> $O/ab_old_300_$r.err
done
echo done
