#!/bin/bash
# A/B of the collision CBF rows' sample terms (ego state, U_k s0) formed once per group into LDS:
# the GPU tests, config 3 and the config-4 share of build/base (previous commit) vs the current
# build, interleaved; collision phase stamps of both stamps builds.   bash tools/r04_smp.sh <tag>
set -e -o pipefail
TAG=${1:-r04smp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
A="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/base/libmpccbf.so"
B="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
bash tools/gpu_ab.sh $TAG/c3 "--steps 300 --warmup 20 --no-cpu-baseline" "$A" "$B"
bash tools/gpu_ab.sh $TAG/share "--agents-total 8192 --rank-share 8 --steps 300 --warmup 20 --no-cpu-baseline" "$A" "$B"
python3 tools/ab_summary.py $O/c3 $O/share
for v in base_stamps stamps; do
  MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > $O/stamps_c3_$v.log 2>&1
done
