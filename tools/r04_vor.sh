#!/bin/bash
# A/B of the FoV kernel's Voronoi operators copied into LDS at setup: FoV tests, FoV and FoV slack
# bench lines of build/base (previous commit) vs the current build, interleaved; FoV phase stamps
# of both stamps builds.   bash tools/r04_vor.sh <tag>
set -e -o pipefail
TAG=${1:-r04vor}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -k "fov" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
A="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/base/libmpccbf.so"
B="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
bash tools/gpu_ab.sh $TAG/fov "--workload fov --steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh $TAG/fovs "--workload fov --slack --steps 300 --warmup 20" "$A" "$B"
python3 tools/ab_summary.py $O/fov $O/fovs
for v in base_stamps stamps; do
  WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $O/stamps_fov_$v.log 2>&1
done
