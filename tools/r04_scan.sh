#!/bin/bash
# A/B of the wave active set with batched LDS reads (row scan, P^-1 / P row products): FoV and FoV
# slack bench lines of build/base (previous commit) vs the current build, interleaved; the FoV
# active-set phase stamps of both prof builds; the FoV GPU tests.   bash tools/r04_scan.sh <tag>
set -e -o pipefail
TAG=${1:-r04scan}
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
for v in base_prof prof; do
  WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $O/stamps_fov_das_$v.log 2>&1
  WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/${v/prof/stamps}/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $O/stamps_fov_$v.log 2>&1
done
for f in $O/stamps_fov_das_*.log; do echo "== $f"; grep -A12 "with 1 step" $f | head -12; done
