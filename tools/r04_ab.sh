#!/bin/bash
# Round-4 A/B on one box (run from the repo root): bench lines of the previous commit's library
# (build/base, built from `git archive HEAD`) against the current one, interleaved
# (tools/gpu_ab.sh); the phase stamps of both (build/base_stamps, build/stamps); then the GPU
# tests on the current build.
#   bash tools/r04_ab.sh <tag> [notest]
set -e -o pipefail
TAG=${1:-r04ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
A="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/base/libmpccbf.so"
B="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
for v in base ""; do
  echo "[$(date +%T)] gs dump ${v:-new}"
  MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/gs_dump.py all gpurun_out/${TAG}_gs_all_${v:-new}.npz > gpurun_out/${TAG}_gs_${v:-new}.log 2>&1
done
bash tools/gpu_ab.sh ${TAG}_driver "--steps 20 --warmup 5" "$A" "$B"
bash tools/gpu_ab.sh ${TAG}_fov "--workload fov --steps 200 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh ${TAG}_share "--rank-share 8 --agents-total 8192 --steps 300 --warmup 20" "$A" "$B"
python3 tools/ab_summary.py gpurun_out/${TAG}_driver gpurun_out/${TAG}_fov gpurun_out/${TAG}_share
for v in base_stamps stamps; do
  echo "[$(date +%T)] stamps $v"
  MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > gpurun_out/${TAG}_stamps_coll_$v.log 2>&1
  WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > gpurun_out/${TAG}_stamps_fov_$v.log 2>&1
done
if [ "$2" != "notest" ]; then
  echo "[$(date +%T)] pytest"
  timeout -k 10 420 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  tail -3 gpurun_out/${TAG}_pytest.log
fi
