#!/bin/bash
# GPU tests + smoke on the current build, then the phase stamps and FoV bench lines against the
# previous commit's library (build/base*). Run from the repo root.   bash tools/r04_check.sh <tag>
set -e -o pipefail
TAG=${1:-r04chk}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/$TAG
echo "[$(date +%T)] pytest"
timeout -k 10 420 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || echo "pytest rc=$?"
tail -3 gpurun_out/$TAG/pytest.log
echo "[$(date +%T)] smoke"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
tail -2 gpurun_out/$TAG/smoke.log
for v in base_stamps stamps; do
  MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > gpurun_out/$TAG/stamps_coll_$v.log 2>&1
  WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > gpurun_out/$TAG/stamps_fov_$v.log 2>&1
done
A="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/base/libmpccbf.so"
B="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
bash tools/gpu_ab.sh $TAG/fov "--workload fov --steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh $TAG/fovs "--workload fov --slack --steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh $TAG/coll "--steps 300 --warmup 20" "$A" "$B"
python3 tools/ab_summary.py gpurun_out/$TAG/fov gpurun_out/$TAG/fovs gpurun_out/$TAG/coll
for f in gpurun_out/$TAG/stamps_*.log; do echo "== $f"; sed -n '2,10p' $f; done
