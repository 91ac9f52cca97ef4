#!/bin/bash
# A/B of a fresh curve's next state from the AZ / AS rows (build/rel_AZ, build/stamps_AZ) against the
# committed build, plus the GPU tests on the variant. Run from the repo root.
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=$ROOT/gpurun_out/r04az
mkdir -p $O
MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/rel_AZ/libmpccbf.so timeout -k 10 420 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || echo "pytest failed"
tail -3 $O/pytest.log
A="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
B="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/rel_AZ/libmpccbf.so"
bash tools/gpu_ab.sh r04az/coll "--steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh r04az/share "--rank-share 8 --agents-total 8192 --steps 300 --warmup 20" "$A" "$B"
python3 tools/ab_summary.py $O/coll $O/share
for v in stamps stamps_AZ; do
  MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > $O/stamps_$v.log 2>&1
  sed -n '2,10p' $O/stamps_$v.log
done
