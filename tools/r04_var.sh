#!/bin/bash
# A/B of kernel variants on one box (run from the repo root): phase stamps of the stamps builds
# (build/base_stamps, build/stamps, build/stamps_<V>) and bench lines of the release builds
# (build/base, build/, build/rel_<V>), interleaved.
#   bash tools/r04_var.sh <tag> "<stamps variants>" "<release variants>"
set -e -o pipefail
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/$TAG
for r in 1 2; do
  for v in $2; do
    echo "[$(date +%T)] stamps $v ($r)"
    MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > gpurun_out/$TAG/stamps_${v}_$r.log 2>&1
  done
done
envs=()
for v in $3; do envs+=("MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so"); done
bash tools/gpu_ab.sh ${TAG}/driver "--steps 300 --warmup 20" "${envs[@]}"
python3 tools/ab_summary.py gpurun_out/${TAG}/driver
for f in gpurun_out/$TAG/stamps_*_1.log; do echo "== $f"; sed -n '2,10p' $f; done
