#!/bin/bash
# A/B timing of bench lines under environment settings (run from the repo root on the GPU box):
#   bash tools/gpu_ab.sh <tag> "<bench args>" "<env A>" "<env B>" ...
# e.g.  bash tools/gpu_ab.sh lean "--steps 20 --warmup 5" "MPCCBF_LIB=mpc-cbf_amd/build/diag/libmpccbf.so MPCCBF_LEAN=1" "MPCCBF_LIB=mpc-cbf_amd/build/diag/libmpccbf.so MPCCBF_LEAN=0"
# (the solver-tuning variables are read by the diagnostics build only: make -C mpc-cbf_amd diag)
# Each setting runs the bench line twice (interleaved A B A B); outputs gpurun_out/<tag>/<i>_<r>.json.
set -e -o pipefail
TAG=$1
ARGS=$2
shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
for r in 1 2; do
  i=0
  for e in "$@"; do
    echo "[$(date +%T)] $e $ARGS ($r)"
    env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline $ARGS > $O/${i}_$r.json 2> $O/${i}_$r.err
    i=$((i + 1))
  done
done
echo done
