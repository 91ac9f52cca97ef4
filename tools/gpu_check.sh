#!/bin/bash
# GPU check of the tree (run from the repo root on the GPU box through gpurun):
#   bash tools/gpu_check.sh <tag> [tests|bench|all]
# tests: the -m gpu suite and smoke(); bench: the driver's bench command plus the bench lines of
# DESIGN §4 (config 3 at 1000 steps, 8192 agents, config 4's per-rank share, FoV, FoV slack).
# Outputs under gpurun_out/<tag>/. Every GPU step has its own time limit; the first failure ends
# the script.
set -e -o pipefail
TAG=${1:-chk}
WHAT=${2:-all}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
step() { echo "[$(date +%T)] $*"; }
B="python3 bench.py --no-cpu-baseline"
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  step pytest
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  step smoke
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  step driver; timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err
  step 1000; timeout -k 10 200 $B > $O/coll.json 2> $O/coll.err
  step 8192; timeout -k 10 200 $B --agents-per-gpu 8192 > $O/8192.json 2> $O/8192.err
  step rank-share; timeout -k 10 200 $B --rank-share 8 --agents-total 8192 > $O/share.json 2> $O/share.err
  step fov; timeout -k 10 200 $B --workload fov > $O/fov.json 2> $O/fov.err
  step fovs; timeout -k 10 200 $B --workload fov --slack > $O/fovs.json 2> $O/fovs.err
fi
step done
