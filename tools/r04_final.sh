#!/bin/bash
# Round-4 final measurement on one box (run from the repo root): GPU tests + smoke, then the round's
# PMC passes and bench lines (tools/profile_round.sh r04 pmc / bench), then kernel traces, the FoV
# slack status check and the stamps (profile_round.sh r04 prof).
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
echo "[$(date +%T)] pytest"
timeout -k 10 420 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r04_pytest_gpu.log 2>&1
tail -2 gpurun_out/r04_pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
tail -1 gpurun_out/r04_smoke.log
bash tools/profile_round.sh r04 pmc
bash tools/profile_round.sh r04 bench
bash tools/profile_round.sh r04 prof
