#!/bin/bash
# Round-5 measurement on one box (run from the repo root): GPU tests + smoke, then the round's
# PMC passes and bench lines (tools/profile_round.sh r05 pmc / bench), then kernel traces, the
# reference instances, stamps and critical-path entries (profile_round.sh r05 prof).
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
echo "[$(date +%T)] smoke"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1
tail -1 gpurun_out/r05_smoke.log
bash tools/profile_round.sh r05 pmc
bash tools/profile_round.sh r05 bench
bash tools/profile_round.sh r05 prof
