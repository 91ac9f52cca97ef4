# round-5 final measurement, part 1: smoke, then the PMC passes (profiles/r05_pmc_summary.json)
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1
tail -1 gpurun_out/r05_smoke.log
bash tools/profile_round.sh r05 pmc
