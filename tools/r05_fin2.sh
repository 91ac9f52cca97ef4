# round-5 final measurement, part 2: the bench lines (reading profiles/r05_pmc_summary.json)
set -e -o pipefail
bash tools/profile_round.sh r05 bench
