# round-5 final measurement, part 3: kernel traces, GPU tests, reference instances, stamps
set -e -o pipefail
bash tools/profile_round.sh r05 prof
