# round-5 bench lines (after the kernel-timing source change) and the reference instances
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash tools/profile_round.sh r05 bench
timeout -k 10 400 python3 -u tools/reference_instances.py --out gpurun_out/r05_reference_instances.json > gpurun_out/r05_reference_instances.log 2>&1
echo done
