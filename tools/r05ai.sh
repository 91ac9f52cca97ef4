# FoV: setup stamps + bench lines (operator batch pinned after the linear term)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05ai}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/setupst/libmpccbf.so timeout -k 10 120 python3 tools/setup_stamps.py 512 100 > $OUT/setup.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload fov > $OUT/bench_fov.json 2> $OUT/bench_fov.err || exit 2
timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload fov --slack > $OUT/bench_fov_slack.json 2> $OUT/bench_fov_slack.err || exit 3
