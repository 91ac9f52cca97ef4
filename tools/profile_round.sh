#!/bin/bash
# Round measurement set, run from the repo root on the GPU box:
#   bench lines (collision = headline config 3, FoV = config 5), rocprofv3 kernel-trace stats of
#   the same commands, and the PMC traffic passes of the collision bench.
# Usage: bash tools/profile_round.sh <tag>   (outputs under gpurun_out/<tag>_*)
set -e -o pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $ROOT/bench.py > $OUT/${TAG}_bench_collision.json 2> $OUT/${TAG}_bench_collision.err
timeout -k 10 300 python3 $ROOT/bench.py --workload fov > $OUT/${TAG}_bench_fov.json 2> $OUT/${TAG}_bench_fov.err
timeout -k 10 300 python3 $ROOT/bench.py --workload fov --slack > $OUT/${TAG}_bench_fov_slack.json 2> $OUT/${TAG}_bench_fov_slack.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_collision -o run \
    -- python3 $ROOT/bench.py --no-cpu-baseline > $OUT/${TAG}_prof_collision.json 2> $OUT/${TAG}_prof_collision.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_fov -o run \
    -- python3 $ROOT/bench.py --workload fov --no-cpu-baseline > $OUT/${TAG}_prof_fov.json 2> $OUT/${TAG}_prof_fov.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_fov_slack -o run \
    -- python3 $ROOT/bench.py --workload fov --slack --no-cpu-baseline > $OUT/${TAG}_prof_fov_slack.json 2> $OUT/${TAG}_prof_fov_slack.err
ARGS="$ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ARGS > $OUT/pmc_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ARGS > $OUT/pmc_write.log 2>&1
FARGS="$ROOT/bench.py --workload fov --no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fov_fetch -o run -- python3 $FARGS > $OUT/pmc_fov_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_fov_write -o run -- python3 $FARGS > $OUT/pmc_fov_write.log 2>&1
SARGS="$FARGS --slack"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fovs_fetch -o run -- python3 $SARGS > $OUT/pmc_fovs_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_fovs_write -o run -- python3 $SARGS > $OUT/pmc_fovs_write.log 2>&1
echo done
