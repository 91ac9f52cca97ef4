set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05o
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 300 python3 bench.py --rank-share 8 --agents-total 8192 --no-cpu-baseline > $OUT/bench_share.json 2> $OUT/bench_share.err || exit 2
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit 3
