# permlane cross-row reductions: full GPU tests, then dense / collision / share / fov bench lines
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05s}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 200 $B --workload dense --steps 20 --warmup 3 > $OUT/bench_dense.json 2> $OUT/bench_dense.err || exit 2
timeout -k 10 200 $B > $OUT/bench_collision.json 2> $OUT/bench_collision.err || exit 3
timeout -k 10 200 $B --rank-share 8 --agents-total 8192 > $OUT/bench_share.json 2> $OUT/bench_share.err || exit 4
timeout -k 10 200 $B --workload fov > $OUT/bench_fov.json 2> $OUT/bench_fov.err || exit 5
timeout -k 10 200 $B --workload fov --slack > $OUT/bench_fov_slack.json 2> $OUT/bench_fov_slack.err || exit 6
