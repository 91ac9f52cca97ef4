# kernel_avg_us from the runtime's kernel events vs rocprof (config 3, share, FoV, FoV slack)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05n
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in "c3:" "share:--rank-share 8 --agents-total 8192" "fov:--workload fov" "fovs:--workload fov --slack"; do
  n=${w%%:*}; a=${w#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-trace --steps 300 --warmup 50 $a > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit 1
done
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_closed_loop.py tests/test_gpu_multirank.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" > $OUT/pytest_rc.txt
