set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "fov" > gpurun_out/q_pytest_fov.log 2>&1; echo "fov tests rc=$?"
timeout -k 10 200 python bench.py --workload fov --slack --no-cpu-baseline > gpurun_out/ab_fovs.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload fov --no-cpu-baseline > gpurun_out/ab_fov.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_pmc/fovs_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 --workload fov --slack > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_pmc/fovs_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 --workload fov --slack > /dev/null 2>&1 || exit 1
