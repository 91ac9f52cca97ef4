set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02f_pytest_gpu.log 2>&1; echo "gpu tests rc=$?"
timeout -k 10 100 python bench.py --steps 20 --warmup 5 > gpurun_out/r02f_bench20.json 2> gpurun_out/r02f_bench20.err || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/r02f_bench1000.json 2> gpurun_out/r02f_bench1000.err || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline --workload fov > gpurun_out/r02f_fov.json 2> gpurun_out/r02f_fov.err || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
