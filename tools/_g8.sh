set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_certify.py -x -v --timeout 200 --timeout-method thread -k "capacity or certif or warm" > gpurun_out/r02g_new.log 2>&1; echo "new tests rc=$?"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r02g_pytest_gpu.log 2>&1; echo "all gpu rc=$?"
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02g_bench20.json 2> gpurun_out/r02g_bench20.err || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/r02g_bench1000.json 2> gpurun_out/r02g_bench1000.err || exit 1
