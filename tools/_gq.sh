set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/q_pytest.log 2>&1; echo "gpu tests rc=$?"
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/q_bench20.json 2> gpurun_out/q_bench20.err || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/q_bench1000.json 2> gpurun_out/q_bench1000.err || exit 1
timeout -k 10 200 python bench.py --workload fov --no-cpu-baseline > gpurun_out/q_fov.json 2> gpurun_out/q_fov.err || exit 1
timeout -k 10 100 env MPCCBF_LIB=mpc-cbf_amd/build/prof/libmpccbf.so python tools/stamp_profile.py 4096 100 0 > gpurun_out/q_stamp.log 2>&1 || exit 1
