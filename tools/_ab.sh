set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/q_pytest.log 2>&1; echo "gpu tests rc=$?"
timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/ab_coll.json 2>/dev/null || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/ab_coll20.json 2>/dev/null || exit 1
timeout -k 10 100 python bench.py --no-cpu-baseline --agents-per-gpu 8192 > gpurun_out/ab_8192.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload fov --no-cpu-baseline > gpurun_out/ab_fov.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload fov --slack --no-cpu-baseline > gpurun_out/ab_fovs.json 2>/dev/null || exit 1
MPCCBF_LIB=mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python tools/stamp_profile.py 4096 100 0 > gpurun_out/ab_stamps.log 2>&1 || exit 1
