set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/q_pytest.log 2>&1; echo "gpu tests rc=$?"
timeout -k 10 100 python bench.py --no-cpu-baseline > gpurun_out/ab_coll.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload fov --slack --no-cpu-baseline > gpurun_out/ab_fovs.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload fov --no-cpu-baseline > gpurun_out/ab_fov.json 2>/dev/null || exit 1
timeout -k 10 300 env MPCCBF_CHECK_SLACK=1 python tools/fov_status_check.py 200 gpurun_out/fovs_status.npz > gpurun_out/fovs_status.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for w in coll fovs; do
  if [ $w = coll ]; then A=""; else A="--workload fov --slack"; fi
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_pmc/${w}_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 $A > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_pmc/${w}_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 $A > /dev/null 2>&1 || exit 1
done
