set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "slack" > gpurun_out/q_pytest_slack.log 2>&1; echo "slack tests rc=$?"
timeout -k 10 100 python bench.py --slack --steps 300 --no-cpu-baseline > gpurun_out/ab_slack_new.json 2>/dev/null || exit 1
timeout -k 10 100 env MPCCBF_LIB=mpc-cbf_amd/build/abref/libmpccbf.so python bench.py --slack --steps 300 --no-cpu-baseline > gpurun_out/ab_slack_ref.json 2>/dev/null || exit 1
