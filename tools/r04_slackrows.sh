#!/bin/bash
# Validation of the slack capacity fallback with its rows in LDS (run from the repo root): the slack
# GPU tests, the all-neighbour slack stress line over 1000 closed-loop steps (UNKNOWN must stay 0),
# and its timing against build/base (previous commit), interleaved.
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r04sr
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -k "slack or status_parity or certify" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py --neighbours all --crowded --slack --agents-per-gpu 256 --steps 1000 --warmup 20 --no-cpu-baseline --no-trace > $O/all256s_1000.json 2> $O/all256s_1000.err
python3 -c "import json; j=json.loads(open('$O/all256s_1000.json').read().strip().splitlines()[-1]); print(j['status_hist'], j['roofline']['kernel_avg_us'])"
bash tools/gpu_ab.sh r04sr/ab "--neighbours all --crowded --slack --agents-per-gpu 256 --steps 200 --warmup 20 --no-trace" "MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/base/libmpccbf.so" "MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
python3 tools/ab_summary.py $O/ab
