set -o pipefail
mkdir -p gpurun_out/r05b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b/prof_share_v$v -o run -- python3 bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 --variant $v > gpurun_out/r05b/bench_share_v$v.json 2> gpurun_out/r05b/bench_share_v$v.err || exit 1
done
timeout -k 10 200 python -u tools/wide_ab.py --agents 1024 --steps 30 --time > gpurun_out/r05b/ab1024.log 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_reference_instances.py > gpurun_out/r05b/ref_inst_test.log 2>&1
echo test rc $?
