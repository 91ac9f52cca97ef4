# wide kernel with LDS-staged operators: rocprof at the config-4 share (variants 5 wide, 4 sep16),
# stamps, and the wide-vs-sep16 A/B at 1024
set -o pipefail
mkdir -p gpurun_out/r05d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 5 4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05d/prof_share_v$v -o run -- python3 bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 --variant $v > gpurun_out/r05d/bench_share_v$v.json 2> gpurun_out/r05d/bench_share_v$v.err || exit 1
done
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 1024 60 5 > gpurun_out/r05d/stamps1024.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/wide_ab.py --agents 1024 --steps 30 > gpurun_out/r05d/ab1024.log 2>&1 || exit 3
