# A/B of the collision layouts at config 4's rank share (1024 agents) and config 3 (4096):
# rocprof kernel stats + bench lines per variant (0 auto, 4 sep16, 5 wide+fallback launch, 6 wide inline)
set -o pipefail
mkdir -p gpurun_out/r05c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 6 5 4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05c/prof_share_v$v -o run -- python3 bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 --variant $v > gpurun_out/r05c/bench_share_v$v.json 2> gpurun_out/r05c/bench_share_v$v.err || exit 1
done
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 1024 60 6 > gpurun_out/r05c/stamps1024.log 2>&1 || exit 2
