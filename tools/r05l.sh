# wide kernel: parity A/B vs the 16-lane kernel, share bench under rocprof, stamps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05l
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/wide_ab.py --agents 1024 --steps 30 > $OUT/ab1024.log 2>&1 || exit 1
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 1024 60 0 > $OUT/stamps1024.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_share -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 > $OUT/bench_share.json 2> $OUT/bench_share.err || exit 3
