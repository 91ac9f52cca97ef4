set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05h
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/wide_ab.py --agents 1024 --steps 30 > $OUT/ab1024.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/wide_ab.py --agents 4096 --steps 30 > $OUT/ab4096.log 2>&1 || exit 3
MPCCBF_LIB=mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 200 python -u tools/wide_stamps.py 1024 60 > $OUT/wide_stamps.log 2>&1 || exit 4
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 1024 60 5 > $OUT/stamps1024.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_share_v5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 --variant 5 > $OUT/bench_share_v5.json 2> $OUT/bench_share_v5.err || exit 6
