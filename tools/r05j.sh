# GPU tests, the launch clock against rocprof (default config, 8-rank share), stamps entries
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05j
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 1
rm -f $OUT/critical_path.json
CP_JSON=$OUT/critical_path.json MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 1024 60 0 > $OUT/stamps1024.log 2>&1 || exit 2
CP_JSON=$OUT/critical_path.json MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 4096 100 0 > $OUT/stamps4096.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 4
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_share -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 > $OUT/bench_share.json 2> $OUT/bench_share.err || exit 5
