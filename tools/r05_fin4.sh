# round-5 final measurement, part 4: the dense line and its kernel trace after the reduction changes,
# the one-QP reduction phase stamps
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $ROOT/bench.py --workload dense --steps 10 --warmup 2 > $OUT/r05_bench_dense.json 2> $OUT/r05_bench_dense.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_prof_dense -o run \
  -- python3 $ROOT/bench.py --no-cpu-baseline --workload dense --steps 10 --warmup 2 > $OUT/r05_prof_dense.json 2> $OUT/r05_prof_dense.err
cd $ROOT
MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/prof/libmpccbf.so MPCCBF_DENSE_STAMPS=1 timeout -k 10 120 python3 tools/dense_stamps.py 20 1 > $OUT/r05_dense_stamps.log 2>&1
