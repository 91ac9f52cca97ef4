# dense bench line three times + kernel trace (variance of the host-bound batch line)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05af}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do timeout -k 10 200 python3 bench.py --workload dense --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_dense_$i.json 2> $OUT/bench_dense_$i.err || exit $i; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_dense -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload dense --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_dense_prof.json 2> $OUT/bench_dense_prof.err || exit 4
