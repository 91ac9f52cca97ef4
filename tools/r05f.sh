# wide kernel with the one-round-trip query: parity A/B (normal, 4096, crowded overflow), stamps,
# rocprof at the config-4 share, PMC passes
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05f
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/wide_ab.py --agents 1024 --steps 30 > $OUT/ab1024.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/wide_ab.py --agents 1024 --steps 20 --scale 0.35 > $OUT/ab1024_dense.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/wide_ab.py --agents 4096 --steps 30 > $OUT/ab4096.log 2>&1 || exit 3
MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 200 python -u tools/stamp_profile.py 1024 60 5 > $OUT/stamps1024.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_share_v5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rank-share 8 --agents-total 8192 --steps 300 --warmup 50 --variant 5 > $OUT/bench_share_v5.json 2> $OUT/bench_share_v5.err || exit 5
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-trace --steps 30 --warmup 5 --rank-share 8 --agents-total 8192 --variant 5"
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
SQB="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
SQC="SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"
i=0
for set in "$SQA" "$SQB" "$SQC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc/share_p$i -o run -- $B > $OUT/pmc_p$i.log 2>&1 || exit $((10+i))
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.json
