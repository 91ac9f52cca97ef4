#!/bin/bash
# Round measurement set, run from the repo root on the GPU box (outputs under gpurun_out/<tag>_*):
#   bench lines — the driver's command (config 3, 20 steps), config 3 at 1000 steps (+ CPU
#   baseline), config 4's 8192 agents on one GPU, config 5 (FoV) and its slack mode;
#   rocprofv3 --kernel-trace --stats of the same commands; PMC passes (one counter group per run,
#   never combined with traces): HBM bytes (FETCH_SIZE, WRITE_SIZE), SQ issue / wait counters,
#   FP64 instruction mix, and the FoV kernels' FP64 MFMA counters.
# Order: PMC passes first (their summary goes to profiles/<tag>_pmc_summary.json, which the bench
# lines read), then the bench lines and kernel traces, then the GPU tests and the stamp profile.
# Usage: bash tools/profile_round.sh <tag> [nopmc|pmc|bench|prof]   (pmc: the PMC passes only;
# nopmc: the rest; bench: the bench lines only; prof: the kernel traces, GPU tests and stamps only)
set -e -o pipefail
TAG=${1:-rNN}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $ROOT/bench.py"
step() { echo "[$(date +%T)] $*"; }
[ "$2" = "nopmc" ] || [ "$2" = "bench" ] || [ "$2" = "prof" ] || {
pmc() {  # dir, bench args..., -- counters
  local d=$1; shift
  local args=()
  while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
  step pmc $d "$@"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/${TAG}_pmc/$d -o run \
    -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 "${args[@]}" > $OUT/${TAG}_pmc_$d.log 2>&1
}
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
SQB="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
SQM="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
pmc collision_fetch -- FETCH_SIZE
pmc collision_write -- WRITE_SIZE
pmc collision_sqa -- $SQA
pmc collision_sqb -- $SQB
pmc fov_fetch --workload fov -- FETCH_SIZE
pmc fov_write --workload fov -- WRITE_SIZE
pmc fov_sqa --workload fov -- $SQA
pmc fov_mfma --workload fov -- $SQM
pmc fovs_fetch --workload fov --slack -- FETCH_SIZE
pmc fovs_write --workload fov --slack -- WRITE_SIZE
pmc fovs_sqa --workload fov --slack -- $SQA
pmc fovs_mfma --workload fov --slack -- $SQM
# the 8-rank share (config 4's per-rank launch: the one-agent-per-wave kernel) under the collision
# table (its kernel has its own name there)
pmc collision_wfetch --rank-share 8 --agents-total 8192 -- FETCH_SIZE
pmc collision_wwrite --rank-share 8 --agents-total 8192 -- WRITE_SIZE
pmc collision_wsqa --rank-share 8 --agents-total 8192 -- $SQA
pmc collision_wsqb --rank-share 8 --agents-total 8192 -- $SQB
pmc collision_cache -- SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES
# the bench lines below read their traffic / VALU figures from this round's summary
python3 $ROOT/tools/pmc_summary.py $OUT/${TAG}_pmc > $ROOT/profiles/${TAG}_pmc_summary.json
cp $ROOT/profiles/${TAG}_pmc_summary.json $OUT/${TAG}_pmc_summary.json
}
[ "$2" = "pmc" ] && { step done; exit 0; }
[ "$2" = "prof" ] || {
step bench driver; timeout -k 10 200 $B --steps 20 --warmup 5 > $OUT/${TAG}_bench_driver.json 2> $OUT/${TAG}_bench_driver.err
step bench 1000; timeout -k 10 300 $B > $OUT/${TAG}_bench_collision.json 2> $OUT/${TAG}_bench_collision.err
step bench 8192; timeout -k 10 300 $B --agents-per-gpu 8192 --no-cpu-baseline > $OUT/${TAG}_bench_8192.json 2> $OUT/${TAG}_bench_8192.err
step bench share; timeout -k 10 300 $B --rank-share 8 --agents-total 8192 --no-cpu-baseline > $OUT/${TAG}_bench_share.json 2> $OUT/${TAG}_bench_share.err
step bench crowded; timeout -k 10 300 $B --crowded --steps 300 --warmup 20 > $OUT/${TAG}_bench_crowded.json 2> $OUT/${TAG}_bench_crowded.err
step bench all256; timeout -k 10 300 $B --neighbours all --agents-per-gpu 256 --crowded --steps 200 --warmup 20 > $OUT/${TAG}_bench_all256.json 2> $OUT/${TAG}_bench_all256.err
step bench all256 slack; timeout -k 10 300 $B --neighbours all --agents-per-gpu 256 --crowded --slack --steps 200 --warmup 20 > $OUT/${TAG}_bench_all256_slack.json 2> $OUT/${TAG}_bench_all256_slack.err
step bench fov; timeout -k 10 300 $B --workload fov > $OUT/${TAG}_bench_fov.json 2> $OUT/${TAG}_bench_fov.err
step bench fov slack; timeout -k 10 300 $B --workload fov --slack > $OUT/${TAG}_bench_fov_slack.json 2> $OUT/${TAG}_bench_fov_slack.err
step bench dense; timeout -k 10 300 $B --workload dense --steps 10 --warmup 2 > $OUT/${TAG}_bench_dense.json 2> $OUT/${TAG}_bench_dense.err
}
[ "$2" = "bench" ] && { step done; exit 0; }
prof() {  # name, bench args
  step prof $1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$1 -o run \
    -- python3 $ROOT/bench.py --no-cpu-baseline ${@:2} > $OUT/${TAG}_prof_$1.json 2> $OUT/${TAG}_prof_$1.err
}
prof driver --steps 20 --warmup 5
prof collision
prof 8192 --agents-per-gpu 8192
prof share --rank-share 8 --agents-total 8192
prof crowded --crowded --steps 300 --warmup 20
prof all256 --neighbours all --agents-per-gpu 256 --crowded --steps 200 --warmup 20 --no-trace
prof fov --workload fov
prof fov_slack --workload fov --slack
prof dense --workload dense --steps 10 --warmup 2
step pytest; (cd $ROOT && timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_gpu.log 2>&1) || true
step reference instances; (cd $ROOT && timeout -k 10 400 python3 -u tools/reference_instances.py --out $OUT/${TAG}_reference_instances.json > $OUT/${TAG}_reference_instances.log 2>&1)
step critical path; rm -f $OUT/${TAG}_critical_path.json
(cd $ROOT && CP_JSON=$OUT/${TAG}_critical_path.json MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 1024 60 0 > $OUT/${TAG}_stamps_share.log 2>&1)
step fovs status; (cd $ROOT && MPCCBF_CHECK_SLACK=1 timeout -k 10 300 python3 $ROOT/tools/fov_status_check.py 1000 $OUT/${TAG}_fovs_status.npz > $OUT/${TAG}_fovs_status.log 2>&1)
step stamps; (cd $ROOT && CP_JSON=$OUT/${TAG}_critical_path.json MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > $OUT/${TAG}_stamps_collision.log 2>&1)
step stamps pdip; (cd $ROOT && MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > $OUT/${TAG}_stamps_collision_das.log 2>&1)
step stamps fov; (cd $ROOT && WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $OUT/${TAG}_stamps_fov.log 2>&1)
step stamps fov das; (cd $ROOT && WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $OUT/${TAG}_stamps_fov_das.log 2>&1)
step determinism; (cd $ROOT && timeout -k 10 200 python3 tools/determinism_loop.py 6 1 30 > $OUT/${TAG}_determinism_fovs.log 2>&1)
echo done
