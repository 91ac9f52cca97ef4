#!/bin/bash
# PMC passes for the bench workload (one counter group per pass; --pmc never combined with
# runtime/sys traces). Output under gpurun_out/pmc_*; run from the repo root on the GPU box.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="$ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/pmc_fetch -o run -- python3 $ARGS > $ROOT/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/pmc_write -o run -- python3 $ARGS > $ROOT/gpurun_out/pmc_write.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $ROOT/gpurun_out/pmc_sq -o run -- python3 $ARGS > $ROOT/gpurun_out/pmc_sq.log 2>&1
