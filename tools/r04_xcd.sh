#!/bin/bash
# A/B of the XCD-aware block order (run from the repo root): bench lines of build/base (previous
# commit) against the current build and build/rel_REGAI, interleaved; HBM fetch / write bytes of
# both (one PMC counter group per run); the phase stamps of both.   bash tools/r04_xcd.sh <tag>
set -e -o pipefail
TAG=${1:-r04xcd}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
A="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/base/libmpccbf.so"
B="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/libmpccbf.so"
C="MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/rel_REGAI/libmpccbf.so"
bash tools/gpu_ab.sh $TAG/coll "--steps 300 --warmup 20" "$A" "$B" "$C"
bash tools/gpu_ab.sh $TAG/fov "--workload fov --steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh $TAG/fovs "--workload fov --slack --steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh $TAG/share "--rank-share 8 --agents-total 8192 --steps 300 --warmup 20" "$A" "$B"
bash tools/gpu_ab.sh $TAG/n8192 "--agents-per-gpu 8192 --steps 200 --warmup 20" "$A" "$B"
python3 tools/ab_summary.py $O/coll $O/fov $O/fovs $O/share $O/n8192
cd /tmp && export TMPDIR=/tmp
for v in base ""; do
  for c in FETCH_SIZE WRITE_SIZE; do
    for w in "" "--workload fov"; do
      n=${v:-new}_${c}_${w:+fov}
      MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$n -o run \
        -- python3 $ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 $w > $O/pmc_$n.log 2>&1
    done
  done
done
cd $ROOT
for v in base_stamps stamps; do
  MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/$v/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > $O/stamps_coll_$v.log 2>&1
done
for f in $O/stamps_*.log; do echo "== $f"; sed -n '2,10p' $f; done
