# A/B of the FoV slack pattern limit (4: default build; 8 / 16: build/pat*): bench lines, 2 rounds.
# Build the alternatives first (CPU side), e.g.
#   make -C mpc-cbf_amd BUILD=build/pat8 HIPFLAGS="<default HIPFLAGS> -DMPCCBF_SLK_PATTERNS=8" build/pat8/libmpccbf.so
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
B="python3 bench.py --workload fov --slack --no-cpu-baseline --steps 500 --warmup 20"
for r in 1 2; do
  timeout -k 10 120 $B > $O/p4_$r.json 2> $O/p4_$r.err
  for n in 8 16; do MPCCBF_LIB=$PWD/mpc-cbf_amd/build/pat$n/libmpccbf.so timeout -k 10 120 $B > $O/p${n}_$r.json 2> $O/p${n}_$r.err; done
done
echo done
