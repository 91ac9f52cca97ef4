#!/bin/bash
# Root cause of the FoV-slack step-0 nondeterminism (round 3): LDS poison runs of the closed loops
# in tools/lds_poison_check.py with static LDS filled with 1e300 (poison_a) and with NaN, once for
# the fixed tree (poison_c) and once for a build of the previous das_wave.hpp (poison_c_old, built
# outside the repo from `git show <rev>:mpc-cbf_amd/csrc/kernels/das_wave.hpp`). Expected: a == c,
# a != c_old in the FoV-slack solver-step counts only.
#   bash tools/poison_rootcause.sh <tag>
set -e -o pipefail
TAG=${1:-poison}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
B=$ROOT/mpc-cbf_amd/build
for v in a c c_old; do
  echo "[$(date +%T)] run $v"
  MPCCBF_LIB=$B/poison_$v/libmpccbf.so timeout -k 10 240 python3 -u tools/lds_poison_check.py run $O/$v.npz > $O/run_$v.log 2>&1
done
python3 tools/lds_poison_check.py cmp $O/a.npz $O/c.npz > $O/cmp_a_c.log 2>&1 || true
python3 tools/lds_poison_check.py cmp $O/a.npz $O/c_old.npz > $O/cmp_a_c_old.log 2>&1 || true
cat $O/cmp_a_c.log $O/cmp_a_c_old.log
