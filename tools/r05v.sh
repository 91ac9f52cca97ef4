# GPU tests + bench lines (tools/r05s.sh), then the FoV stamp profiles (phases, das steps)
set -o pipefail
T=${TAGO:-r05v}
TAGO=$T bash tools/r05s.sh || exit $?
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
cd $GRAFT_REPO_ROOT
WORKLOAD=fov MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $OUT/stamps_fov.log 2>&1 || exit 7
WORKLOAD=fov MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $OUT/stamps_fov_das.log 2>&1 || exit 8
