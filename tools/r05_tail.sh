# the tail of profile_round.sh r05 prof (after the prof build was rebuilt)
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=r05
cd $ROOT
MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 4096 100 0 > $OUT/${TAG}_stamps_collision_das.log 2>&1
MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python3 tools/wide_stamps.py 1024 60 > $OUT/${TAG}_stamps_share_das.log 2>&1
WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/stamps/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $OUT/${TAG}_stamps_fov.log 2>&1
WORKLOAD=fov MPCCBF_LIB=$ROOT/mpc-cbf_amd/build/prof/libmpccbf.so timeout -k 10 120 python3 tools/stamp_profile.py 512 100 0 > $OUT/${TAG}_stamps_fov_das.log 2>&1
timeout -k 10 200 python3 tools/determinism_loop.py 6 1 30 > $OUT/${TAG}_determinism_fovs.log 2>&1
echo done
