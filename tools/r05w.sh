# launch clock against the phase stamps (wide share, 16-lane config 3)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05w}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/stamps/libmpccbf.so
MPCCBF_LIB=$L timeout -k 10 120 python3 tools/clock_vs_stamps.py 1024 20 > $OUT/cvs_1024.log 2>&1 || exit 1
MPCCBF_LIB=$L timeout -k 10 120 python3 tools/clock_vs_stamps.py 4096 20 > $OUT/cvs_4096.log 2>&1 || exit 2
