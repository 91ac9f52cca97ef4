set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05ac
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/prof/libmpccbf.so MPCCBF_DENSE_STAMPS=1 timeout -k 10 120 python3 tools/dense_stamps.py 20 1 > $OUT/stamps1.log 2> $OUT/stamps1.err || exit 2
