# dense: GPU tests (asymmetric / index-edge case), one-QP reduction phase stamps
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAGO:-r05aa}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_dense_qp.py tests/test_qpcpp_adapter.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_dense.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/pytest_rc.txt; [ $rc -le 1 ] || exit 1
MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/prof/libmpccbf.so MPCCBF_DENSE_STAMPS=1 timeout -k 10 120 python3 tools/dense_stamps.py 20 1 > $OUT/stamps1.log 2> $OUT/stamps1.err || exit 2
MPCCBF_LIB=$GRAFT_REPO_ROOT/mpc-cbf_amd/build/prof/libmpccbf.so MPCCBF_DENSE_STAMPS=1 timeout -k 10 120 python3 tools/dense_stamps.py 10 1024 > $OUT/stamps1024.log 2> $OUT/stamps1024.err || exit 3
