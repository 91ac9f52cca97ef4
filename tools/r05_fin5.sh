# round-5 closing check on the final tree: GPU tests, smoke, the driver's bench command, then the
# dense line / trace / reduction stamps (tools/r05_fin4.sh)
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd $ROOT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/r05_pytest_gpu.log 2>&1 || true
tail -1 $OUT/r05_pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/r05_smoke.log 2>&1
tail -1 $OUT/r05_smoke.log
timeout -k 10 300 python3 bench.py > $OUT/r05_bench_default.json 2> $OUT/r05_bench_default.err
bash tools/r05_fin4.sh
