# GPU check of the tree: GPU tests, the driver's bench command, FoV slack, smoke, then A/B timing
# (block-size variants of the separable kernel: 256 / 64 / 128 threads)
set -e -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/h_pytest.log 2>&1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/h_driver.json 2> $O/h_driver.err
timeout -k 10 300 python3 bench.py --workload fov --slack --no-cpu-baseline > $O/h_fovs.json 2> $O/h_fovs.err
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/h_smoke.log 2>&1
B="python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline"
for r in 1 2; do
  for v in 0 4 5; do timeout -k 10 120 $B --variant $v > $O/h_var${v}_$r.json 2> $O/h_var${v}_$r.err; done
  for v in 0 4 5; do timeout -k 10 120 $B --steps 20 --warmup 5 --variant $v > $O/h_drv${v}_$r.json 2> $O/h_drv${v}_$r.err; done
done
echo done
