#!/bin/bash
# A/B of the IMPC iteration-1 active-set warm start threshold (mpccbf_options.das_warm_steps) on the
# driver's bench command and the 1000-step line; interleaved, two repetitions each.
O=gpurun_out/${1:-ab_daswarm}; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-trace"
for r in 1 2; do
  for w in 0 2 1 -1; do
    timeout -k 10 200 $B --steps 20 --warmup 5 --das-warm $w > $O/drv_w${w}_r$r.json 2>/dev/null || exit 1
    timeout -k 10 200 $B --das-warm $w > $O/k1000_w${w}_r$r.json 2>/dev/null || exit 1
  done
done
python3 - <<'PY' $O
import json, glob, sys, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), "%.4g" % d["value"], "kern %.2f max %.2f" % (d["roofline"]["kernel_avg_us"], d["roofline"]["kernel_max_us"]))
PY
