"""Summary of tools/gpu_ab.sh outputs: per directory and setting, value and kernel mean / max of
each repetition.   python tools/ab_summary.py <dir>..."""
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    print(os.path.basename(d))
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        try:
            j = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            print(f"  {os.path.basename(f)}: no result")
            continue
        r = j.get("roofline", {})
        print(f"  {os.path.basename(f)}: value {j['value']:.4g} ms/step {j['ms_per_step']:.4f} "
              f"kernel {r.get('kernel_avg_us', float('nan')):.2f} / {r.get('kernel_max_us', float('nan')):.2f} us "
              f"steps/QP {j.get('newton_steps_per_qp', {}).get('mean', float('nan')):.4f}")
