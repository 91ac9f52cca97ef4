"""Launch-to-launch structure of a rocprofv3 --kernel-trace CSV: per kernel name, the duration
(mean / p50 / max) and the idle gap from the previous kernel's end to its start on the same
queue, over the consecutive launches of the dominant kernel (what the per-step HIP-event
figures include beyond the kernel itself).

    python tools/kernel_gaps.py <kernel_trace.csv> [name_substring]
"""
import csv
import sys

import numpy as np


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("empty trace")
        return
    keys = rows[0].keys()
    kn = next(k for k in keys if k.lower() in ("kernel_name", "kernelname", "name"))
    ks = next(k for k in keys if "start" in k.lower() and "timestamp" in k.lower())
    ke = next(k for k in keys if "end" in k.lower() and "timestamp" in k.lower())
    ev = sorted(((int(r[ks]), int(r[ke]), r[kn]) for r in rows), key=lambda t: t[0])
    names = {}
    for i, (s, e, n) in enumerate(ev):
        if sub and sub not in n:
            continue
        gap = s - ev[i - 1][1] if i > 0 else None
        d = names.setdefault(n.split("(")[0][:90], {"dur": [], "gap": []})
        d["dur"].append(e - s)
        if gap is not None:
            d["gap"].append(gap)
    for n, d in sorted(names.items(), key=lambda kv: -len(kv[1]["dur"])):
        du = np.array(d["dur"]) / 1e3
        g = np.array(d["gap"]) / 1e3 if d["gap"] else np.zeros(1)
        print(f"{n}: {len(du)} launches, duration mean {du.mean():.1f} p50 {np.median(du):.1f} max {du.max():.1f} us; "
              f"gap before it mean {g.mean():.2f} p50 {np.median(g):.2f} p90 {np.percentile(g, 90):.2f} us")


if __name__ == "__main__":
    main()
