"""Per-kernel statistics from a rocprofv3 SQLite database (run_results.db): calls, mean / min /
max duration in microseconds, as rocprofv3 --stats would print them.

usage: python tools/rocpd_stats.py path/to/run_results.db"""
import sqlite3
import sys

import numpy as np


def stats(path):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = c.execute(f"select s.display_name, d.start, d.end from {disp} d join {sym} s on d.kernel_id = s.id").fetchall()
    by = {}
    for name, a, b in rows:
        by.setdefault(name, []).append((b - a) / 1e3)
    out = []
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v = np.array(v)
        out.append((name, len(v), v.mean(), np.median(v), v.min(), v.max()))
    return out


if __name__ == "__main__":
    for name, n, mean, med, mn, mx in stats(sys.argv[1]):
        print(f"{n:6d} mean {mean:8.2f} med {med:8.2f} min {mn:8.2f} max {mx:8.2f} us  {name[:110]}")
