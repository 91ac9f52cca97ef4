"""Phase split of the dense reduction's latency for one QP (the profiling build's shader-clock
stamps of QP 0): run with MPCCBF_LIB=mpc-cbf_amd/build/prof/libmpccbf.so MPCCBF_DENSE_STAMPS=1;
the library prints one 'dense_stamps' line per call to stderr (cycles per phase: staging, parse,
E^T image, QR, particular solution, Z formation, Hs / P / q, Cholesky, rows, outputs).

    python tools/dense_stamps.py [calls] [batch] 2> stamps.txt"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
import mpccbf  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "golden_qps.npz"))
qp = dict(H=g["c0_H"], c=g["c0_c"], A=g["c0_A"], lo=g["c0_lo"], hi=g["c0_hi"])
ts = []
for _ in range(calls):
    t0 = time.perf_counter()
    st, xs, obj = mpccbf.dense_qp_solve_batch([qp] * batch)
    ts.append(time.perf_counter() - t0)
print(f"batch {batch}: call median {1e3 * np.median(ts[2:]):.3f} ms, status {st[0]}")
