"""Writes the golden MPC-CBF QPs (tests/golden/golden_qps.npz) as a flat binary for
tools/dense_pack_bench.cpp: count, then per QP n, m, H (n x n), c, A (m x n), lo, hi (float64)."""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = np.load(os.path.join(REPO, "tests", "golden", "golden_qps.npz"))
count = int(g["count"])
with open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/golden.bin", "wb") as f:
    f.write(struct.pack("i", count))
    for i in range(count):
        H, c, A, lo, hi = (np.ascontiguousarray(g[f"c{i}_{k}"], dtype=np.float64) for k in ("H", "c", "A", "lo", "hi"))
        f.write(struct.pack("ii", c.shape[0], A.shape[0]))
        for a in (H, c, A, lo, hi):
            f.write(a.tobytes())
