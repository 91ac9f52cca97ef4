"""Per-Newton-step traces of the first PDIP solve and of phase 1 for every agent over a range of
closed-loop steps (trace build), saved for offline analysis of early-exit rules.

    MPCCBF_LIB=mpc-cbf_amd/build/trace/libmpccbf.so python tools/pdip_trace_stats.py [first] [last] [out]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

FIRST = int(sys.argv[1]) if len(sys.argv) > 1 else 12
LAST = int(sys.argv[2]) if len(sys.argv) > 2 else 30
OUT = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/trace_stats.npz"
N = 4096
cfg = swarm.config(15)
states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
ctx = Context(cfg)
tg = torch.tensor(targets_h, device=dev)
out = ctx.alloc_outputs(N)
traj_t = torch.full((N,), -1.0, dtype=torch.float64, device=dev)
a = torch.tensor(states_h, device=dev)
b = torch.empty_like(a)
radius = 3.0 * cfg["d_min"]
common = dict(targets=tg, knn_k=8, knn_radius=radius, x=out["x"], obj=out["obj"], traj_t=traj_t,
              pos_std=0.001, vel_std=0.01, noise_seed=20251015)
cur, alt = a, b
if FIRST > 0:
    r = ctx.run_steps(cur, alt, FIRST, status=out["status"], iters=out["iters"], **common)
    if r["final"] is not cur:
        cur, alt = alt, cur
stamps = torch.zeros(N * 8 + N * 2 * 256, dtype=torch.int64, device=dev)
ST, IT, TR = [], [], []
for s in range(FIRST, LAST):
    stamps.zero_()
    ctx.impc_solve(cur, targets=tg, knn_k=8, knn_radius=radius, x=out["x"], status=out["status"],
                   obj=out["obj"], iters=out["iters"], stamps=stamps)
    torch.cuda.synchronize()
    ST.append(out["status"].cpu().numpy().copy())
    IT.append(out["iters"].cpu().numpy().copy())
    TR.append(stamps.cpu().numpy()[N * 8:].view(np.float64).reshape(N, 2, 64, 4).astype(np.float32))
    r = ctx.run_steps(cur, alt, 1, status=out["status"], iters=out["iters"], step_index=s, **common)
    if r["final"] is not cur:
        cur, alt = alt, cur
np.savez_compressed(OUT, status=np.array(ST), iters=np.array(IT), trace=np.array(TR))
print("saved", OUT)
