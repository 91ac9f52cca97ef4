"""Per-Newton-step trace (primal residual, mu, step length, dual residual) of the first PDIP solve
of each IMPC iteration, for the agents whose solve took longest, at a chosen closed-loop step.
Needs the trace build (make -C mpc-cbf_amd trace).

    MPCCBF_LIB=mpc-cbf_amd/build/trace/libmpccbf.so python tools/pdip_trace.py [step] [N]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

STEP = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
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
r = ctx.run_steps(a, b, STEP, status=out["status"], iters=out["iters"], **common)
cur = r["final"]
stamps = torch.zeros(N * 8 + N * 2 * 256, dtype=torch.int64, device=dev)
ctx.impc_solve(cur, targets=tg, knn_k=8, knn_radius=radius, x=out["x"], status=out["status"],
               obj=out["obj"], iters=out["iters"], stamps=stamps)
torch.cuda.synchronize()
st = out["status"].cpu().numpy()
it = out["iters"].cpu().numpy()
tr = stamps.cpu().numpy()[N * 8:].view(np.float64).reshape(N, 2, 64, 4)
tot = it % 100 + (it // 100) % 100 + it // 10000
order = np.argsort(tot.max(axis=1))[::-1]
for ai in order[:8]:
    for j in (0, 1):
        w, c, p1 = it[ai, j] % 100, (it[ai, j] // 100) % 100, it[ai, j] // 10000
        n = w if j == 1 and w else c
        print(f"agent {ai} iteration {j}: status {st[ai, j]} warm {w} cold {c} phase1 {p1}")
        for k in range(min(n, 64)):
            rp, mu, al, rd = tr[ai, j, k]
            print(f"   {k:2d} rp {rp:9.2e} mu {mu:9.2e} alpha {al:7.4f} rd {rd:9.2e}")
