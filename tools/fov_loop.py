"""FoV closed loop on the GPU: per-step status mix and kernel time (config 5 workload)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 60
SCALE = float(sys.argv[3]) if len(sys.argv) > 3 else 0.7
cfg = swarm.fov_config(20)
states_h, targets_h = swarm.heading_swarm(N)
states_h[:, :2] *= SCALE
dev = torch.device("cuda", 0)
ctx = Context(cfg)
tg = torch.tensor(targets_h, device=dev)
a = torch.tensor(states_h, device=dev)
b = torch.empty_like(a)
out = ctx.alloc_outputs(N)
logs = torch.empty((STEPS, N, 2), dtype=torch.int32, device=dev)
itl = torch.empty((STEPS, N, 2), dtype=torch.int32, device=dev)
r = ctx.run_steps(a, b, STEPS, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], x=out["x"], obj=out["obj"],
                  status_log=logs, iters_log=itl, timing=True)
s = logs.cpu().numpy()
it = itl.cpu().numpy()
for k in list(range(0, STEPS, max(1, STEPS // 12))):
    att = ~((s[k] == 5) & (it[k] == 0))
    print(f"step {k:3d}: {r['solve_ms'][k] * 1e3:8.1f} us  optimal {np.sum(s[k] == 0):5d}/{att.sum():5d} "
          f"infeasible {np.sum(s[k] == 3):5d} error {np.sum(s[k] == 4):4d} iters mean {it[k][s[k] == 0].mean():.1f} max {it[k].max()}")
