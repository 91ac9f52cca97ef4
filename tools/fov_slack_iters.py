"""Iteration distribution of the FoV controller in the bench's closed loop (slack or not)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

slack = len(sys.argv) > 1 and sys.argv[1] == "slack"
steps = 300
n = 512
kw = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if slack else {}
cfg = swarm.fov_config(20, **kw)
states_h, targets_h = swarm.heading_swarm(n)
dev = torch.device("cuda", 0)
ctx = Context(cfg)
a = torch.tensor(states_h, device=dev)
b = torch.empty_like(a)
cov = torch.tensor(np.tile([0.1, 0.0, 0.1], (n, 1)), device=dev) if slack else None
out = ctx.alloc_outputs(n)
sl = torch.empty((steps, n, 2), dtype=torch.int32, device=dev)
il = torch.empty((steps, n, 2), dtype=torch.int32, device=dev)
traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
r = ctx.run_steps(a, b, steps, targets=torch.tensor(targets_h, device=dev), knn_k=8,
                  knn_radius=cfg["fov_Rs"], x=out["x"], obj=out["obj"], status_log=sl, iters_log=il,
                  traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=20251015, cov=cov,
                  timing=True)
torch.cuda.synchronize()
st = sl.cpu().numpy()
it = il.cpu().numpy()
att = ~((st == 5) & (it == 0))
print(f"slack={slack}: iters mean {it[att].mean():.2f} p50 {np.median(it[att])} p99 {np.percentile(it[att], 99)} "
      f"max {it.max()}; optimal {np.mean(st[att] == 0):.4f}; status counts {np.bincount(st[att].ravel())}")
print("per-step max iters (first 40):", it.reshape(steps, -1).max(axis=1)[:40].tolist())
print("steps with max iters >= 30:", int(np.sum(it.reshape(steps, -1).max(axis=1) >= 30)))
print("step_ms p50 %.3f p99 %.3f max %.3f" % (np.median(r["step_ms"]), np.percentile(r["step_ms"], 99), r["step_ms"].max()))
hist = np.bincount(it[att].ravel())
print("hist:", {i: int(c) for i, c in enumerate(hist) if c})
