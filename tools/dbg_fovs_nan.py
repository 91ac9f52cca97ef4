"""FoV slack mode: one IMPC launch on the status-check swarm; report agents whose outputs are not
finite (status, iters, objective, x)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9)
states, targets = swarm.heading_swarm(512)
dev = torch.device("cuda", 0)
TWO = os.environ.get("TWO", "0") == "1"  # a PDIP-only context solving the same states first
if TWO:
    os.environ["MPCCBF_DUAL_AS"] = "0"
    ctx_p = Context(cfg)
    del os.environ["MPCCBF_DUAL_AS"]
    op = ctx_p.alloc_outputs(512)
ctx = Context(cfg)
st = torch.tensor(states, device=dev)
tg = torch.tensor(targets, device=dev)
cov = torch.tensor(np.tile([0.1, 0.0, 0.1], (512, 1)), dtype=torch.float64, device=dev)
o = ctx.alloc_outputs(512)
traj_t = torch.full((512,), -1.0, dtype=torch.float64, device=dev)
o["x"].fill_(float("nan"))
for step in range(4):
    if TWO:
        ctx_p.impc_solve(st, x=op["x"], status=op["status"], obj=op["obj"], iters=op["iters"],
                         targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], cov=cov)
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], cov=cov, traj_t=traj_t,
                   step_index=step, pos_std=0.001, vel_std=0.01, noise_seed=20251015, **o)
    torch.cuda.synchronize()
    x = o["x"].cpu().numpy()
    ns = o["next_states"].cpu().numpy()
    bad = np.nonzero(~np.isfinite(ns).all(axis=1))[0]
    print("step", step, "non-finite agents", len(bad), bad[:10].tolist())
    for a in bad[:5]:
        print(a, o["status"][a].tolist(), o["iters"][a].tolist(), o["obj"][a].tolist(),
              o["primal_res"][a].tolist(), o["dual_res"][a].tolist(), x[a][:6].tolist())
    st = o["next_states"].clone()
