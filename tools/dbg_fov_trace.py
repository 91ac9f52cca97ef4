"""Debug: per-iteration PDIP trace (debug build, MPCCBF_DEBUG_TRACE) of one FoV slack QP."""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mpccbf import Context, swarm  # noqa: E402

S = np.load(os.path.join(REPO, "dbgdata", "bad_states.npy"))
step, agent, k = np.load(os.path.join(REPO, "dbgdata", "bad_agent.npy"))
n = len(S)
_, targets_h = swarm.heading_swarm(n)
cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9)
rp, col = swarm.fov_csr(S, 8, cfg["fov_Rs"], cfg["fov_beta"])
dev = torch.device("cuda", 0)
ctx = Context(cfg)
out = ctx.alloc_outputs(n)
stamps = torch.zeros(n * 8 + n * 512, dtype=torch.int64, device=dev)
ctx.impc_solve(torch.tensor(S, device=dev), torch.tensor(rp, device=dev), torch.tensor(col, device=dev),
               targets=torch.tensor(targets_h, device=dev),
               cov=torch.tensor(np.tile([0.1, 0.0, 0.1], (n, 1)), device=dev), stamps=stamps, **out)
torch.cuda.synchronize()
st = out["status"].cpu().numpy()
it = out["iters"].cpu().numpy()
print("agent", agent, "status", st[agent], "iters", it[agent], "nb", col[rp[agent]:rp[agent + 1]])
tr = stamps.cpu().numpy()[n * 8:].reshape(n, 512).view(np.float64)[agent].reshape(64, 8)
print(" it        mu        rp        rd     alpha     sigma        ap        ad  fok")
for i in range(min(64, int(it[agent][1]) % 1000 + 1)):
    r = tr[i]
    print(f"{i:3d} " + " ".join(f"{v:9.2e}" for v in r[:7]) + f"  {int(r[7])}")
