"""Debug: closed-loop FoV slack QPs that end UNKNOWN on the GPU, re-solved by the oracle."""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from mpccbf import Context, swarm  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 512
cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9)
states_h, targets_h = swarm.heading_swarm(n)
dev = torch.device("cuda", 0)
ctx = Context(cfg)
st = torch.tensor(states_h, device=dev)
nxt = torch.empty_like(st)
tg = torch.tensor(targets_h, device=dev)
cov_h = np.tile([0.1, 0.0, 0.1], (n, 1))
cov = torch.tensor(cov_h, device=dev)
out = ctx.alloc_outputs(n)
out.pop("next_states")
traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
p = O.make_params(cfg)
refs = swarm.refs_from_targets(targets_h, 20)
found = 0
for s in range(steps):
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], next_states=nxt, traj_t=traj_t,
                   pos_std=0.001, vel_std=0.01, noise_seed=20251015, step_index=s, cov=cov, **out)
    torch.cuda.synchronize()
    it = out["iters"].cpu().numpy()
    stt = out["status"].cpu().numpy()
    bad = np.nonzero((stt == 5) & (it >= 30))
    if len(bad[0]):
        S = st.cpu().numpy()
        rp, col = swarm.fov_csr(S, 8, cfg["fov_Rs"], cfg["fov_beta"])
        for a, k in zip(*bad):
            r = O.impc_optimize(p, S, int(a), col[rp[a]:rp[a + 1]], refs[a], covs=cov_h)
            print(f"step {s} agent {a} iter {k}: gpu st {stt[a]} it {it[a]} | oracle st {r['status']} "
                  f"it {r['qp_iters']} obj {r['obj']} nnb {rp[a+1]-rp[a]}", flush=True)
            if found == 0:
                np.save(os.path.join(REPO, "gpurun_out", "bad_states.npy"), S)
                np.save(os.path.join(REPO, "gpurun_out", "bad_agent.npy"), np.array([s, a, k]))
            found += 1
    st, nxt = nxt, st
print("found", found)
