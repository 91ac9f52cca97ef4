"""Debug: FoV slack mode GPU vs oracle mismatches (statuses, iterations, objectives)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from mpccbf import Context, swarm  # noqa: E402
from test_gpu_parity import _estimate_covs  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.6
decay = float(sys.argv[2]) if len(sys.argv) > 2 else 0.9
cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=decay)
n = 100
states, targets = swarm.heading_swarm(n, seed=2)
states[:, :2] *= scale
cov = _estimate_covs(n, 5)
rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
dev = torch.device("cuda", 0)
p = O.make_params(cfg)
refs = swarm.refs_from_targets(targets, 20)
plain = swarm.fov_config(20)
ctx = Context(plain)
out = ctx.alloc_outputs(n)
ctx.impc_solve(torch.tensor(states, device=dev), torch.tensor(rp, device=dev),
               torch.tensor(col, device=dev), targets=torch.tensor(targets, device=dev), **out)
torch.cuda.synchronize()
it_ = out["iters"].cpu().numpy()
st_ = out["status"].cpu().numpy()
print(f"no slack: iters mean {it_[st_ == 0].mean():.2f} max {it_.max()} optimal {np.mean(st_ == 0):.3f}")
for maxit, tol in [(0, 0.0), (0, 1e-8)]:
    ctx = Context(cfg, max_iters=maxit, tol=tol)
    out = ctx.alloc_outputs(n)
    ctx.impc_solve(torch.tensor(states, device=dev), torch.tensor(rp, device=dev),
                   torch.tensor(col, device=dev), targets=torch.tensor(targets, device=dev),
                   cov=torch.tensor(cov, device=dev), **out)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in out.items()}
    bad = 0
    for a in range(n):
        r = O.impc_optimize(p, states, a, col[rp[a]:rp[a + 1]], refs[a], covs=cov)
        if list(g["status"][a]) != list(r["status"]):
            bad += 1
            print(f"maxit={maxit} tol={tol} agent {a}: gpu st {g['status'][a]} it {g['iters'][a]} "
                  f"obj {g['obj'][a]} | oracle st {r['status']} it {r['qp_iters']} obj {r['obj']} "
                  f"nnb {rp[a+1]-rp[a]}")
    print(f"maxit={maxit} tol={tol}: {bad} mismatches; gpu iters mean {g['iters'][g['status']==0].mean():.2f} "
          f"max {g['iters'].max()}")
