"""Debug: slack-mode statuses / iterations on the GPU vs the oracle for one seeded swarm."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import oracle_lib as O  # noqa: E402
from mpccbf import Context, swarm  # noqa: E402

scale, k = float(sys.argv[1]), int(sys.argv[2])
slack = int(sys.argv[3]) if len(sys.argv) > 3 else 1
cfg = swarm.config(k, slack_mode=slack)
states, targets = swarm.lattice_swarm(64, seed=21)
states[:, :2] *= scale
rp, col = swarm.knn_csr(states, 8, 6.0)
dev = torch.device("cuda", 0)
ctx = Context(cfg)
out = ctx.alloc_outputs(64)
stamps = torch.zeros(64 * 8 + 64 * 16 + 64 * 16 + 16, dtype=torch.int64, device=dev) if os.environ.get("MPCCBF_LIB") else None
ctx.impc_solve(torch.tensor(states, device=dev), torch.tensor(rp, device=dev), torch.tensor(col, device=dev),
               targets=torch.tensor(targets, device=dev), stamps=stamps, **out)
torch.cuda.synchronize()
st = out["status"].cpu().numpy()
it = out["iters"].cpu().numpy()
ob = out["obj"].cpu().numpy()
np.savez(os.path.join(os.path.dirname(__file__), "..", "gpurun_out", f"dbg_slack_{scale}_{k}_{slack}.npz"),
         x=out["x"].cpu().numpy(), status=st, obj=ob, iters=it)
dd = stamps.cpu().numpy()[64 * 8:64 * 24].view(np.float64).reshape(64, 16) if stamps is not None else np.zeros((64, 16))
lane_exit = stamps.cpu().numpy()[64 * 24:64 * 40].reshape(64, 16) if stamps is not None else None
p = O.make_params(cfg)
refs = swarm.refs_from_targets(targets, k)
for a in range(64):
    r = O.impc_optimize(p, states, a, col[rp[a]:rp[a + 1]], refs[a])
    flag = "" if list(r["status"]) == list(st[a]) else "  <-- MISMATCH"
    print(a, st[a], it[a], ob[a], "| oracle", r["status"], r["qp_iters"], r["obj"], flag)
    if lane_exit is not None and len(set(lane_exit[a].tolist())) > 1:
        print("    lanes exit at different iterations:", lane_exit[a].tolist())
    if stamps is not None and dd[a, 13] > 0:
        print("    acc non-uniform from iteration", int(dd[a, 13]) - 1, "by", dd[a, 12])
    if stamps is not None and dd[a, 15] > 0:
        print("    y diverges across lanes from iteration", int(dd[a, 15]) - 1, "by", dd[a, 14])
    if flag and it[a, 0] >= 4000:
        print("    failed matrices:", np.array2string(dd[a, :12], precision=3))
