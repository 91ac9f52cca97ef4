"""Debug: ConnectivityControl slack-mode objective mismatches, GPU vs oracle."""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
import mpccbf  # noqa: E402
from test_connectivity_control import _teams, _cfg  # noqa: E402

sizes = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 6, 6, 6, 3, 16]
S, ud, ptr = _teams(sizes, 11)
cfg = _cfg(True)
dev = torch.device("cuda", 0)
t = lambda v, dt=torch.float64: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
R = len(S)
u = torch.empty((R, 3), dtype=torch.float64, device=dev)
status = torch.empty(R, dtype=torch.int32, device=dev)
obj = torch.empty(R, dtype=torch.float64, device=dev)
it = torch.empty(R, dtype=torch.int32, device=dev)
mpccbf.connectivity_control_solve(cfg, t(ptr, torch.int32), t(S), t(ud), u, status=status, obj=obj, iters=it)
torch.cuda.synchronize()
u, status, obj, it = u.cpu().numpy(), status.cpu().numpy(), obj.cpu().numpy(), it.cpu().numpy()


def objective(Sk, i, uu, udi):
    n = len(Sk)
    l2, ev = O.lambda2(Sk[:, :2], cfg["d_max"])
    o = float(np.sum((uu - udi) ** 2))
    vs = np.zeros(n)
    others = [j for j in range(n) if j != i]
    for k, j in enumerate(others):
        a, b = O.safety_cbf(Sk[i], Sk[j], cfg["d_min"])
        vs[k] = max(vs[k], -a @ uu - b)
        if l2 <= 0.1:
            a2, b2 = O.clf_cbf(Sk[i], Sk[j])
            vs[k] = max(vs[k], a2 @ uu + b2)
    if l2 > 0.1:
        a3, b3, _ = O.conn_cbf(Sk, i, ev, l2, cfg["d_max"])
        vs[n - 1] = max(vs[n - 1], -a3 @ uu - b3)
    w = cfg["slack_cost"] * cfg["slack_decay_rate"] ** np.arange(n)
    return o + float(np.sum(w * np.maximum(vs, 0))), vs


for k in range(len(sizes)):
    Sk = S[ptr[k]:ptr[k + 1]]
    for i in range(len(Sk)):
        r = ptr[k] + i
        st, ur, objr, _ = O.connectivity_control(cfg, Sk, i, ud[r])
        if st == 0 and abs(obj[r] - objr) > 1e-6 * max(1, abs(objr)):
            og, vg = objective(Sk, i, u[r], ud[r])
            oo, vo = objective(Sk, i, ur, ud[r])
            print(f"team {k} robot {i}: it {it[r]} obj gpu {obj[r]:.6f} orc {objr:.6f} | recomputed gpu-u {og:.6f} "
                  f"orc-u {oo:.6f} | du {np.max(np.abs(u[r]-ur)):.2e}")
            print("   v(gpu u)", np.round(vg, 6), "\n   v(orc u)", np.round(vo, 6))
