"""The FoV kernel's setup split by the setupst build's stamps (make -C mpc-cbf_amd setupst): stamp 0
at the start, 2 after the operator loads' issue, 3 after the linear term, 4 after the box rows, 5
after the neighbour states, 6 after the constant rows, 1 after the operator stores (s_memrealtime,
100 MHz). Prints mean / p50 / max of each interval over agents, in microseconds.

    MPCCBF_LIB=mpc-cbf_amd/build/setupst/libmpccbf.so python tools/setup_stamps.py [N] [warm]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
WARM = int(sys.argv[2]) if len(sys.argv) > 2 else 100
cfg = swarm.fov_config(20)
states_h, targets_h = swarm.heading_swarm(N)
dev = torch.device("cuda", 0)
st = torch.tensor(states_h, device=dev)
tg = torch.tensor(targets_h, device=dev)
ctx = Context(cfg)
out = ctx.alloc_outputs(N)
out.pop("primal_res", None)
out.pop("dual_res", None)
for _ in range(WARM):
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], **out)
    st.copy_(out["next_states"])
stamps = torch.zeros(N * 8, dtype=torch.int64, device=dev)
for rep in range(3):
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], stamps=stamps, **out)
torch.cuda.synchronize()
s = stamps.cpu().numpy().reshape(N, 8).astype(np.float64) * 0.01
order = [0, 2, 3, 4, 5, 6, 1]
names = ["operator loads issued", "linear term", "box rows", "neighbour states", "constant rows",
         "operator stores"]
ok = np.all(s[:, order] > 0, axis=1)
print(f"agents {ok.sum()} of {N}; setup (0 -> 1) mean {np.mean(s[ok, 1] - s[ok, 0]):.2f} us")
for k in range(len(names)):
    d = s[ok, order[k + 1]] - s[ok, order[k]]
    print(f"   {names[k]:22s} mean {d.mean():6.2f} p50 {np.median(d):6.2f} max {d.max():6.2f} us")
