"""Closed-loop diagnostics: per-step kernel time, status mix and iteration tail of the fused IMPC
kernel (grid neighbours), plus a dump of the swarm state at chosen steps for CPU replay.

    python tools/loop_stats.py [N] [steps] [out.npz]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 100
OUT = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/loop_stats.npz"
cfg = swarm.config(15)
states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
st = torch.tensor(states_h, device=dev)
tg = torch.tensor(targets_h, device=dev)
ctx = Context(cfg)
out = ctx.alloc_outputs(N)
radius = 3.0 * cfg["d_min"]
dumps = {}
rows = []
for step in range(STEPS):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    snap = st.clone()
    e0.record()
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=radius, **out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    s = out["status"].cpu().numpy()
    it = out["iters"].cpu().numpy()
    att = ~((s == 5) & (it == 0))
    nonopt = np.argwhere((s != 0) & att)
    rows.append((step, ms * 1e3, int(att.sum()), int((s == 0).sum()), int((s == 3).sum()),
                 int((s == 4).sum()), int(it.max()), float(np.percentile(it[att], 99))))
    if step in (0, 1, 5, 20, 50) or (len(nonopt) and f"first_bad" not in dumps):
        key = f"step{step}" if step in (0, 1, 5, 20, 50) else "first_bad"
        dumps[key + "_states"] = snap.cpu().numpy()
        dumps[key + "_status"] = s
        dumps[key + "_iters"] = it
        dumps[key + "_step"] = np.array(step)
    st.copy_(out["next_states"])
print("step  us   attempted optimal infeas error itmax itp99")
for r in rows:
    if r[0] < 10 or r[0] % 10 == 0:
        print("%4d %7.1f %6d %6d %5d %4d %3d %5.1f" % r)
ms = np.array([r[1] for r in rows])
print(f"kernel us: mean {ms.mean():.1f} p50 {np.median(ms):.1f} max {ms.max():.1f}")
dumps["targets"] = targets_h
np.savez_compressed(OUT, **dumps)

# re-time frozen states: first step vs. a late step, repeated
for key in ("step0", "step50"):
    if key + "_states" not in dumps:
        continue
    s_ = torch.tensor(dumps[key + "_states"], device=dev)
    for _ in range(3):
        ctx.impc_solve(s_, targets=tg, knn_k=8, knn_radius=radius, **out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ctx.impc_solve(s_, targets=tg, knn_k=8, knn_radius=radius, **out)
    e1.record()
    torch.cuda.synchronize()
    print(f"frozen {key}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
