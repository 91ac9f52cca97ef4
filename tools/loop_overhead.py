"""Wall time per control step of mpccbf_run_steps under different timing-event settings
(events add barrier packets between kernels)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N, K = 4096, 1000
cfg = swarm.config(15)
states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
ctx = Context(cfg)
tg = torch.tensor(targets_h, device=dev)
out = ctx.alloc_outputs(N)
a = torch.tensor(states_h, device=dev)
b = torch.empty_like(a)
common = dict(targets=tg, knn_k=8, knn_radius=6.0, x=out["x"], obj=out["obj"], status=out["status"],
              iters=out["iters"], reserve_steps=K)
ctx.run_steps(a, b, 50, **common)
for name, kw in [("no events", dict()), ("step events", dict(timing=True, solve_stride=10 ** 9)),
                 ("step + solve/16", dict(timing=True, solve_stride=16)),
                 ("solve/16 only", dict(timing=True, solve_stride=16, step_timing=False)),
                 ("all events", dict(timing=True, solve_stride=1))]:
    a.copy_(torch.tensor(states_h, device=dev))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = ctx.run_steps(a, b, K, **common, **kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e6
    extra = ""
    if kw.get("timing"):
        if r["step_ms"] is not None:
            extra += f" step p50 {np.median(r['step_ms']) * 1e3:.1f} us"
        if len(r["solve_ms"]):
            extra += f" solve {np.mean(r['solve_ms']) * 1e3:.1f} us"
    print(f"{name:16s} {dt:7.1f} us/step{extra}")
