"""Where a launch's time goes outside the stamped phases: runs closed-loop steps with both the
launch clock (every wave's start / end) and the diagnostics build's phase stamps (each agent's
stamp 0 after the prologue, stamp 7 after its outputs), all s_memrealtime (100 MHz), and prints the
launch split into prologue (first wave start -> first stamp 0), stamped span, and epilogue (last
stamp 7 -> last wave end), with per-agent prologue / epilogue distributions.

    MPCCBF_LIB=mpc-cbf_amd/build/stamps/libmpccbf.so python tools/clock_vs_stamps.py [N] [steps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = swarm.config(15)
states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
st = torch.tensor(states_h, device=dev)
alt = st.clone()
tg = torch.tensor(targets_h, device=dev)
ctx = Context(cfg)
out = ctx.alloc_outputs(N)
kw = dict(targets=tg, knn_k=8, knn_radius=3.0 * cfg["d_min"], x=out["x"], status=out["status"],
          obj=out["obj"], iters=out["iters"])
ctx.run_steps(st, alt, 50, **kw)
waves = ctx.launch_waves(N)
for rep in range(3):
    clock = torch.zeros((STEPS, waves, 2), dtype=torch.int64, device=dev)
    stamps = torch.zeros(N * 8 + N * 16, dtype=torch.int64, device=dev)
    ctx.run_steps(st, alt, STEPS, kernel_clock=clock, stamps=stamps, **kw)
    torch.cuda.synchronize()
c = clock[-1].cpu().numpy().astype(np.float64) * 0.01
s = stamps[:N * 8].cpu().numpy().reshape(N, 8).astype(np.float64) * 0.01
c = c[c[:, 0] > 0]
t0, t1 = c[:, 0].min(), c[:, 1].max()
ok = (s[:, 0] > 0) & (s[:, 7] > 0)
s0, s7 = s[ok, 0], s[ok, 7]
print(f"N {N}, waves {len(c)}, agents stamped {ok.sum()}")
print(f"launch (clock) {t1 - t0:.2f} us = prologue {s0.min() - t0:.2f} + stamped span {s7.max() - s0.min():.2f} "
      f"+ epilogue {t1 - s7.max():.2f}")
print(f"wave start skew: p50 {np.median(c[:, 0] - t0):.2f} max {(c[:, 0] - t0).max():.2f} us; "
      f"first stamp 0 per agent after launch start: p50 {np.median(s0 - t0):.2f} max {(s0 - t0).max():.2f}")
print(f"wave end after launch start: p50 {np.median(c[:, 1] - t0):.2f} max {(c[:, 1] - t0).max():.2f}; "
      f"stamp 7 p50 {np.median(s7 - t0):.2f} max {(s7 - t0).max():.2f}")
print(f"wave durations: p50 {np.median(c[:, 1] - c[:, 0]):.2f} max {(c[:, 1] - c[:, 0]).max():.2f}; "
      f"agent stamp0->7: p50 {np.median(s7 - s0):.2f} max {(s7 - s0).max():.2f}")
