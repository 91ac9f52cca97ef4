"""Sub-phase cycle stamps of the wide kernel's IMPC iteration 0 (profiling build, make prof:
MPCCBF_PDIP_STAMPS; impc_wide.hpp WST): mean / p50 shader cycles between consecutive stamps over
the agents whose iteration 0 took 0 solver steps (the fast path), then over those with 1 step.

    MPCCBF_LIB=mpc-cbf_amd/build/prof/libmpccbf.so python tools/wide_stamps.py [N] [warm_steps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
WARM = int(sys.argv[2]) if len(sys.argv) > 2 else 60
NAMES = {0: "rows: entry", 1: "rows: sample table", 2: "rows: row math", 3: "rows: compaction", 4: "rows: lanes+weight",
         5: "solve entry", 6: "solve setup", 7: "scan", 8: "reduce", 9: "-> converged", 10: "dual residual",
         11: "exit", 12: "objective"}
cfg = swarm.config(15)
states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
st = torch.tensor(states_h, device=dev)
tg = torch.tensor(targets_h, device=dev)
ctx = Context(cfg)
ctx.set_variant(5)
out = ctx.alloc_outputs(N)
out.pop("primal_res")
out.pop("dual_res")
for _ in range(WARM):
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=6.0, **out)
    st.copy_(out["next_states"])
stamps = torch.zeros(N * 8 + N * 16, dtype=torch.int64, device=dev)
for _ in range(3):
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=6.0, stamps=stamps, **out)
torch.cuda.synchronize()
s = stamps.cpu().numpy()[N * 8:].reshape(N, 16).astype(np.float64)
it0 = out["iters"].cpu().numpy()[:, 0]
st0 = out["status"].cpu().numpy()[:, 0]
for steps in (0, 1, 2):
    sel = (it0 == steps) & (st0 == 0) & np.all(s[:, :13] > 0, axis=1)
    if not sel.any():
        continue
    print(f"iteration 0 with {steps} solver step(s): {sel.sum()} agents; cycles between stamps (s_memtime)")
    seq = list(range(13))
    tot = 0.0
    for a, b in zip(seq[:-1], seq[1:]):
        d = s[sel, b] - s[sel, a]
        tot += d.mean()
        print(f"   {NAMES[a]:>20s} -> {NAMES[b]:<20s} mean {d.mean():8.0f}  p50 {np.median(d):8.0f}")
    print(f"   total {tot:.0f} cycles")
