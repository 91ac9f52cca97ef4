"""IMPC iteration-1 warm start sweep (MPCCBF_WARM_DELTA, read at context creation): closed-loop
bench workload (config 3) per delta — step time, kernel time, Newton steps of both IMPC
iterations — and a same-input check of objectives / control points against the cold start.

    python tools/warm_sweep.py [steps] [delta ...]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 300
DELTAS = [float(v) for v in sys.argv[2:]] or [0.0, 1e-1, 3e-2, 1e-2, 1e-3]
N = 4096
cfg = swarm.config(15)
states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
radius = 3.0 * cfg["d_min"]
targets = torch.tensor(targets_h, device=dev)
probe = None
ref = None
for delta in DELTAS:
    os.environ["MPCCBF_WARM_DELTA"] = repr(delta)
    ctx = Context(cfg)
    out = ctx.alloc_outputs(N)
    out.pop("next_states")
    tables = [torch.tensor(states_h, device=dev), torch.empty((N, 6), dtype=torch.float64, device=dev)]
    traj_t = torch.full((N,), -1.0, dtype=torch.float64, device=dev)
    common = dict(targets=targets, agent_first=0, num_agents=N, knn_k=8, knn_radius=radius,
                  x=out["x"], obj=out["obj"], traj_t=traj_t, pos_std=0.001, vel_std=0.01,
                  noise_seed=20251015)
    r = ctx.run_steps(tables[0], tables[1], 50, status=out["status"], iters=out["iters"],
                      reserve_steps=STEPS, **common)
    if r["final"] is not tables[0]:
        tables.reverse()
    if probe is None:
        probe = tables[0].clone()  # same-input check: the cold start's state after warm-up
    st_log = torch.empty((STEPS, N, 2), dtype=torch.int32, device=dev)
    it_log = torch.empty((STEPS, N, 2), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = ctx.run_steps(tables[0], tables[1], STEPS, status_log=st_log, iters_log=it_log, timing=True,
                      solve_stride=16, step_index=50, **common)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / STEPS * 1e3
    st, it = st_log.cpu().numpy(), it_log.cpu().numpy()
    it1 = it[..., 1][st[..., 1] == 0]
    it0 = it[..., 0][st[..., 0] == 0]
    wave1 = it[..., 1].reshape(STEPS, N // 4, 4).max(-1)
    wave0 = it[..., 0].reshape(STEPS, N // 4, 4).max(-1)
    crit = (wave0 + wave1).max(-1)
    # same input, one solve
    o = ctx.alloc_outputs(N)
    ctx.impc_solve(probe, targets=targets, agent_first=0, num_agents=N, knn_k=8, knn_radius=radius, **o)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in o.items()}
    line = (f"delta={delta:g} ms/step={dt:.4f} kern_us={np.mean(r['solve_ms'])*1e3:.1f} "
            f"it0 mean={it0.mean():.2f} max={it0.max()} it1 mean={it1.mean():.2f} p99={np.percentile(it1, 99):.0f} "
            f"max={it1.max()} crit_wave mean={crit.mean():.1f} max={crit.max()} "
            f"status0={np.bincount(st[...,0].ravel(), minlength=7)[:7].tolist()} "
            f"status1={np.bincount(st[...,1].ravel(), minlength=7)[:7].tolist()}")
    if ref is None:
        ref = res
    else:
        ok = (res["status"] == ref["status"]).all()
        m = (ref["status"][:, -1] == 0) & (res["status"][:, -1] == 0)
        dobj = np.abs(res["obj"][m] - ref["obj"][m]) / np.maximum(1, np.abs(ref["obj"][m]))
        dx = np.abs(res["x"][m] - ref["x"][m]).max()
        line += f" | vs cold: status_eq={ok} max_rel_obj={dobj.max():.2e} max_dx={dx:.2e}"
    print(line, flush=True)
