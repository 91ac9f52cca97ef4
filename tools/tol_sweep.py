"""PDIP tolerance vs kernel time and parity: closed-loop bench workload (config 3 and config 5)
at several relative tolerances; parity of one step's QPs against the oracle."""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
from mpccbf import Context, swarm  # noqa: E402

dev = torch.device("cuda", 0)
for wl in ("collision", "fov"):
    fov = wl == "fov"
    n = 512 if fov else 4096
    cfg = swarm.fov_config(20) if fov else swarm.config(15)
    states_h, targets_h = (swarm.heading_swarm if fov else swarm.lattice_swarm)(n)
    radius = cfg["fov_Rs"] if fov else 6.0
    for tol in (1e-9, 1e-8, 1e-7):
        ctx = Context(cfg, tol=tol)
        a = torch.tensor(states_h, device=dev)
        b = torch.empty_like(a)
        tg = torch.tensor(targets_h, device=dev)
        out = ctx.alloc_outputs(n)
        traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        common = dict(targets=tg, knn_k=8, knn_radius=radius, x=out["x"], obj=out["obj"], traj_t=traj_t,
                      pos_std=0.001, vel_std=0.01, noise_seed=20251015)
        r = ctx.run_steps(a, b, 50, status=out["status"], iters=out["iters"], **common)
        t0 = r["final"]
        t1 = b if t0 is a else a
        il = torch.empty((300, n, 2), dtype=torch.int32, device=dev)
        r = ctx.run_steps(t0, t1, 300, iters_log=il, timing=True, solve_stride=1, step_index=50, **common)
        it = il.cpu().numpy()
        kern = np.mean(r["solve_ms"]) * 1e3
        # parity on one step from the state the loop reached
        S = r["final"].cpu().numpy()
        o2 = ctx.alloc_outputs(n)
        ctx.impc_solve(r["final"], targets=tg, knn_k=8, knn_radius=radius, **o2)
        torch.cuda.synchronize()
        st, obj, x = o2["status"].cpu().numpy(), o2["obj"].cpu().numpy(), o2["x"].cpu().numpy()
        rp, col = (swarm.fov_csr(S, 8, radius, cfg["fov_beta"]) if fov else swarm.knn_csr(S, 8, radius))
        p = O.make_params(cfg)
        refs = swarm.refs_from_targets(targets_h, cfg["k_hor"])
        worst_obj = worst_x = 0.0
        mism = 0
        for ag in range(0, n, 8 if not fov else 2):
            ref = O.impc_optimize(p, S, ag, col[rp[ag]:rp[ag + 1]], refs[ag])
            if list(st[ag]) != list(ref["status"]):
                mism += 1
                continue
            last = [k for k in range(2) if ref["status"][k] == 0]
            for k in last:
                worst_obj = max(worst_obj, abs(obj[ag, k] - ref["obj"][k]) / max(1, abs(ref["obj"][k])))
            if last:
                worst_x = max(worst_x, np.max(np.abs(x[ag] - ref["x"][last[-1]][:x.shape[1]])))
        print(f"{wl} tol {tol:g}: kernel {kern:.1f} us, iters mean {it[it > 0].mean():.2f} max {it.max()}, "
              f"status mismatches {mism}, worst obj rel {worst_obj:.2e}, worst x {worst_x:.2e}", flush=True)
