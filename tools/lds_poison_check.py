"""Uninitialised-LDS check (diagnostics, GPU): run closed loops of the IMPC kernels with one
library build and save every step's statuses, solver steps, objectives and next states.
Run once per `make poison` build (static LDS filled with 1e300 / -7.25 at block start) and
compare: any difference is a read of LDS the kernel never wrote.

    MPCCBF_LIB=mpc-cbf_amd/build/poison_a/libmpccbf.so python tools/lds_poison_check.py run a.npz
    MPCCBF_LIB=mpc-cbf_amd/build/poison_b/libmpccbf.so python tools/lds_poison_check.py run b.npz
    python tools/lds_poison_check.py cmp a.npz b.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))


def run(path, steps=30):
    import torch
    import mpccbf
    from mpccbf import swarm
    dev = torch.device("cuda", 0)
    res = {}
    cases = {
        "fov": (swarm.fov_config(20), "heading", 512, None),
        "fovs": (swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9), "heading", 512, 0.1),
        "coll": (swarm.config(15), "lattice", 4096, None),
        "coll_slack": (swarm.config(15, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9), "lattice", 1024, None),
        "crowded": (swarm.config(15), "crowded", 1024, None),
    }
    for name, (cfg, kind, n, covv) in cases.items():
        if kind == "heading":
            states, targets = swarm.heading_swarm(n)
        elif kind == "crowded":
            states, targets = swarm.lattice_swarm(n, spacing_scale=0.6)
        else:
            states, targets = swarm.lattice_swarm(n)
        ctx = mpccbf.Context(cfg)
        out = ctx.alloc_outputs(n)
        traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        out["x"].fill_(float("nan"))
        cur = torch.tensor(states, device=dev)
        tg = torch.tensor(targets, device=dev)
        cov = torch.tensor(np.tile([covv, 0.0, covv], (n, 1)), device=dev) if covv else None
        radius = cfg["fov_Rs"] if "fov_Rs" in cfg else 3.0 * cfg.get("d_min", 2.0)
        log = {k: [] for k in ("status", "iters", "obj", "next_states")}
        for s in range(steps):
            kw = dict(cov=cov) if cov is not None else {}
            ctx.impc_solve(cur, targets=tg, knn_k=8, knn_radius=radius, traj_t=traj_t, step_index=s,
                           pos_std=0.001, vel_std=0.01, noise_seed=20251015, **kw, **out)
            for k in log:
                log[k].append(out[k].cpu().numpy().copy())
            cur = out["next_states"].clone()
        torch.cuda.synchronize()
        for k, v in log.items():
            res[f"{name}_{k}"] = np.stack(v)
        print(name, "done", flush=True)
    np.savez(path, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        same = (x == y) | (np.isnan(x) & np.isnan(y)) if x.dtype.kind == "f" else x == y
        if not same.all():
            idx = np.argwhere(~same)
            print(f"DIFF {k}: {len(idx)} entries, first (step, agent, ...) {idx[:4].tolist()}")
            bad += 1
        else:
            print(f"same {k}")
    print("RESULT", "identical" if bad == 0 else f"{bad} arrays differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
