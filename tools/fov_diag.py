"""Re-solve the FoV (config 5) QPs of a `bench.py --workload fov --dump` trace on the GPU, once with
the default solver and once with the PDIP alone (mpccbf_options.dual_as_steps < 0), and list the agents whose
default solve took many steps: which QPs the dual active set hands to the PDIP.

    python tools/fov_diag.py gpurun_out/<tag>/fov.npz [first_step] [last_step] [min_steps] [--slack]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))


def main():
    import torch
    from mpccbf import Context, swarm
    slack = "--slack" in sys.argv
    av = [a for a in sys.argv[1:] if not a.startswith("--")]
    d = np.load(av[0])
    s0 = int(av[1]) if len(av) > 1 else 0
    s1 = int(av[2]) if len(av) > 2 else 10
    min_steps = int(av[3]) if len(av) > 3 else 8
    traj, warm = d["traj"], int(d["warmup"])
    n = traj.shape[0]
    over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if slack else {}
    cfg = swarm.fov_config(20, **over)
    _, targets = swarm.heading_swarm(n)
    dev = torch.device("cuda", 0)
    ctx_p = Context(cfg, dual_as_steps=-1)  # the PDIP alone
    ctx = Context(cfg)
    tg = torch.tensor(targets, device=dev)
    common = dict(targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"])
    if slack:
        common["cov"] = torch.tensor(np.tile([0.1, 0.0, 0.1], (n, 1)), dtype=torch.float64, device=dev)
    for s in range(s0, s1):
        cur = torch.tensor(traj[:, warm + s, :], device=dev)
        res = []
        for c in (ctx, ctx_p):
            o = c.alloc_outputs(n)
            o.pop("next_states")
            if "primal_res" not in o:
                o["primal_res"] = torch.empty((n, cfg["impc_iter"]), dtype=torch.float64, device=dev)
                o["dual_res"] = torch.empty_like(o["primal_res"])
            c.impc_solve(cur, **o, **common)
            torch.cuda.synchronize()
            r = {k: v.cpu().numpy() for k, v in o.items()}
            r["pr"], r["dr"] = r["primal_res"], r["dual_res"]
            res.append(r)
        a, b = res
        agents = np.nonzero(a["iters"].max(axis=1) >= min_steps)[0]
        print(f"step {s}: dump max {int(d['iters'][s].max())}, re-solve max {int(a['iters'].max())}; "
              f"{len(agents)} agents >= {min_steps} steps")
        for i in agents[:12]:
            print(f"   agent {i}: default iters {a['iters'][i].tolist()} status {a['status'][i].tolist()} "
                  f"rp {np.array2string(a['pr'][i], precision=2)} rd {np.array2string(a['dr'][i], precision=2)} | "
                  f"pdip iters {b['iters'][i].tolist()} status {b['status'][i].tolist()}", flush=True)


if __name__ == "__main__":
    main()
