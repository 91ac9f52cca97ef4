"""Closed-loop config-3 run (the bench workload) with per-step status histograms, plus the state
table entering selected steps and the GPU's statuses / objectives / iterations at those steps,
saved for an offline oracle comparison (tools/status_check.py).

    python tools/status_dump.py [--agents 4096 --steps 150 --snap 0,10,50,100,149] -o gpurun_out/sd.npz
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=4096)
    ap.add_argument("--k-hor", type=int, default=15)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--snap", default="0,10,50,100,149")
    ap.add_argument("--slack", action="store_true")
    ap.add_argument("-o", default=os.path.join(REPO, "gpurun_out", "status_dump.npz"))
    a = ap.parse_args()
    import torch
    from mpccbf import swarm, Context
    dev = torch.device("cuda", 0)
    over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if a.slack else {}
    cfg = swarm.config(a.k_hor, **over)
    radius = 3.0 * cfg["d_min"]
    states_h, targets_h = swarm.lattice_swarm(a.agents)
    n = a.agents
    ctx = Context(cfg)
    targets = torch.tensor(targets_h, device=dev)
    out = ctx.alloc_outputs(n)
    traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    status_log = torch.empty((a.steps, n, 2), dtype=torch.int32, device=dev)
    iters_log = torch.empty((a.steps, n, 2), dtype=torch.int32, device=dev)
    snaps = sorted(int(s) for s in a.snap.split(",") if int(s) < a.steps)
    cur = torch.tensor(states_h, device=dev)
    alt = torch.empty_like(cur)
    saved = {}
    common = dict(targets=targets, knn_k=8, knn_radius=radius, x=out["x"], obj=out["obj"],
                  traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=20251015)
    s = 0
    objs = {}

    def advance(k):
        nonlocal s, cur, alt
        r = ctx.run_steps(cur, alt, k, status_log=status_log[s:s + k], iters_log=iters_log[s:s + k],
                          step_index=s, **common)
        if r["final"] is not cur:
            cur, alt = alt, cur
        s += k

    for b in snaps + [a.steps]:
        if b > s:  # advance to the snapshot step
            advance(b - s)
        if b < a.steps:
            saved[b] = cur.cpu().numpy().copy()
            advance(1)  # the snapshot step itself; its objectives
            objs[b] = out["obj"].cpu().numpy().copy()
    torch.cuda.synchronize()
    st = status_log.cpu().numpy()
    it = iters_log.cpu().numpy()
    # per-step histogram: OPTIMAL / INFEASIBLE / ERROR / UNKNOWN attempted / not attempted
    print("step  it0: OPT INF ERR UNK | it1: OPT INF ERR UNK skip | max iters it0 it1")
    for k in range(a.steps):
        h0 = [int(np.sum(st[k, :, 0] == v)) for v in (0, 3, 4, 5)]
        att1 = ~((st[k, :, 1] == 5) & (it[k, :, 1] == 0))
        h1 = [int(np.sum((st[k, :, 1] == v) & att1)) for v in (0, 3, 4, 5)] + [int(np.sum(~att1))]
        if k < 5 or k % 10 == 0 or k in snaps:
            print(k, h0, h1, int(it[k, :, 0].max()), int(it[k, :, 1].max()))
    res = {}
    for k in snaps:
        res[f"states_{k}"] = saved[k]
        res[f"status_{k}"] = st[k]
        res[f"iters_{k}"] = it[k]
        res[f"obj_{k}"] = objs[k]
    np.savez_compressed(a.o, targets=targets_h, snaps=np.array(snaps), status_log=st, iters_log=it,
                        **res)
    print("saved", a.o)


if __name__ == "__main__":
    main()
