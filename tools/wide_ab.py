"""A/B of the one-agent-per-wave kernel (variant 0, impc_wide.hip) against the 16-lane separable
kernel (variant 4, impc_kernel.hip) on identical inputs: closed-loop-evolved state tables of the
bench swarms, one mpccbf_impc_solve per table and variant. Prints per-table status agreement,
objective / control-point differences and iteration counts, then launch times of both variants.

usage: python tools/wide_ab.py [--agents 4096] [--steps 60] [--crowded] [--time]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-cbf_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--crowded", action="store_true")
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--knn", type=int, default=8)
    ap.add_argument("--scale", type=float, default=0.0, help="lattice spacing scale (default 1, --crowded 0.6)")
    ap.add_argument("--variants", default="5,4", help="A,B: the variant under test and the reference")
    args = ap.parse_args()
    import torch
    from mpccbf import swarm, Context

    dev = torch.device("cuda", 0)
    cfg = swarm.config(15)
    scale = args.scale if args.scale > 0 else (0.6 if args.crowded else 1.0)
    states_h, targets_h = swarm.lattice_swarm(args.agents, spacing_scale=scale)
    targets = torch.tensor(targets_h, device=dev)
    va, vb = (int(v) for v in args.variants.split(","))
    ctx = {va: Context(cfg), vb: Context(cfg)}
    for v, c in ctx.items():
        c.set_variant(v)
    print("kernels:", {v: c.kernel_name for v, c in ctx.items()}, flush=True)
    radius = 3.0 * cfg["d_min"]
    # evolve the swarm with variant 4, keeping some tables
    tables = []
    st = torch.tensor(states_h, device=dev)
    out = ctx[vb].alloc_outputs(args.agents)
    keep_at = set([0, 1, 2, 3, 5, 8, 12, 20, 30, 45] + list(range(60, args.steps + 1, 30)))
    for s in range(args.steps + 1):
        if s in keep_at:
            tables.append((s, st.clone()))
        nxt = torch.empty_like(st)
        ctx[vb].impc_solve(st, targets=targets, knn_k=args.knn, knn_radius=radius, next_states=nxt,
                          x=out["x"], status=out["status"], obj=out["obj"], iters=out["iters"], step_index=s,
                          pos_std=0.001, vel_std=0.01, noise_seed=20251015)
        st = nxt
    torch.cuda.synchronize()
    worst = dict(obj=0.0, x=0.0, nxt=0.0)
    tot_mismatch = 0
    for s, tb in tables:
        res = {}
        for v, c in ctx.items():
            o = c.alloc_outputs(args.agents)
            nbo = torch.empty((args.agents, 16), dtype=torch.int32, device=dev)
            c.impc_solve(tb, targets=targets, knn_k=args.knn, knn_radius=radius, nb_out=nbo, **o)
            torch.cuda.synchronize()
            res[v] = {k: t.cpu().numpy() for k, t in o.items()}
            res[v]["nb"] = nbo.cpu().numpy()
        a, b = res[va], res[vb]
        mism = int(np.sum(a["status"] != b["status"]))
        tot_mismatch += mism
        nbm = int(np.sum(np.any(a["nb"] != b["nb"], axis=1)))
        ok = (a["status"] == 0) & (b["status"] == 0)
        dobj = np.abs(a["obj"][ok] - b["obj"][ok]) / np.maximum(1.0, np.abs(b["obj"][ok]))
        okx = ok[:, -1] | ok[:, 0]
        dx = np.nanmax(np.abs(a["x"] - b["x"])) if okx.any() else 0.0
        dn = np.max(np.abs(a["next_states"] - b["next_states"]))
        bit = int(np.sum(np.any(a["x"] != b["x"], axis=1) & ~(np.isnan(a["x"]) & np.isnan(b["x"])).all(axis=1)))
        worst["obj"] = max(worst["obj"], float(dobj.max()) if dobj.size else 0.0)
        worst["x"] = max(worst["x"], float(dx))
        worst["nxt"] = max(worst["nxt"], float(dn))
        hist = {int(k): int(n) for k, n in zip(*np.unique(a["status"], return_counts=True))}
        print(f"step {s:4d}: status mismatch {mism}, nb-list mismatch {nbm}, statuses {hist}, "
              f"max rel obj diff {dobj.max() if dobj.size else 0:.2e}, max |dx| {dx:.2e}, "
              f"max |d next| {dn:.2e}, agents with x not bit-equal {bit}, "
              f"iters mean {a['iters'].mean():.3f}/{b['iters'].mean():.3f} max {a['iters'].max()}/{b['iters'].max()}",
              flush=True)
        if mism:
            idx = np.argwhere(a["status"] != b["status"])[:8]
            for ai, it in idx:
                print(f"   agent {ai} it {it}: wide {a['status'][ai]} ({a['iters'][ai]}) vs sep16 {b['status'][ai]} "
                      f"({b['iters'][ai]}), obj {a['obj'][ai]} vs {b['obj'][ai]}")
    print(f"TOTAL status mismatches {tot_mismatch}; worst rel obj {worst['obj']:.2e}, |dx| {worst['x']:.2e}, "
          f"|d next| {worst['nxt']:.2e}", flush=True)
    if args.time:
        for v, c in ctx.items():
            a0 = torch.tensor(states_h, device=dev)
            a1 = torch.empty_like(a0)
            traj_t = torch.full((args.agents,), -1.0, dtype=torch.float64, device=dev)
            o = c.alloc_outputs(args.agents)
            common = dict(targets=targets, knn_k=args.knn, knn_radius=radius, x=o["x"], obj=o["obj"],
                          traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=20251015)
            c.run_steps(a0, a1, 50, status=o["status"], iters=o["iters"], reserve_steps=300, **common)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = c.run_steps(a0, a1, 300, timing=True, step_index=50, **common)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(f"variant {v} ({c.kernel_name}): 300 steps {el * 1e3:.1f} ms wall, step mean "
                  f"{np.mean(r['step_ms']) * 1e3:.1f} us, kernel(s) mean {np.mean(r['solve_ms']) * 1e3:.1f} us "
                  f"max {np.max(r['solve_ms']) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
