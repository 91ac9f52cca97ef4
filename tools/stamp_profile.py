"""Per-phase timing of the fused IMPC kernel from its s_memrealtime stamps (100 MHz).

Runs the bench workload closed-loop for a few steps, then one instrumented launch per variant,
and prints, over agents: start skew, per-phase durations (setup, neighbours, CBF rows, solves,
outputs) as mean / p50 / p99 / max in microseconds, and the critical (latest-ending) agent.

    python tools/stamp_profile.py [N] [warm_steps] [variants...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import Context, swarm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
WARM = int(sys.argv[2]) if len(sys.argv) > 2 else 100
VARIANTS = [int(v) for v in sys.argv[3:]] or [0, 3]
PH = ["setup", "neighbours", "cbf_rows0", "solve0", "cbf_rows1", "solve1", "outputs"]
FOV = os.environ.get("WORKLOAD", "") == "fov"
SLACK = os.environ.get("SLACK", "") == "1"
COV = None
if FOV:
    cfg = swarm.fov_config(20, **(dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if SLACK else {}))
    states_h, targets_h = swarm.heading_swarm(N)
    states_h[:, :2] *= float(os.environ.get("SCALE", "1.0"))
else:
    cfg = swarm.config(15)
    states_h, targets_h = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
st = torch.tensor(states_h, device=dev)
tg = torch.tensor(targets_h, device=dev)
radius = cfg["fov_Rs"] if FOV else 3.0 * cfg["d_min"]
ctx = Context(cfg)
out = ctx.alloc_outputs(N)
if os.environ.get("RESIDUALS", "") != "1":  # as the bench: no residual outputs (no dual-residual check)
    out.pop("primal_res", None)
    out.pop("dual_res", None)
if FOV and SLACK:
    COV = torch.tensor(np.tile([0.1, 0.0, 0.1], (N, 1)), device=dev)
for _ in range(WARM):
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=radius, cov=COV, **out)
    st.copy_(out["next_states"])
torch.cuda.synchronize()
snap = st.clone()
PDIP = os.environ.get("MPCCBF_LIB", "").find("prof") >= 0  # profiling build: in-loop stamps
TRACE = os.environ.get("MPCCBF_LIB", "").find("trace") >= 0  # trace build: per-step traces
PPH_FOV = ["rows+LDS", "gram (MFMA)", "reduce+Py+rd", "cholesky", "pred solve", "pred rows+red",
           "corr G^T v", "corr solve", "step rows+red", "update y", "tail"]
PPH = ["rows+acc", "reduce acc", "rp/py/conv", "cholesky", "pred solve", "pred steps+min",
       "mua", "corr rows+vc", "corr solve", "corr steps+min", "update"]
for v in VARIANTS:
    ctx.set_variant(v)
    stamps = torch.zeros(N * 8 + (N * 32 if PDIP else 0) + (N * 2 * 256 if TRACE else 0), dtype=torch.int64,
                         device=dev)
    for rep in range(3):  # last rep measured (warm caches)
        ctx.impc_solve(snap, targets=tg, knn_k=8, knn_radius=radius, stamps=stamps, cov=COV, **out)
    torch.cuda.synchronize()
    allst = stamps.cpu().numpy()
    s = allst[:N * 8].reshape(N, 8).astype(np.float64) * 0.01  # 10 ns ticks -> us
    if PDIP and v == 0:
        # shader cycles (per agent: 32 stamps in the 16-lane kernel, 16 in the FoV kernel)
        ps = (allst[N * 8:N * 24].reshape(N, 16) if FOV else allst[N * 8:N * 40].reshape(N, 32)[:, :16]).astype(np.float64)
        okp = ps[:, 11] > 0
        d = np.diff(ps[okp, :12], axis=1)
        tot = ps[okp, 11] - ps[okp, 0]
        print(f"variant {v}: Newton step 2 of solve 0, {okp.sum()} agents, cycles mean {tot.mean():.0f} "
              f"p50 {np.median(tot):.0f}")
        s_tmp = allst[:N * 8].reshape(N, 8)
        crit0 = int(np.argmax(s_tmp[:, 7] - s_tmp[:, 0].min()))
        dc = np.diff(ps[crit0, :12]) if okp[crit0] else None
        for k, name in enumerate(PPH_FOV if FOV else PPH):
            print(f"   {name:15s} mean {d[:, k].mean():7.0f}  p50 {np.median(d[:, k]):7.0f} cycles"
                  + (f"   critical agent {dc[k]:7.0f}" if dc is not None else ""))
    if PDIP and v == 0 and not FOV:  # dual active-set stamps (solve 0, first steps)
        # (the 16-lane kernel: 32 stamps per agent, 16 .. 21 around the solver call)
        ps = allst[N * 8:N * 40].reshape(N, 32).astype(np.float64)
        its0_ = out["iters"].cpu().numpy()[:, 0]
        for nstep in (0, 1, 2):
            m = (ps[:, 21] > 0) & (its0_ == nstep) & (ps[:, 16] > 0) & (ps[:, 19] > 0)
            if m.sum() == 0:
                continue
            print(f"variant {v}: solve phase around the solver, {nstep} step(s): {m.sum()} agents")
            for name, a, b in [("nfin checks", 16, 17), ("to solver entry", 17, 12), ("solver", 12, 10),
                               ("to solve exit", 10, 18), ("objective", 18, 19), ("ykeep", 19, 20),
                               ("write_iteration", 20, 21)]:
                d = ps[m, b] - ps[m, a]
                print(f"   {name:17s} mean {d.mean():7.0f}  p50 {np.median(d):7.0f} cycles")
        its0 = out["iters"].cpu().numpy()[:, 0]
        # (the first scan is the fast-start test; the first side joins an empty active set
        # without substitutions, so stamps 4 and 5 belong to later steps only)
        names = [("solver entry", 12, 13), ("call", 13, 0), ("init", 0, 1),
                 ("scan 1/fast start", 1, 2), ("stage", 2, 3), ("first side", 3, 6),
                 ("scan 2", 6, 8), ("dual residual", 8, 9), ("exit", 9, 10)]
        names0 = [("solver entry", 12, 13), ("call", 13, 0), ("init", 0, 1),
                  ("scan/fast start", 1, 2), ("converged", 2, 9), ("exit", 9, 10)]
        # the second step (k = 1 -> 2, the general step with substitutions) of two-step solves
        names2 = [("solver entry", 12, 13), ("call", 13, 0), ("init", 0, 1),
                  ("scan 1/fast start", 1, 2), ("stage 1", 2, 3), ("first side", 3, 6),
                  ("scan 2", 6, 8), ("stage 2", 8, 7), ("subst v, rho", 7, 4), ("step lengths", 4, 11),
                  ("update y, u", 11, 5), ("join", 5, 14), ("scan 3 + rd", 14, 9), ("exit", 9, 10)]
        for nstep in (0, 1, 2):
            m = (ps[:, 15] == 1) & (its0 == nstep) & (ps[:, 10] > 0)
            if m.sum() == 0:
                continue
            print(f"variant {v}: dual active-set solves with {nstep} step(s): {m.sum()} agents, "
                  f"cycles entry->exit mean {np.mean(ps[m, 10] - ps[m, 12]):.0f}")
            for name, a, b in (names0 if nstep == 0 else (names2 if nstep == 2 else names)):
                d = ps[m, b] - ps[m, a]
                print(f"   {name:15s} mean {d.mean():7.0f}  p50 {np.median(d):7.0f} cycles")
    if PDIP and v == 0 and FOV:  # the wave dual active set's stamps (das_wave.hpp, solve 0)
        ps = allst[N * 8:N * 24].reshape(N, 16).astype(np.float64)
        names = [("init", 0, 1), ("scan 1", 1, 2), ("candidate P^-1 g", 2, 3), ("subst + dots", 3, 4),
                 ("step lengths", 4, 5), ("update y, u", 5, 6), ("join", 6, 7), ("scan 2", 7, 8)]
        names0 = [("init", 0, 1), ("scan", 1, 2), ("converged", 2, 9), ("dual residual", 9, 10)]
        for nstep in (0, 1, 2, 3):
            m = (ps[:, 15] == 2) & (ps[:, 14] == nstep) & (ps[:, 10] > 0)
            if m.sum() == 0:
                continue
            print(f"variant {v}: wave active-set solves with {nstep} step(s): {m.sum()} agents, "
                  f"cycles entry->exit mean {np.mean(ps[m, 10] - ps[m, 0]):.0f}")
            for name, a, b in (names0 if nstep == 0 else names + [("rest to exit", 8, 10)]):
                d = ps[m, b] - ps[m, a]
                print(f"   {name:17s} mean {d.mean():7.0f}  p50 {np.median(d):7.0f} cycles")
    status = out["status"].cpu().numpy()
    t0 = s[:, 0].min()
    start = s[:, 0] - t0
    end = s[:, 7] - t0
    print(f"variant {v}: span {end.max():.1f} us, start skew p50 {np.median(start):.1f} "
          f"max {start.max():.1f} us, agent wall mean {np.mean(end - start):.1f} max {np.max(end - start):.1f}")
    # phases; iteration-1 phases only for agents that attempted iteration 1
    for k, name in enumerate(PH):
        d = s[:, k + 1] - s[:, k]
        if k >= 4:
            d = d[status[:, 0] == 0]
        if k == 4 or k == 5:
            pass
        print(f"   {name:11s} mean {d.mean():7.2f} p50 {np.median(d):7.2f} p99 {np.percentile(d, 99):7.2f} "
              f"max {d.max():7.2f} us")
    its = out["iters"].cpu().numpy()
    ok0 = (status[:, 0] == 0) & (its[:, 0] > 0)
    per = (s[ok0, 4] - s[ok0, 3]) / its[ok0, 0]
    print(f"   solve0 per Newton iteration: mean {per.mean():.2f} p50 {np.median(per):.2f} us "
          f"(iters mean {its[ok0, 0].mean():.1f})")
    crit = int(np.argmax(end))
    if os.environ.get("CP_JSON"):  # bench.py's roofline.critical_path reads these entries
        import json
        path = os.environ["CP_JSON"]
        d = json.load(open(path)) if os.path.exists(path) else {"entries": []}
        d["entries"].append({"kernel": ctx.kernel_name, "workload": "fov" if FOV else "collision", "agents": N,
                             "variant": v, "span_us": float(end.max()), "agent_wall_max_us": float(np.max(end - start)),
                             "agent_wall_mean_us": float(np.mean(end - start)),
                             "phases_mean_us": {nm: float(np.mean((s[:, k + 1] - s[:, k])[(s[:, k] > 0) & (s[:, k + 1] > 0)]))
                                                for k, nm in enumerate(PH)},
                             "critical_agent_phases_us": [float(x) for x in np.diff(s[crit])]})
        json.dump(d, open(path, "w"), indent=1)
    print(f"   critical agent {crit}: status {status[crit]}, start {start[crit]:.1f}, "
          f"phases {np.round(np.diff(s[crit]), 2)}")
    print(f"   critical agent iters {its[crit]}")
    w0 = (crit // 4) * 4
    for a in range(w0, w0 + 4):  # the critical wave (4 agents of 16 lanes)
        sp = [(int(v) % 100, int(v) // 100 % 100, int(v) // 10000) for v in its[a]] if TRACE else its[a]
        print(f"      wave agent {a}: status {status[a]} iters (warm, cold, phase1) {sp}")
    # how many agents end late, and the latest end per iteration-0 status
    print(f"   agents ending after 0.8*span: {(end > 0.8 * end.max()).sum()}")
    for stv in np.unique(status[:, 0]):
        m = status[:, 0] == stv
        print(f"   status0 {stv}: {m.sum()} agents, wall max {np.max(end[m] - start[m]):.1f} "
              f"p99 {np.percentile(end[m] - start[m], 99):.1f} us, solve0 iters max {its[m, 0].max()}")
