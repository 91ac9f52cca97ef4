"""Offline study of the dual active-set (Goldfarb-Idnani) step counts on real QPs: for the agents a
`bench.py --dump` (with the state trace) records, the oracle assembles IMPC iteration 0's QP, the
equalities are eliminated (null space), and the range-space dual active-set method of
pdip_sep.hpp sep_dual_as runs in numpy with different candidate rules:
  scaled  — the device's rule: the largest violation scaled by 1 / (1 + |bound|)
  normal  — the violation divided by the side's norm in the P^-1 metric, sqrt(g P^-1 g)
Prints the step counts per rule (test infrastructure: CPU only).

    python tools/das_sim.py gpurun_out/<tag>/dump.npz [min_steps] [sample] [--fov [--slack]] [--it1]
(--fov: a `bench.py --workload fov` dump, config 5 with the FoV-filtered neighbours.)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
import oracle_lib as O  # noqa: E402
from mpccbf import swarm  # noqa: E402


def reduce_qp(qp):
    """x = xp + Z y over the equality rows; returns P, q, sides (N y <= b)."""
    A, lo, hi = qp["A"], qp["lo"], qp["hi"]
    eq = lo == hi
    E, e = A[eq], lo[eq]
    xp = np.linalg.lstsq(E, e, rcond=None)[0]
    _, s, vt = np.linalg.svd(E)
    r = int((s > 1e-10 * s[0]).sum())
    Z = vt[r:].T
    H2 = qp["H"] + qp["H"].T  # objective x^T H x (H upper): Hessian H + H^T
    P = Z.T @ H2 @ Z
    q = Z.T @ (H2 @ xp + qp["c"])
    Gi, l, h = A[~eq] @ Z, lo[~eq] - A[~eq] @ xp, hi[~eq] - A[~eq] @ xp
    keep = np.abs(Gi).sum(axis=1) > 1e-12
    Gi, l, h = Gi[keep], l[keep], h[keep]
    N = np.vstack([Gi, -Gi])
    b = np.concatenate([h, -l])
    fin = np.isfinite(b) & (np.abs(b) < 1e19)
    return P, q, N[fin], b[fin]


def gi(P, q, N, b, rule, tol=1e-6, maxstep=64):
    Pi = np.linalg.inv(P)
    y = -Pi @ q
    sc = 1.0 / (1.0 + np.abs(b))
    if rule == "diag":
        nrm = np.sqrt((N * N) @ np.diag(Pi))
    elif rule == "euclid":
        nrm = np.linalg.norm(N, axis=1)
    else:
        nrm = np.sqrt(np.einsum("ij,jk,ik->i", N, Pi, N))
    A, u = [], []
    steps = 0
    while True:
        v = (N @ y - b)
        m = (v * sc).max()
        if m <= 0.1 * tol:
            return steps, len(A), y
        if rule == "scaled":
            sel = v * sc
        elif rule.startswith("pow"):  # v / |g|^e, e = the digits / 100 (pow150: 1.5)
            sel = v / nrm ** (int(rule[3:]) / 100.0)
        else:
            sel = v / nrm**2 if rule == "normal2" else v / nrm
        p = int(np.argmax(np.where(v * sc > 0.1 * tol, sel, -np.inf)))
        up = 0.0
        while True:
            steps += 1
            if steps > maxstep:
                return -1, len(A), y
            npv = N[p]
            if A:
                NA = N[A]
                K = NA @ Pi @ NA.T
                rho = np.linalg.solve(K, NA @ Pi @ npv)
                z = Pi @ (npv - NA.T @ rho)
            else:
                rho = np.zeros(0)
                z = Pi @ npv
            zn = npv @ z
            blk = [(u[i] / rho[i], i) for i in range(len(A)) if rho[i] > 0]
            t1, l = min(blk) if blk else (np.inf, -1)
            t2 = (npv @ y - b[p]) / zn if zn > 1e-10 * (npv @ Pi @ npv) else np.inf
            if l < 0 and not np.isfinite(t2):
                return 1000 + steps, len(A), y  # infeasible (1000 + steps)
            t = min(t1, t2)
            if np.isfinite(t2):
                y = y - t * z
            u = [u[i] - t * rho[i] for i in range(len(A))]
            up += t
            if t2 <= t1:
                A.append(p)
                u.append(up)
                break
            del A[l]
            del u[l]


def main():
    fov = "--fov" in sys.argv
    it1 = "--it1" in sys.argv
    slack = "--slack" in sys.argv
    av = [a for a in sys.argv[1:] if not a.startswith("--")]
    d = np.load(av[0])
    min_steps = int(av[1]) if len(av) > 1 else 4
    sample = int(av[2]) if len(av) > 2 else 0
    traj, warm = d["traj"], int(d["warmup"])
    iters = d["iters"]
    n = traj.shape[0]
    if fov:
        over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if slack else {}
        cfg = swarm.fov_config(20, **over)
        _, targets = swarm.heading_swarm(n)
    else:
        cfg = swarm.config(15)
        _, targets = swarm.lattice_swarm(n)
    p = O.make_params(cfg)
    refs = swarm.refs_from_targets(targets, cfg["k_hor"])
    rng = np.random.default_rng(0)
    tot = {r: [] for r in (os.environ.get("DAS_RULES") or "scaled,normal,normal2,diag,euclid").split(",")}
    for s in range(iters.shape[0]):
        ags = list(np.where(iters[s, :, 1 if it1 else 0] >= min_steps)[0])
        if sample:
            more = np.where((iters[s, :, 0] > 0) & (iters[s, :, 0] < min_steps))[0]
            ags += list(rng.choice(more, min(sample, len(more)), replace=False)) if len(more) else []
        if not ags:
            continue
        states = traj[:, warm + s, :]
        if fov:
            rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
        else:
            rp, col = swarm.knn_csr(states, 8, 3.0 * cfg["d_min"])
        for a in ags:
            nb = col[rp[a]:rp[a + 1]]
            qp = O.assemble_qp(p, states[a], refs[a], states[nb], it=0)
            if it1:  # IMPC iteration 1: CBF rows at the iteration-0 curve's h_samples(k)
                r0 = O.impc_optimize(p, states, a, nb, refs[a])
                if r0["status"][0] != O.OPTIMAL:
                    continue
                x0 = r0["x"][0][:qp["n"]]
                pred = np.array([np.concatenate([O.eval_curve(p, x0, k * cfg["h"], 0),
                                                 O.eval_curve(p, x0, k * cfg["h"], 1)])
                                 for k in range(cfg["cbf_horizon"])])
                qp = O.assemble_qp(p, states[a], refs[a], states[nb], it=1, pred=pred)
            P, q, N, b = reduce_qp(qp)
            res = {rule: gi(P, q, N, b, rule) for rule in tot}
            for rule in tot:
                tot[rule].append(res[rule][0])
            print(f"step {s} agent {a}: gpu {iters[s, a, 1 if it1 else 0]}  " +
                  "  ".join(f"{k} {v[0]} (k={v[1]})" for k, v in res.items()))
    for rule, v in tot.items():
        v = np.array(v)
        f, inf = v[(v >= 0) & (v < 1000)], v[v >= 1000] - 1000
        print(rule, "feasible: n", len(f), "mean", f.mean() if len(f) else 0, "max", f.max() if len(f) else 0,
              "| infeasible: n", len(inf), "mean", inf.mean() if len(inf) else 0, "max", inf.max() if len(inf) else 0,
              "| gave up", int((v == -1).sum()))


if __name__ == "__main__":
    main()
