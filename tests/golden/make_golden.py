"""Golden QP fixtures: an independent numpy restatement of the reference assembly plus an
independent solve (scipy SLSQP, then an exact active-set KKT re-solve), written to
golden_qps.npz. The C oracle and the GPU path are both checked against these.

Restated (paths under workspace/lib of ywang760/mpc-cbf):
  model/src/DoubleIntegrator.cpp:9-51, DoubleIntegratorXYYaw.cpp:9-20   (A0, Lambda)
  splines/src/detail/BezierOperations.cpp:11-121                         (Bernstein basis)
  mpc/src/optimization/PiecewiseBezierMPCQPOperations.cpp:9-90,190-223   (U_basis, tracking cost)
  splines/src/optimization/BezierQPOperations.cpp:149-246                (eval/bound rows, effort cost)
  mpc/src/optimization/PiecewiseBezierMPCQPGenerator.cpp:148-321         (continuity, i<=j costs)
  cbf/src/detail/ConnectivityCBF.cpp:152-198 + ConnectivityMPCCBFQPOperations.cpp:192-272 (CBF rows)
  mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:102-197                 (per-iteration assembly)
Run:  python tests/golden/make_golden.py    (numpy + scipy; seconds)
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "mpc-cbf_amd"))
from mpccbf import swarm  # noqa: E402  (parameters + synthetic swarm only)

EPS100 = np.finfo(float).eps * 100.0
INF = np.finfo(float).max


def bernstein(deg, T, t, d):
    out = np.zeros(deg + 1)
    for i in range(deg + 1):
        acc = 0.0
        for j in range(deg + 1 - d):
            if j + d >= i:
                acc += (math.comb(deg - i, j + d - i) * (1.0 / T) ** (j + d) * math.perm(j + d, d)
                        * t ** j * (1 if (j + d - i) % 2 == 0 else -1))
        out[i] = acc * math.comb(deg, i)
    return out


def linspaced(K, high):
    if K == 1:
        return np.array([high])
    step = high / (K - 1)
    v = np.array([i * step for i in range(K)])
    v[-1] = high
    return v


def locate(cum, T, t):
    i = int(np.searchsorted(cum, t, side="left"))
    local = t if i == 0 else t - cum[i - 1]
    return i, min(max(local, 0.0), T)


def assemble(cfg, state, ref, nbs, it, pred):
    P, C, K, cont = cfg["num_pieces"], cfg["num_control_points"], cfg["k_hor"], \
        cfg["continuity_upto_degree"]
    T, h = cfg["piece_max_parameter"], cfg["h"]
    npc = 3 * C
    n = P * npc
    cum = np.cumsum([T] * P)
    hs = linspaced(K, (K - 1) * h)

    def row(t, dim, d):
        i, loc = locate(cum, T, t)
        r = np.zeros(n)
        r[i * npc + dim * C: i * npc + dim * C + C] = bernstein(C - 1, T, loc, d)
        return r

    U = np.array([row(hs[k], dim, 2) for k in range(K) for dim in range(3)])
    A = np.eye(6)
    A[:3, 3:] = h * np.eye(3)
    B = np.vstack([0.5 * h ** 2 * np.eye(3), h * np.eye(3)])
    A0 = np.zeros((3 * K, 6))
    Lam = np.zeros((3 * K, 3 * K))
    prev, prevL = np.eye(6), np.zeros((6, 3 * K))
    for k in range(K):
        prev = A @ prev
        addb = np.zeros((6, 3 * K))
        addb[:, 3 * k:3 * k + 3] = B
        prevL = A @ prevL + addb
        A0[3 * k:3 * k + 3] = prev[:3]
        Lam[3 * k:3 * k + 3] = prevL[:3]
    Q = np.zeros(3 * K)
    Q[3 * (K - cfg["spd_f"]):] = cfg["w_pos_err"]
    Phi = Lam @ U
    quad_pe = Phi.T @ (Q[:, None] * Phi)
    lin = (2.0 * (A0 @ state) * Q - 2.0 * ref * Q) @ Phi
    q = np.zeros((n, n))

    def add(term, off):
        m = term.shape[0]
        for i in range(m):
            for j in range(m):
                v = term[i, j]
                if abs(v) <= EPS100:
                    continue
                a, b = sorted((off + i, off + j))
                q[a, b] += v
    add(quad_pe, 0)
    c = np.where(np.abs(lin) <= EPS100, 0.0, lin)
    for d in range(1, cont + 1):
        if d > C - 1:
            continue
        # bernsteinCoefficientMatrix (monomial coefficients of the d-th derivative) * SQI * B^T
        Bm = np.zeros((C, C))
        for i in range(C):
            for j in range(i, C):
                Bm[i, j] = math.comb(C - 1, i) * math.comb(C - 1 - i, j - i) * (-1) ** (j - i) / T ** j
        Der = np.zeros((C, C))
        for j in range(d, C):
            Der[j, j - d] = math.perm(j, d)
        Bd = Bm @ Der
        SQI = np.array([[T ** (i + j + 1) / (i + j + 1) for j in range(C)] for i in range(C)])
        cost = cfg["w_u_eff"] * Bd @ SQI @ Bd.T
        blk = np.kron(np.eye(3), cost)
        for pc in range(P):
            add(blk, pc * npc)
    H = np.triu(q, 1) * 0.5
    H = H + H.T + np.diag(np.diag(q))
    rows, lo, hi = [], [], []
    for d in (0, 1):
        for dim in range(3):
            rows.append(row(0.0, dim, d))
            lo.append(state[3 * d + dim])
            hi.append(state[3 * d + dim])
    for pc in range(P - 1):
        for d in range(cont + 1):
            for dim in range(3):
                r = np.zeros(n)
                r[pc * npc + dim * C: pc * npc + dim * C + C] = bernstein(C - 1, T, T, d)
                r[(pc + 1) * npc + dim * C:(pc + 1) * npc + dim * C + C] = -bernstein(C - 1, T, 0.0, d)
                rows.append(r)
                lo.append(0.0)
                hi.append(0.0)
    gamma, dmin = 5.0, cfg["d_min"]

    def cbf(e, nb):
        dx, dy, dvx, dvy = e[0] - nb[0], e[1] - nb[1], e[3] - nb[3], e[4] - nb[4]
        hh = dx * dx + dy * dy - dmin ** 2
        lf_alpha = 3 * gamma * hh ** 2 * (2 * dx * e[3] + 2 * dy * e[4])
        b = 2 * (dvx ** 2 + dvy ** 2) + lf_alpha + gamma * (2 * (dx * dvx + dy * dvy) + gamma * hh ** 3) ** 3
        return np.array([2 * dx, 2 * dy, 0.0]), b
    egos = [(state, 0)] if it == 0 else [(pred[k], k) for k in range(cfg["cbf_horizon"])]
    for nb in nbs:
        for e, k in egos:
            a, b = cbf(e, nb)
            rows.append(-(a @ U[3 * k:3 * k + 3]))
            lo.append(-INF)
            hi.append(b)
    for deriv, lb, ub in ((2, cfg["a_min"], cfg["a_max"]), (1, cfg["v_min"], cfg["v_max"])):
        for k in range(K):
            for dim in range(3):
                rows.append(row(hs[k], dim, deriv))
                lo.append(lb[dim])
                hi.append(ub[dim])
    return H, c, np.array(rows), np.array(lo), np.array(hi)


def solve(H, c, A, lo, hi):
    """Independent solve: scipy SLSQP from a feasible-ish start, then an exact KKT re-solve on
    the detected active set (x* and multipliers); returns x, obj, max KKT residual."""
    from scipy.optimize import minimize
    n = len(c)
    eq = lo == hi
    fin_lo = (lo > -1e300) & ~eq
    fin_hi = (hi < 1e300) & ~eq
    cons = [{"type": "eq", "fun": lambda x, A=A[eq], b=lo[eq]: A @ x - b, "jac": lambda x, A=A[eq]: A}]
    if fin_lo.any():
        cons.append({"type": "ineq", "fun": lambda x, A=A[fin_lo], b=lo[fin_lo]: A @ x - b,
                     "jac": lambda x, A=A[fin_lo]: A})
    if fin_hi.any():
        cons.append({"type": "ineq", "fun": lambda x, A=A[fin_hi], b=hi[fin_hi]: b - A @ x,
                     "jac": lambda x, A=A[fin_hi]: -A})
    x0 = np.linalg.lstsq(A[eq], lo[eq], rcond=None)[0]
    res = minimize(lambda x: x @ H @ x + c @ x, x0, jac=lambda x: 2 * H @ x + c, method="SLSQP",
                   constraints=cons, options={"ftol": 1e-15, "maxiter": 1000})
    x = res.x
    # exact active-set re-solve
    act = [i for i in range(len(lo)) if eq[i] or (fin_lo[i] and abs(A[i] @ x - lo[i]) < 1e-7)
           or (fin_hi[i] and abs(A[i] @ x - hi[i]) < 1e-7)]
    bnd = np.array([lo[i] if (eq[i] or (fin_lo[i] and abs(A[i] @ x - lo[i]) < 1e-7)) else hi[i]
                    for i in act])
    Aa = A[act]
    KKT = np.block([[2 * H, Aa.T], [Aa, np.zeros((len(act), len(act)))]])
    sol = np.linalg.lstsq(KKT, np.concatenate([-c, bnd]), rcond=None)[0]
    xe = sol[:n]
    viol = max(np.max(lo - A @ xe, initial=0), np.max(A @ xe - hi, initial=0))
    if viol < 1e-9:
        x = xe
    return x, float(x @ H @ x + c @ x), res.success


def main():
    cases = []
    for K, nag, spacing_scale, seed in ((10, 6, 1.0, 1), (15, 6, 1.0, 2), (15, 9, 0.5, 3)):
        cfg = swarm.config(K)
        states, targets = swarm.lattice_swarm(nag, seed=seed)
        states[:, :2] *= spacing_scale
        refs = swarm.refs_from_targets(targets, K)
        for a in range(nag):
            nbs = np.delete(states, a, axis=0)
            H, c, A, lo, hi = assemble(cfg, states[a], refs[a], nbs, 0, None)
            x, obj, ok = solve(H, c, A, lo, hi)
            cases.append(dict(K=K, it=0, state=states[a], ref=refs[a], nbs=nbs,
                              pred=np.zeros((cfg["cbf_horizon"], 6)), H=H, c=c, A=A, lo=lo, hi=hi,
                              x=x, obj=obj, ok=ok))
            # iteration 1 with predicted states from this solution's curve at h_samples(0..1)
            pred = np.zeros((cfg["cbf_horizon"], 6))
            C = cfg["num_control_points"]
            for k in range(cfg["cbf_horizon"]):
                t = k * cfg["h"]
                for d in (0, 1):
                    bb = bernstein(C - 1, cfg["piece_max_parameter"], t, d)
                    for dim in range(3):
                        pred[k, 3 * d + dim] = bb @ x[dim * C:dim * C + C]
            H, c, A, lo, hi = assemble(cfg, states[a], refs[a], nbs, 1, pred)
            x1, obj1, ok1 = solve(H, c, A, lo, hi)
            cases.append(dict(K=K, it=1, state=states[a], ref=refs[a], nbs=nbs, pred=pred, H=H, c=c,
                              A=A, lo=lo, hi=hi, x=x1, obj=obj1, ok=ok1))
    out = {}
    for i, cs in enumerate(cases):
        for k, v in cs.items():
            out[f"c{i}_{k}"] = np.asarray(v)
    out["count"] = np.array(len(cases))
    path = os.path.join(HERE, "golden_qps.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(cases), "cases; all SLSQP ok:", all(c["ok"] for c in cases))


if __name__ == "__main__":
    main()
