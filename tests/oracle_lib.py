"""ctypes binding of oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference hot path (see oracle/oracle.h). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

OPTIMAL, FEASIBLE, UNBOUNDED, INFEASIBLE, ERROR, UNKNOWN, INFEASIBLEORUNBOUNDED = range(7)
STATUS_NAMES = ["OPTIMAL", "FEASIBLE", "UNBOUNDED", "INFEASIBLE", "ERROR", "UNKNOWN",
                "INFEASIBLEORUNBOUNDED"]


class OrcParams(C.Structure):
    _fields_ = [
        ("h", C.c_double), ("Ts", C.c_double), ("k_hor", C.c_int32),
        ("w_pos_err", C.c_double), ("w_u_eff", C.c_double), ("spd_f", C.c_int32),
        ("v_min", C.c_double * 3), ("v_max", C.c_double * 3),
        ("a_min", C.c_double * 3), ("a_max", C.c_double * 3),
        ("d_min", C.c_double),
        ("cbf_horizon", C.c_int32), ("impc_iter", C.c_int32), ("slack_mode", C.c_int32),
        ("slack_cost", C.c_double), ("slack_decay_rate", C.c_double),
        ("num_pieces", C.c_int32), ("num_control_points", C.c_int32),
        ("piece_max_parameter", C.c_double), ("continuity_upto_degree", C.c_int32),
        ("cbf_mode", C.c_int32), ("fov_beta", C.c_double), ("fov_Ds", C.c_double),
        ("fov_Rs", C.c_double), ("bbox", C.c_double * 3),
    ]


def make_params(cfg: dict) -> OrcParams:
    p = OrcParams()
    for k, v in cfg.items():
        if isinstance(v, (list, tuple)):
            arr = getattr(p, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(p, k, v)
    return p


def build(quiet: bool = True) -> str:
    """Compile the oracle (plain g++)."""
    out = subprocess.run(["make", "-C", ORACLE_DIR], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    return ORACLE_SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = C.CDLL(ORACLE_SO)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int32)
        L.orc_fac.restype = C.c_uint64
        L.orc_fac.argtypes = [C.c_uint64]
        L.orc_comb.restype = C.c_uint64
        L.orc_comb.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_perm.restype = C.c_uint64
        L.orc_perm.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_bernstein_basis.argtypes = [C.c_uint64, C.c_double, C.c_double, C.c_uint64, dp]
        L.orc_bernstein_coefficient_matrix.argtypes = [C.c_uint64, C.c_double, C.c_uint64, dp]
        L.orc_safety_cbf.argtypes = [dp, dp, C.c_double, dp, dp]
        L.orc_apply_input.argtypes = [C.c_double, dp, dp, dp]
        L.orc_fov_cbf.argtypes = [dp, dp, C.c_double, C.c_double, C.c_double, dp, dp, ip]
        L.orc_prediction_matrices.argtypes = [C.c_double, C.c_int32, dp, dp]
        L.orc_fov_control_slack.argtypes = [C.c_double, C.c_double, C.c_double, dp, dp, dp, dp,
                                            dp, dp, C.c_int32, dp, C.c_int32, C.c_double,
                                            C.c_double, dp, dp, dp]
        L.orc_lambda2.argtypes = [C.c_int32, dp, C.c_double, dp, dp]
        L.orc_lambda2.restype = None
        L.orc_conn_cbf.argtypes = [C.c_int32, dp, C.c_int32, dp, C.c_double, C.c_double, dp, dp, dp]
        L.orc_conn_cbf.restype = None
        L.orc_clf_cbf.argtypes = [dp, dp, dp, dp]
        L.orc_clf_cbf.restype = None
        L.orc_connectivity_control.argtypes = [C.c_double, C.c_double, dp, dp, C.c_int32, C.c_double,
                                               C.c_double, C.c_int32, dp, C.c_int32, dp, dp, dp, dp]
        L.orc_fov_control.argtypes = [C.c_double, C.c_double, C.c_double, dp, dp, dp, dp, dp, dp,
                                      C.c_int32, dp, dp, dp]
        L.orc_num_vars.argtypes = [C.POINTER(OrcParams), C.c_int32]
        L.orc_assemble_qp.argtypes = [C.POINTER(OrcParams), dp, dp, C.c_int32, dp, dp, C.c_int32,
                                      dp, C.c_int32, dp, dp, dp, dp, dp, dp, dp, dp]
        L.orc_solve_dense_qp.argtypes = [C.c_int32, dp, dp, C.c_double, C.c_int32, dp, dp, dp, dp,
                                         dp, dp, dp, ip, dp]
        L.orc_impc_optimize.argtypes = [C.POINTER(OrcParams), C.c_int32, dp, C.c_int32, C.c_int32,
                                        ip, dp, ip, dp, dp, ip]
        L.orc_impc_optimize_cov.argtypes = [C.POINTER(OrcParams), C.c_int32, dp, C.c_int32,
                                            C.c_int32, ip, dp, dp, ip, dp, dp, ip]
        L.orc_distance_to_ellipse.restype = C.c_double
        L.orc_distance_to_ellipse.argtypes = [dp, dp, dp]
        L.orc_voronoi.argtypes = [dp, dp, dp, dp, dp]
        L.orc_impc_batch.restype = C.c_int64
        L.orc_impc_batch.argtypes = [C.POINTER(OrcParams), C.c_int32, dp, dp, ip, ip, C.c_int32,
                                     C.c_int32, C.c_int32, ip, dp, dp, dp]
        L.orc_eval_curve.argtypes = [C.POINTER(OrcParams), dp, C.c_double, C.c_int32, dp]
        _lib = L
    return _lib


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    return np.ascontiguousarray(a, dtype=np.int32).ctypes.data_as(C.POINTER(C.c_int32))


def bernstein_basis(deg, T, t, d):
    out = np.zeros(deg + 1)
    rc = lib().orc_bernstein_basis(deg, T, t, d, _d(out))
    if rc != 0:
        raise ValueError("parameter out of range")
    return out


def safety_cbf(state, nb, d_min):
    a = np.zeros(3)
    b = np.zeros(1)
    st = np.ascontiguousarray(state, dtype=np.float64)
    nbv = np.ascontiguousarray(nb, dtype=np.float64)
    lib().orc_safety_cbf(_d(st), _d(nbv), d_min, _d(a), _d(b))
    return a, float(b[0])


def apply_input(ts, state, u):
    out = np.zeros(6)
    st = np.ascontiguousarray(state, dtype=np.float64)
    uu = np.ascontiguousarray(u, dtype=np.float64)
    lib().orc_apply_input(ts, _d(st), _d(uu), _d(out))
    return out


def prediction_matrices(ts, K):
    A0 = np.zeros((3 * K, 6))
    Lm = np.zeros((3 * K, 3 * K))
    lib().orc_prediction_matrices(ts, K, _d(A0), _d(Lm))
    return A0, Lm


def assemble_qp(p: OrcParams, state, ref, neighbors, it=0, pred=None, slack_w=None,
                max_rows=4096):
    nb = 0 if neighbors is None else len(neighbors)
    n = lib().orc_num_vars(C.byref(p), nb)
    H = np.zeros((n, n))
    c = np.zeros(n)
    c0 = np.zeros(1)
    A = np.zeros((max_rows, n))
    lo = np.zeros(max_rows)
    hi = np.zeros(max_rows)
    vlo = np.zeros(n)
    vhi = np.zeros(n)
    nbs = np.ascontiguousarray(neighbors if nb else np.zeros((1, 6)), dtype=np.float64)
    pr = np.ascontiguousarray(pred if pred is not None else np.zeros((max(1, p.cbf_horizon), 6)),
                              dtype=np.float64)
    st = np.ascontiguousarray(state, dtype=np.float64)
    rf = np.ascontiguousarray(ref, dtype=np.float64)
    sw = None if slack_w is None else np.ascontiguousarray(slack_w, dtype=np.float64)
    m = lib().orc_assemble_qp(C.byref(p), _d(st), _d(rf), nb, _d(nbs),
                              None if sw is None else _d(sw), it, _d(pr), max_rows, _d(H), _d(c),
                              _d(c0), _d(A), _d(lo), _d(hi), _d(vlo), _d(vhi))
    if m < 0:
        raise RuntimeError(f"assemble failed: {m}")
    return dict(n=n, H=H, c=c, c0=float(c0[0]), A=A[:m].copy(), lo=lo[:m].copy(),
                hi=hi[:m].copy(), vlo=vlo, vhi=vhi)


def solve_dense_qp(qp):
    n = qp["n"]
    m = len(qp["lo"])
    x = np.zeros(n)
    obj = np.zeros(1)
    iters = np.zeros(1, dtype=np.int32)
    kkt = np.zeros(4)
    H = np.ascontiguousarray(qp["H"], dtype=np.float64)
    c = np.ascontiguousarray(qp["c"], dtype=np.float64)
    A = np.ascontiguousarray(qp["A"], dtype=np.float64).reshape(m, n) if m else np.zeros((1, n))
    lo = np.ascontiguousarray(qp["lo"] if m else np.zeros(1), dtype=np.float64)
    hi = np.ascontiguousarray(qp["hi"] if m else np.zeros(1), dtype=np.float64)
    vlo = np.ascontiguousarray(qp["vlo"], dtype=np.float64)
    vhi = np.ascontiguousarray(qp["vhi"], dtype=np.float64)
    st = lib().orc_solve_dense_qp(n, _d(H), _d(c), qp.get("c0", 0.0), m, _d(A), _d(lo), _d(hi),
                                  _d(vlo), _d(vhi), _d(x), _d(obj),
                                  iters.ctypes.data_as(C.POINTER(C.c_int32)), _d(kkt))
    return dict(status=st, x=x, obj=float(obj[0]), iters=int(iters[0]), kkt=kkt)


def distance_to_ellipse(robot, mean, cov3):
    """FovBezierIMPCCBF::distanceToEllipse; cov3 = (cxx, cxy, cyy)."""
    return lib().orc_distance_to_ellipse(_d(robot), _d(mean), _d(cov3))


def voronoi(self_xy, other_xy, bbox=(0.0, 0.0, 0.0)):
    """(normal (3), offset) of the Voronoi hyperplane of two planar points, box-shifted."""
    n = np.zeros(3)
    off = np.zeros(1)
    lib().orc_voronoi(_d(np.asarray(self_xy, dtype=np.float64)), _d(np.asarray(other_xy, dtype=np.float64)),
                      _d(np.asarray(bbox, dtype=np.float64)), _d(n), _d(off))
    return n, float(off[0])


def impc_optimize(p: OrcParams, states, self_idx, neighbor_idx, ref, covs=None):
    """One agent's IMPC optimize; covs (num_states x 3: cxx, cxy, cyy) feeds the FoV slack
    weights (FovBezierIMPCCBF.cpp:58-81), None = unknown covariances."""
    states = np.ascontiguousarray(states, dtype=np.float64)
    nbi = np.ascontiguousarray(neighbor_idx, dtype=np.int32)
    nb = len(nbi)
    n = lib().orc_num_vars(C.byref(p), nb)
    it_n = p.impc_iter
    status = np.full(it_n, UNKNOWN, dtype=np.int32)
    obj = np.full(it_n, np.nan)
    x = np.zeros((it_n, n))
    qi = np.zeros(it_n, dtype=np.int32)
    rf = np.ascontiguousarray(ref, dtype=np.float64)
    cv = None if covs is None else np.ascontiguousarray(covs, dtype=np.float64)
    att = lib().orc_impc_optimize_cov(C.byref(p), len(states), _d(states), self_idx, nb,
                                      nbi.ctypes.data_as(C.POINTER(C.c_int32)) if nb else None,
                                      _d(rf), None if cv is None else _d(cv),
                                      status.ctypes.data_as(C.POINTER(C.c_int32)), _d(obj),
                                      _d(x), qi.ctypes.data_as(C.POINTER(C.c_int32)))
    if att < 0:
        raise RuntimeError("orc_impc_optimize failed")
    return dict(attempted=att, status=status, obj=obj, x=x, qp_iters=qi)


def impc_batch(p: OrcParams, states, refs, row_ptr, col, first, count, nthreads=1, covs=None):
    states = np.ascontiguousarray(states, dtype=np.float64)
    cv = None if covs is None else np.ascontiguousarray(covs, dtype=np.float64)
    refs = np.ascontiguousarray(refs, dtype=np.float64)
    rp = np.ascontiguousarray(row_ptr, dtype=np.int32)
    cl = np.ascontiguousarray(col if len(col) else np.zeros(1), dtype=np.int32)
    it_n = p.impc_iter
    status = np.full((count, it_n), UNKNOWN, dtype=np.int32)
    obj = np.full((count, it_n), np.nan)
    nc = p.num_pieces * 3 * p.num_control_points
    xl = np.zeros((count, nc))
    solved = lib().orc_impc_batch(C.byref(p), len(states), _d(states), _d(refs),
                                  rp.ctypes.data_as(C.POINTER(C.c_int32)),
                                  cl.ctypes.data_as(C.POINTER(C.c_int32)), first, count, nthreads,
                                  status.ctypes.data_as(C.POINTER(C.c_int32)), _d(obj), _d(xl),
                                  None if cv is None else _d(cv))
    return dict(solved=int(solved), status=status, obj=obj, x_last=xl)


def fov_cbf(state, target, fov, Ds, Rs):
    """FovCBF rows (safety, left border, right border, range): (a (4, 3), b (4,), present (4,))."""
    st = np.ascontiguousarray(state, dtype=np.float64)
    tg = np.ascontiguousarray(target, dtype=np.float64)
    a = np.zeros(12)
    b = np.zeros(4)
    pr = np.zeros(4, dtype=np.int32)
    lib().orc_fov_cbf(_d(st), _d(tg), fov, Ds, Rs, _d(a), _d(b), pr.ctypes.data_as(C.POINTER(C.c_int32)))
    return a.reshape(4, 3), b, pr


def fov_control(cfg: dict, state, desired_u, nb_xy, nb_cov=None):
    """FovControl::optimize restated: (status, u (3,), objective incl. constant and, in slack
    mode (cfg control_slack_mode / slack_cost / slack_decay_rate), the slack cost). nb_cov: per-neighbour
    (cxx, cxy, cyy) for the slack weights, None = unknown."""
    f = lambda v: np.ascontiguousarray(v, dtype=np.float64)  # noqa: E731
    umin = cfg.get("u_min", cfg["a_min"])
    umax = cfg.get("u_max", cfg["a_max"])
    nb = np.ascontiguousarray(np.reshape(nb_xy, (-1, 2)), dtype=np.float64)
    u = np.zeros(3)
    obj = np.zeros(1)
    vmin, vmax, umin, umax, st, ud = (f(cfg["v_min"]), f(cfg["v_max"]), f(umin), f(umax), f(state),
                                      f(desired_u))
    cv = None if nb_cov is None else np.ascontiguousarray(np.reshape(nb_cov, (-1, 3)), dtype=np.float64)
    stt = lib().orc_fov_control_slack(cfg["fov_beta"], cfg["fov_Ds"], cfg["fov_Rs"], _d(vmin),
                                      _d(vmax), _d(umin), _d(umax), _d(st), _d(ud), len(nb),
                                      _d(nb) if len(nb) else None, int(cfg.get("control_slack_mode", 0)),
                                      float(cfg.get("slack_cost", 0.0)),
                                      float(cfg.get("slack_decay_rate", 1.0)),
                                      None if cv is None or not len(cv) else _d(cv), _d(u), _d(obj))
    return stt, u, float(obj[0])


def eval_curve(p: OrcParams, x, t, d):
    out = np.zeros(3)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    rc = lib().orc_eval_curve(C.byref(p), _d(xx), t, d, _d(out))
    if rc != 0:
        raise ValueError("eval out of range")
    return out


def lambda2(pos2, dmax):
    """ConnectivityCBF::getLambda2: (lambda2, unit Fiedler vector)."""
    pos = np.ascontiguousarray(np.reshape(pos2, (-1, 2)), dtype=np.float64)
    l2 = np.zeros(1)
    v = np.zeros(len(pos))
    lib().orc_lambda2(len(pos), _d(pos), float(dmax), _d(l2), _d(v))
    return float(l2[0]), v


def conn_cbf(states, self_idx, eigvec, l2, dmax):
    """Connectivity CBF row of robot self_idx: (Ac (3,), Bc, [gx, gy, Hxx, Hxy, Hyy, Lfh, Lf2h])."""
    st = np.ascontiguousarray(states, dtype=np.float64)
    a = np.zeros(3)
    b = np.zeros(1)
    dbg = np.zeros(7)
    lib().orc_conn_cbf(len(st), _d(st), int(self_idx), _d(eigvec), float(l2), float(dmax), _d(a),
                       _d(b), _d(dbg))
    return a, float(b[0]), dbg


def clf_cbf(state, neighbor):
    a = np.zeros(3)
    b = np.zeros(1)
    lib().orc_clf_cbf(_d(state), _d(neighbor), _d(a), _d(b))
    return a, float(b[0])


def connectivity_control(cfg: dict, states, self_idx, desired_u):
    """ConnectivityControl::optimize restated: (status, u (3,), objective, lambda2). cfg keys:
    d_min, d_max, v_min, v_max, control_slack_mode, slack_cost, slack_decay_rate."""
    st = np.ascontiguousarray(states, dtype=np.float64)
    u = np.zeros(3)
    obj = np.zeros(1)
    l2 = np.zeros(1)
    f = lambda v: np.ascontiguousarray(v, dtype=np.float64)  # noqa: E731
    stt = lib().orc_connectivity_control(
        float(cfg["d_min"]), float(cfg["d_max"]), _d(f(cfg["v_min"])), _d(f(cfg["v_max"])),
        int(cfg.get("control_slack_mode", 0)), float(cfg.get("slack_cost", 0.0)),
        float(cfg.get("slack_decay_rate", 1.0)), len(st), _d(st), int(self_idx), _d(f(desired_u)),
        _d(u), _d(obj), _d(l2))
    return stt, u, float(obj[0]), float(l2[0])


# ---- closed loop in the reference example's order (test infrastructure) -----------------------
_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def normal_sample(seed: int, step: int, agent: int, comp: int, sub: int = 0) -> float:
    """The counter-based state noise of the product (impc_common.hpp normal_sample: splitmix64 keyed
    by (seed, step, agent, component, sub-step) + Box-Muller), in place of math::addRandomNoise's
    std::mt19937 seeded from std::random_device (Random.cpp:7-28), which no two runs share."""
    k = _mix64(seed & _M64)
    k = _mix64(k ^ (step & _M64))
    k = _mix64(k ^ ((agent * 8 + comp) & _M64))
    if sub > 0:
        k = _mix64(k ^ ((sub << 40) & _M64))
    u1 = float((k >> 11) + 1) * 2.0 ** -53
    u2 = float(_mix64(k) >> 11) * 2.0 ** -53
    return float(np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2))


def knn_list(states, i, k, radius):
    """Agent i's k nearest others (planar) within radius, ties by index, sorted by index (the
    device grid query's rule, mpccbf.swarm.knn_csr for one agent)."""
    p = states[:, :2]
    d2 = np.sum((p - p[i]) ** 2, axis=1)
    d2[i] = np.inf
    cand = np.nonzero(d2 <= radius * radius)[0]
    order = np.lexsort((cand, d2[cand]))[:k]
    return np.sort(cand[order]).astype(np.int32)


def closed_loop_gauss_seidel(cfg: dict, states, targets, steps, k=8, radius=6.0, pos_std=0.0, vel_std=0.0,
                             seed=0, neighbours="knn", inputs=None):
    """MPCCBFFormationControl_example.cpp:131-226 restated in its own order: per control step the
    robots in index order (:140), each optimize()d against the current table (robots before it
    already moved, :201), the kept curve (last successful trajectory, :150-165) evaluated int(h/Ts)
    sub-steps ahead with the noise (:188-207), or the position held at zero velocity (:208-221).
    Returns (trace: steps+1 x n x 6 states after each step, status: steps x n x impc_iter).
    inputs (a trace of another run, steps+1 x n x 6): robot i of step s plans from that run's table
    as it stood at its turn — robots < i at inputs[s+1], the others at inputs[s] — instead of this
    loop's own: every update checked on the same inputs, without the amplification a free-running
    comparison accumulates through the CBF rows (Bc is cubic in the distance margin)."""
    p = make_params(cfg)
    n = len(states)
    cur = np.array(states, dtype=np.float64)
    refs = np.tile(np.asarray(targets, dtype=np.float64), (1, cfg["k_hor"]))
    nsub = int(cfg["h"] / cfg["Ts"])
    eval_step = cfg["Ts"] * nsub
    tmax = cfg["num_pieces"] * cfg["piece_max_parameter"]
    xs = [None] * n
    traj_t = np.full(n, -1.0)
    trace = [cur.copy()]
    own = cur.copy()
    stats = []
    for s in range(steps):
        st = np.full((n, cfg["impc_iter"]), UNKNOWN, dtype=np.int32)
        for i in range(n):
            if inputs is not None:
                cur = np.concatenate([inputs[s + 1][:i], inputs[s][i:]]).astype(np.float64)
            nb = (np.array([j for j in range(n) if j != i], dtype=np.int32) if neighbours == "all"
                  else knn_list(cur, i, k, radius))
            r = impc_optimize(p, cur, i, nb, refs[i])
            st[i] = r["status"]
            ok = np.nonzero(r["status"] == OPTIMAL)[0]
            if len(ok):
                xs[i] = r["x"][ok[-1]].copy()
                traj_t[i] = 0.0
            nxt = np.zeros(6)
            if xs[i] is not None:
                t_new = min(traj_t[i] + eval_step, tmax)
                pos, vel = eval_curve(p, xs[i], t_new, 0), eval_curve(p, xs[i], t_new, 1)
                for c in range(6):
                    sd = pos_std if c < 3 else vel_std
                    v = pos[c] if c < 3 else vel[c - 3]
                    nxt[c] = v + sd * normal_sample(seed, s, i, c) if sd > 0.0 else v
                traj_t[i] = t_new
            else:
                for c in range(6):
                    sd = pos_std if c < 3 else vel_std
                    v = cur[i, c] if c < 3 else 0.0
                    for kk in range(1, nsub + 1):
                        dn = sd * normal_sample(seed, s, i, c, nsub - kk) if sd > 0.0 else 0.0
                        v = v + dn if c < 3 else dn
                    nxt[c] = v
            cur[i] = nxt
            if inputs is not None:
                own[i] = nxt
        if inputs is not None:
            trace.append(own.copy())
        else:
            trace.append(cur.copy())
        stats.append(st)
    return np.array(trace), np.array(stats)
