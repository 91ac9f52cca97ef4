"""ConnectivityControl::optimize (cbf/src/controller/ConnectivityControl.cpp:22-99): the CBF-only
controller with safety, velocity and connectivity rows — the lambda2 CBF when the team's
algebraic connectivity exceeds 0.1, the per-neighbour CLF rows otherwise.

CPU: the oracle restatement pinned by the reference's known-answer tests
(TestInitConnectivity.cpp:103-153 and the values that test run printed, results.log), LAPACK
eigenvalues and finite differences. GPU: the batched kernel (one team per wavefront: Laplacian
eigenproblem in LDS, one robot QP per 16-lane group) against the oracle."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def test_connectivity_cbf_known_answers(oracle):
    k = KATS["connectivity_cbf"]
    for case in k["cases"]:
        S = np.array(case["robot_states"], dtype=np.float64)
        l2, v = O.lambda2(S[:, :2], k["d_max"])
        a, b, dbg = O.conn_cbf(S, case["self"], v, l2, k["d_max"])
        np.testing.assert_allclose(a, case["Ac"], atol=k["tolerance_Ac"])
        assert abs(b - case["Bc"]) <= 4 * np.spacing(abs(case["Bc"])) + 1e-15, (b, case["Bc"])
        assert abs(l2 - case["log_lambda2"]) <= 1e-15
        np.testing.assert_allclose(dbg[:2], case["log_grad_h"], atol=1e-6)
        H = np.array([[dbg[2], dbg[3]], [dbg[3], dbg[4]]])
        np.testing.assert_allclose(H, case["log_hessian"], atol=1e-6)
        assert abs(dbg[5] - case["log_Lfh"]) <= 1e-14
        assert abs(dbg[6] - case["log_Lf2h"]) <= 1e-14


def _laplacian(pos, dmax):
    n = len(pos)
    sigma = dmax ** 4 / np.log(2.0)
    A = np.zeros((n, n))
    for i in range(n):
        for j in range(n):
            if i != j:
                d2 = np.sum((pos[i] - pos[j]) ** 2)
                if d2 <= dmax * dmax:
                    A[i, j] = np.exp((dmax * dmax - d2) ** 2 / sigma) - 1
    return np.diag(A.sum(axis=1)) - A


def test_lambda2_matches_lapack(oracle):
    rng = np.random.default_rng(3)
    for n in (2, 3, 5, 8, 13, 16):
        for _ in range(4):
            pos = rng.uniform(-2.5, 2.5, (n, 2))
            l2, v = O.lambda2(pos, 4.0)
            w, V = np.linalg.eigh(_laplacian(pos, 4.0))
            assert abs(l2 - w[1]) <= 1e-10 * max(1.0, abs(w[-1]))
            assert abs(abs(v @ V[:, 1]) - 1.0) <= 1e-8 or abs(w[2] - w[1]) < 1e-6


def test_clf_and_conn_rows_match_finite_differences(oracle):
    rng = np.random.default_rng(5)
    eps = 1e-6
    for _ in range(10):
        st = np.concatenate([rng.uniform(-3, 3, 2), [0.3], rng.uniform(-1, 1, 2), [0.1]])
        nb = np.concatenate([rng.uniform(-3, 3, 2), [0.0], rng.uniform(-1, 1, 2), [0.0]])
        a, b = O.clf_cbf(st, nb)
        V = lambda p: (np.linalg.norm(p - nb[:2]) - 2.0) ** 2  # noqa: E731
        grad = lambda p: np.array([(V(p + e) - V(p - e)) / (2 * eps) for e in np.eye(2) * eps])  # noqa: E731
        p = st[:2]
        np.testing.assert_allclose(a[:2], grad(p), rtol=1e-6, atol=1e-6)
        h2 = 1e-4
        H = np.array([(grad(p + e) - grad(p - e)) / (2 * h2) for e in np.eye(2) * h2])
        vel = st[3:5]
        want = vel @ H @ vel + 5 * (a[:2] @ vel) + 2 * V(p)
        assert abs(b - want) <= 1e-3 * max(1.0, abs(want))
    # connectivity row: the Hessian over the self position (Fiedler vector held fixed)
    for n in (3, 6):
        S = np.zeros((n, 6))
        S[:, :2] = rng.uniform(-2, 2, (n, 2))
        S[:, 3:5] = rng.uniform(-1, 1, (n, 2))
        l2, v = O.lambda2(S[:, :2], 4.0)
        _, _, d0 = O.conn_cbf(S, 0, v, l2, 4.0)
        for k, (gi, hrow) in enumerate([(0, (2, 3)), (1, (3, 4))]):
            Sp, Sm = S.copy(), S.copy()
            Sp[0, k] += 1e-6
            Sm[0, k] -= 1e-6
            dp = O.conn_cbf(Sp, 0, v, l2, 4.0)[2]
            dm = O.conn_cbf(Sm, 0, v, l2, 4.0)[2]
            fd = (dp[:2] - dm[:2]) / 2e-6
            np.testing.assert_allclose(fd, [d0[hrow[0]], d0[hrow[1]]], rtol=1e-5, atol=1e-6)


def _team(n, seed, spread):
    rng = np.random.default_rng(seed)
    S = np.zeros((n, 6))
    S[:, :2] = rng.uniform(-spread, spread, (n, 2))
    S[:, 2] = rng.uniform(-0.5, 0.5, n)
    S[:, 3:5] = rng.uniform(-0.8, 0.8, (n, 2))
    targets = rng.uniform(-3, 3, (n, 3))
    ud = 0.5 * (targets - S[:, :3]) - 2 * np.sqrt(0.5) * S[:, 3:6]  # criticallyDampedSpringControl
    return S, ud


def _cfg(slack=False):
    c = dict(d_min=0.8, d_max=3.0, v_min=[-1.0, -1.0, -2.6179938779914944],
             v_max=[1.0, 1.0, 2.6179938779914944])
    if slack:
        c.update(control_slack_mode=1, slack_cost=1e5, slack_decay_rate=0.1)
    return c


def test_oracle_connectivity_control_branches(oracle):
    """Tight teams take the lambda2 row, spread-out ones the CLF rows; slack mode always solves."""
    seen = set()
    for seed, spread in [(1, 1.0), (2, 1.2), (3, 4.0), (4, 6.0)]:
        S, ud = _team(6, seed, spread)
        for i in range(6):
            st, u, obj, l2 = O.connectivity_control(_cfg(), S, i, ud[i])
            seen.add(l2 > 0.1)
            st2, u2, obj2, _ = O.connectivity_control(_cfg(True), S, i, ud[i])
            assert st2 == O.OPTIMAL
            if st == O.OPTIMAL:
                assert obj2 <= obj + 1e-6 * max(1.0, abs(obj))
    assert seen == {True, False}


def _teams(sizes, seed):
    """Teams of the given sizes, alternating tight (lambda2 row) and spread-out (CLF rows)."""
    S_all, U_all, ptr = [], [], [0]
    for t, n in enumerate(sizes):
        S, ud = _team(n, seed + t, 1.0 if t % 2 == 0 else 5.0)
        S_all.append(S)
        U_all.append(ud)
        ptr.append(ptr[-1] + n)
    return np.vstack(S_all), np.vstack(U_all), np.array(ptr, dtype=np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("slack", [False, True])
def test_gpu_connectivity_control_matches_oracle(mpclib, slack):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a visible MI355X")
    sizes = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 6, 6, 6, 3, 16]
    S, ud, ptr = _teams(sizes, 11)
    cfg = _cfg(slack)
    dev = torch.device("cuda", 0)
    t = lambda v, dt=torch.float64: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    R = len(S)
    u = torch.empty((R, 3), dtype=torch.float64, device=dev)
    status = torch.empty(R, dtype=torch.int32, device=dev)
    obj = torch.empty(R, dtype=torch.float64, device=dev)
    l2 = torch.empty(len(sizes), dtype=torch.float64, device=dev)
    mpclib.connectivity_control_solve(cfg, t(ptr, torch.int32), t(S), t(ud), u, status=status, obj=obj,
                                      lambda2=l2)
    torch.cuda.synchronize()
    u, status, obj, l2 = u.cpu().numpy(), status.cpu().numpy(), obj.cpu().numpy(), l2.cpu().numpy()
    branches = set()
    n_opt = 0
    for k in range(len(sizes)):
        Sk = S[ptr[k]:ptr[k + 1]]
        lref, _ = O.lambda2(Sk[:, :2], cfg["d_max"])
        assert abs(l2[k] - lref) <= 1e-10 * max(1.0, abs(lref)), (k, l2[k], lref)
        branches.add(lref > 0.1)
        for i in range(len(Sk)):
            r = ptr[k] + i
            st, ur, objr, _ = O.connectivity_control(cfg, Sk, i, ud[r])
            assert status[r] == st, (k, i, status[r], st)
            if st == O.OPTIMAL:
                n_opt += 1
                np.testing.assert_allclose(u[r], ur, atol=1e-5, rtol=1e-5)
                assert abs(obj[r] - objr) <= 1e-4 * max(1.0, abs(objr)), (k, i, obj[r], objr)
    assert branches == {True, False}
    assert n_opt >= 20  # the rest: safety rows against close, fast neighbours are infeasible
    if slack:
        assert np.all(status == O.OPTIMAL)


@pytest.mark.gpu
def test_gpu_connectivity_control_team_too_large(mpclib):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a visible MI355X")
    S, ud, ptr = _teams([17, 3], 2)
    dev = torch.device("cuda", 0)
    t = lambda v, dt=torch.float64: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    u = torch.empty((len(S), 3), dtype=torch.float64, device=dev)
    status = torch.empty(len(S), dtype=torch.int32, device=dev)
    mpclib.connectivity_control_solve(_cfg(), t(ptr, torch.int32), t(S), t(ud), u, status=status)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert np.all(st[:17] == O.ERROR) and np.all(st[17:] != O.ERROR)
