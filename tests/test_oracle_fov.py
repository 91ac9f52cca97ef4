"""CPU: the oracle's FoV controller restatement (BASELINE config 5, FovBezierIMPCCBF).

FoV CBF rows against an independent 40-digit symbolic derivation (tests/golden/fov_cbf_golden.json,
make_fov_golden.py — the reference has no known-answer tests for these rows), and the assembled
QP's structure against FovBezierIMPCCBF.cpp:96-217: continuity d < degree, Voronoi rows on the
piece-0 control points, 4 FoV rows per neighbour (per predicted state in iteration 1).
"""
import json
import math
import os

import numpy as np

import oracle_lib as O
from mpccbf import swarm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fov_cbf_golden.json")


def test_fov_rows_match_symbolic_derivation(oracle):
    g = json.load(open(GOLDEN))
    assert len(g["cases"]) == 24
    for case in g["cases"]:
        a, b, present = O.fov_cbf(case["state"], case["target"], case["fov"], case["Ds"], case["Rs"])
        for r, ref in enumerate(case["rows"]):
            if ref is None:
                assert present[r] == 0
                continue
            assert present[r] == 1
            np.testing.assert_allclose(a[r], ref[:3], rtol=1e-12, atol=1e-12)
            assert abs(b[r] - ref[3]) <= 1e-11 * max(1.0, abs(ref[3])), (r, b[r], ref[3])


def _voronoi(self_xy, other_xy, bbox):
    d = np.array(other_xy) - np.array(self_xy)
    n = d / np.linalg.norm(d)
    mid = 0.5 * (np.array(self_xy) + np.array(other_xy))
    off = -n @ mid + bbox[0] * abs(n[0]) + bbox[1] * abs(n[1])
    return n, off


def test_fov_qp_structure(oracle):
    cfg = swarm.fov_config(20)
    p = O.make_params(cfg)
    st = np.array([0.3, -0.2, 0.4, 0.5, -0.3, 0.2])
    nbs = np.array([[2.0, 1.0, 0, 0, 0, 0], [-1.5, 2.5, 0, 0, 0, 0], [0.5, -3.0, 0, 0, 0, 0]])
    ref = np.tile([1.0, 1.0, 0.0], 20)
    q0 = oracle.assemble_qp(p, st, ref, nbs, it=0)
    n = 4 * 3 * 4
    assert q0["H"].shape == (n, n)
    eq = q0["lo"] == q0["hi"]
    assert eq.sum() == 6 + 3 * 3 * 3  # initial pos/vel + C^0..C^2 at 3 joints x 3 dims
    ineq = ~eq
    # rows after the equalities: Voronoi (4 per neighbour), FoV (4 per neighbour), box (2 x 3 x K)
    A = q0["A"][ineq]
    hi = q0["hi"][ineq]
    assert A.shape[0] == 3 * 4 + 3 * 4 + 2 * 3 * 20
    C = 4
    for i in range(3):
        nvec, off = _voronoi(st[:2], nbs[i, :2], cfg["bbox"])
        for cp in range(C):
            row = A[i * C + cp]
            expect = np.zeros(n)
            expect[0 * C + cp] = nvec[0]       # piece 0, dim x, control point cp
            expect[1 * C + cp] = nvec[1]       # dim y
            np.testing.assert_allclose(row, expect, atol=1e-15)
            assert abs(hi[i * C + cp] - (-off - 1e-8)) < 1e-12
    # FoV rows: -a^T U_0 x <= b (ConnectivityMPCCBFQPOperations-style, FovMPCCBFQPOperations.cpp:19-29)
    for i in range(3):
        a, b, _ = O.fov_cbf(st, nbs[i, :2], cfg["fov_beta"], cfg["fov_Ds"], cfg["fov_Rs"])
        for r in range(4):
            assert abs(hi[3 * C + 4 * i + r] - b[r]) <= 1e-12 * max(1, abs(b[r]))
    q1 = oracle.assemble_qp(p, st, ref, nbs, it=1, pred=np.vstack([st, st + 0.01]))
    assert (~(q1["lo"] == q1["hi"])).sum() == 3 * 4 + 3 * 4 * 2 + 2 * 3 * 20


def test_fov_impc_oracle_solves_with_certificate(oracle):
    cfg = swarm.fov_config(20)
    p = O.make_params(cfg)
    states, targets = swarm.lattice_swarm(9, seed=4)
    refs = swarm.refs_from_targets(targets, 20)
    for a in range(9):
        nb = np.array([j for j in range(9) if j != a], dtype=np.int32)
        r = O.impc_optimize(p, states, a, nb, refs[a])
        assert r["status"][0] in (O.OPTIMAL, O.INFEASIBLE)
        if r["status"][0] == O.OPTIMAL:
            # the solution satisfies every row of its QP
            q = oracle.assemble_qp(p, states[a], refs[a], states[nb], it=0)
            x = r["x"][0]
            act = q["A"] @ x
            fin_lo = q["lo"] > -1e300
            fin_hi = q["hi"] < 1e300
            assert np.all(act[fin_lo] >= q["lo"][fin_lo] - 1e-6)
            assert np.all(act[fin_hi] <= q["hi"][fin_hi] + 1e-6)
    assert math.isclose(cfg["fov_beta"], 2 * math.pi / 3)


# ---- slack mode (FovBezierIMPCCBF.cpp:58-81, 150-205; FovMPCCBFQPGenerator.cpp:110-207) ------

def _dist_to_ellipse_eig(robot, mean, cov):
    """Independent restatement of FovBezierIMPCCBF::distanceToEllipse (:226-280) through a general
    (non-symmetric) eigen-solver, as the reference's Eigen::EigenSolver."""
    if math.isinf(cov[0][0]):
        return -5.0
    w, V = np.linalg.eig(np.array(cov, dtype=np.float64)[:2, :2])
    w, V = w.real, V.real
    s = 4.605
    with np.errstate(invalid="ignore"):
        a, b = math.sqrt(s * w[0]) if s * w[0] >= 0 else math.nan, \
            math.sqrt(s * w[1]) if s * w[1] >= 0 else math.nan
    if a < b:
        a, b = b, a
    m = 1 if w[1] > w[0] else 0
    th = math.atan2(V[1, m], V[0, m])
    if th < 0:
        th += math.pi
    sl = math.atan2(-mean[1] + robot[1], -mean[0] + robot[0])
    xn = mean[0] + a * math.cos(sl - th) * math.cos(th) - b * math.sin(sl - th) * math.sin(th)
    yn = mean[1] + a * math.cos(sl - th) * math.sin(th) + b * math.sin(sl - th) * math.cos(th)
    dist = math.hypot(xn - robot[0], yn - robot[1])
    if math.isnan(dist):
        return 5.0
    d = math.hypot(mean[0] - robot[0], mean[1] - robot[1])
    rng_ = math.hypot(mean[0] - xn, mean[1] - yn)
    return -dist if d < rng_ else dist


def test_distance_to_ellipse_matches_eigen_restatement(oracle):
    rng = np.random.default_rng(7)
    cases = [((3.0, 0.0), (0.0, 0.0), [[0.1, 0, 0], [0, 0.1, 0], [0, 0, 0.1]]),  # FoV example cov
             ((0.2, 0.1), (0.0, 0.0), [[0.1, 0, 0], [0, 0.1, 0], [0, 0, 0.1]]),  # inside
             ((1.0, 2.0), (0.5, -1.0), [[math.inf, 0, 0], [0, 1, 0], [0, 0, 1]]),  # unknown
             ((1.0, 2.0), (0.5, -1.0), [[0.3, 0.5, 0], [0.5, 0.2, 0], [0, 0, 1]])]  # not PSD
    for _ in range(40):
        L = rng.normal(size=(2, 2))
        c = L @ L.T * rng.uniform(0.01, 2.0)
        cov = [[c[0, 0], c[0, 1], 0], [c[1, 0], c[1, 1], 0], [0, 0, 1]]
        cases.append((tuple(rng.uniform(-5, 5, 2)), tuple(rng.uniform(-5, 5, 2)), cov))
    for robot, mean, cov in cases:
        want = _dist_to_ellipse_eig(robot, mean, cov)
        got = O.distance_to_ellipse(robot, mean, [cov[0][0], cov[0][1], cov[1][1]])
        assert abs(got - want) <= 1e-12 * max(1.0, abs(want)), (robot, mean, cov, got, want)
    # isotropic: the nearest circle point; signed
    s = math.sqrt(4.605 * 0.1)
    assert abs(O.distance_to_ellipse((3.0, 0.0), (0.0, 0.0), [0.1, 0.0, 0.1]) - (3.0 - s)) < 1e-14
    assert abs(O.distance_to_ellipse((0.2, 0.0), (0.0, 0.0), [0.1, 0.0, 0.1]) + (s - 0.2)) < 1e-14
    assert O.distance_to_ellipse((1.0, 2.0), (0.5, -1.0), [0.3, 0.5, 0.2]) == 5.0


def _fov_slack_weights(cfg, st, nbs, covs):
    """slack_weights[i] = w * decay^{idx[i]}, idx = argsort by distanceToEllipse (stable)."""
    de = [_dist_to_ellipse_eig(st, nb, [[c[0], c[1], 0], [c[1], c[2], 0], [0, 0, 1]])
          for nb, c in zip(nbs, covs)]
    idx = sorted(range(len(de)), key=lambda i: de[i])
    return np.array([cfg["slack_cost"] * cfg["slack_decay_rate"] ** idx[i] for i in range(len(de))])


def test_fov_slack_qp_structure_and_weights(oracle):
    cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.5)
    p = O.make_params(cfg)
    states = np.array([[0.0, 0.0, 0.3, 0.4, 0.1, 0.0],
                       [2.6, 0.9, 0, 0, 0, 0], [1.2, 2.9, 0, 0, 0, 0], [3.5, -1.0, 0, 0, 0, 0],
                       [0.9, 1.4, 0, 0, 0, 0]])
    covs = np.array([[0.1, 0.0, 0.1], [0.5, 0.2, 0.3], [0.1, 0.0, 0.1], [2.0, -0.4, 0.2],
                     [0.05, 0.01, 0.02]])
    nb = np.array([1, 2, 3, 4], dtype=np.int32)
    ref = np.tile([2.0, 1.0, 0.3], 20)
    sw = _fov_slack_weights(cfg, states[0], states[nb], covs[nb])
    # the quirk is visible here: weights are not a monotone function of the distance rank
    assert sorted(sw.tolist(), reverse=True) != sw.tolist()
    q = oracle.assemble_qp(p, states[0], ref, states[nb], it=0, slack_w=sw)
    nc = 48
    assert q["n"] == nc + 4
    np.testing.assert_array_equal(q["vlo"][nc:], 0.0)
    np.testing.assert_array_equal(q["c"][nc:], sw)
    ineq = ~(q["lo"] == q["hi"])
    A = q["A"][ineq]
    # Voronoi rows (first 4 x 4) carry no slack; FoV row block of neighbour i carries -1 on slack i
    assert np.all(A[:16, nc:] == 0)
    for i in range(4):
        blk = A[16 + 4 * i:16 + 4 * i + 4, nc:]
        expect = np.zeros((4, 4))
        expect[:, i] = -1.0
        np.testing.assert_array_equal(blk, expect)
    assert np.all(A[32:, nc:] == 0)  # box rows
    # optimize() computes the same weights internally: its iteration-0 QP is this one
    r = O.impc_optimize(p, states, 0, nb, ref, covs=covs)
    sol = oracle.solve_dense_qp(q)
    assert r["status"][0] == sol["status"] == O.OPTIMAL
    assert abs(r["obj"][0] - sol["obj"]) <= 1e-9 * max(1, abs(sol["obj"]))
    # without covariances every distance is -5: weights follow the list order
    q2 = oracle.assemble_qp(p, states[0], ref, states[nb], it=0,
                            slack_w=1000.0 * 0.5 ** np.arange(4))
    r2 = O.impc_optimize(p, states, 0, nb, ref)
    assert abs(r2["obj"][0] - oracle.solve_dense_qp(q2)["obj"]) <= 1e-9 * max(1, abs(r2["obj"][0]))


def voronoi_kat_checks(vor_fn, case, tol):
    """The expectations of separating_hyperplanes/tests/VoronoiTest.cpp:10-73 for one case;
    vor_fn(p1, p2) -> (normal (2+), offset) with bbox 0."""
    p1, p2 = np.array(case["p1"]), np.array(case["p2"])
    n, off = vor_fn(p1, p2)
    n = np.asarray(n, dtype=np.float64)[:2]
    ev = lambda p: float(n @ p + off)  # noqa: E731
    if case["name"] == "ComputeVoronoiHyperplane2D":
        np.testing.assert_allclose(n, case["expected_normal"], atol=tol)
        assert abs(ev(np.array(case["midpoint"]))) <= tol
        assert ev(p1) < 0.0 and ev(p2) > 0.0
        nn = np.linalg.norm(n)
        assert abs(abs(ev(p1)) / nn - abs(ev(p2)) / nn) <= tol
    else:
        perp = np.array([-n[1], n[0]])
        for t in case["t"]:
            pt = perp * t - n * off / (n @ n)
            assert abs(ev(pt)) <= tol
            assert abs(np.linalg.norm(pt - p1) - np.linalg.norm(pt - p2)) <= tol


def test_voronoi_kats(oracle):
    """The oracle's Voronoi rows (oracle.cpp voronoi_shifted, zero box) pass the reference's own
    VoronoiTest known-answer tests (reference_kats.json "voronoi")."""
    k = json.load(open(os.path.join(os.path.dirname(GOLDEN), "reference_kats.json")))["voronoi"]
    assert [c["name"] for c in k["cases"]] == ["ComputeVoronoiHyperplane2D", "EquidistanceProperty"]
    for case in k["cases"]:
        voronoi_kat_checks(lambda a, b: O.voronoi(a, b), case, k["tolerance"])
        # the shift by the robot box moves the plane towards self by |n| . box (planar extents)
        n0, off0 = O.voronoi(case["p1"], case["p2"])
        n1, off1 = O.voronoi(case["p1"], case["p2"], (0.2, 0.3, 0.1))
        np.testing.assert_array_equal(n0, n1)
        assert abs(off1 - (off0 + 0.2 * abs(n0[0]) + 0.3 * abs(n0[1]))) <= 1e-14
