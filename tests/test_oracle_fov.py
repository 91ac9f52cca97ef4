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
