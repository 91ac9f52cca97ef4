"""CPU: pin the oracle against the reference's own known-answer tests and the independent numpy
restatement (tests/golden). No GPU needed."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


def test_safety_cbf_kats(oracle, kats):
    spec = kats["safety_cbf"]
    for case in spec["cases"]:
        a, b = oracle.safety_cbf(case["state"], case["neighbor"], spec["d_min"])
        np.testing.assert_allclose(a, case["Ac"], rtol=1e-12, atol=1e-12, err_msg=case["name"])
        assert abs(b - case["Bc"]) <= spec["tolerance_Bc"], (case["name"], b, case["Bc"])
        if case["sign"] == ">0":
            assert b > 0
        elif case["sign"] == "<0":
            assert b < 0
        else:
            assert b == 0.0


def test_cplex_toy_qp(oracle, kats):
    t = kats["cplex_toy_qp"]
    qp = dict(n=2, H=np.array(t["H"]), c=np.array(t["c"]), c0=0.0, A=np.array(t["A"]),
              lo=np.array(t["lo"]), hi=np.array([np.finfo(float).max]),
              vlo=np.full(2, np.finfo(float).min), vhi=np.full(2, np.finfo(float).max))
    r = oracle.solve_dense_qp(qp)
    assert r["status"] == O.OPTIMAL
    np.testing.assert_allclose(r["x"], t["x"], atol=t["tolerance"])


def test_apply_input_kat(oracle, kats):
    t = kats["xyyaw_apply_input"]
    out = oracle.apply_input(t["ts"], t["state"], t["u"])
    np.testing.assert_allclose(out, t["expected"], atol=t["tolerance"])
    A0, L = oracle.prediction_matrices(t["ts"], t["prediction_shapes"]["horizon"])
    assert list(A0.shape) == t["prediction_shapes"]["A0_pos"]
    assert list(L.shape) == t["prediction_shapes"]["Lambda_pos"]


def test_combinatorics_kats(oracle, kats):
    t = kats["combinatorics"]
    L = oracle.lib()
    for n, v in t["fac"]:
        assert L.orc_fac(n) == v
    for n, k, v in t["comb"]:
        assert L.orc_comb(n, k) == v
    for n, k, v in t["perm"]:
        assert L.orc_perm(n, k) == v


def test_bernstein_partition_of_unity_and_range(oracle):
    for t in np.linspace(0, 0.5, 7):
        b = oracle.bernstein_basis(3, 0.5, t, 0)
        assert abs(b.sum() - 1.0) < 1e-14
        assert abs(oracle.bernstein_basis(3, 0.5, t, 1).sum()) < 1e-12
    with pytest.raises(ValueError):
        oracle.bernstein_basis(3, 0.5, 0.6, 0)


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "golden_qps.npz"))


def test_oracle_assembly_matches_numpy_restatement(oracle, golden):
    for i in range(int(golden["count"])):
        g = lambda k: golden[f"c{i}_{k}"]  # noqa: E731
        p = O.make_params(swarm.config(int(g("K"))))
        qp = oracle.assemble_qp(p, g("state"), g("ref"), g("nbs"), it=int(g("it")), pred=g("pred"))
        H = g("H")
        assert np.abs(qp["H"] - H).max() <= 1e-14 * np.abs(H).max()
        np.testing.assert_allclose(qp["c"], g("c"), rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(qp["A"], g("A"), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(qp["lo"], g("lo"), rtol=1e-12)
        np.testing.assert_allclose(qp["hi"], g("hi"), rtol=1e-12)


def test_oracle_solutions_match_golden(oracle, golden):
    for i in range(int(golden["count"])):
        g = lambda k: golden[f"c{i}_{k}"]  # noqa: E731
        p = O.make_params(swarm.config(int(g("K"))))
        qp = oracle.assemble_qp(p, g("state"), g("ref"), g("nbs"), it=int(g("it")), pred=g("pred"))
        r = oracle.solve_dense_qp(qp)
        assert r["status"] == O.OPTIMAL
        obj = float(g("obj"))
        assert abs(r["obj"] - obj) <= 1e-7 * max(1.0, abs(obj)), (i, r["obj"], obj)
        # KKT certificate of the oracle's own solution
        assert r["kkt"][1] <= 1e-8 and r["kkt"][2] <= 1e-8


def test_impc_infeasible_initial_velocity(oracle):
    cfg = swarm.config(10)
    p = O.make_params(cfg)
    states = np.array([[0.0, 0.0, 0.0, 2.5, 0.0, 0.0]])
    r = oracle.impc_optimize(p, states, 0, np.zeros(0, np.int32), np.tile([5.0, 0, 0], 10))
    assert r["status"][0] == O.INFEASIBLE and r["status"][1] == O.UNKNOWN and r["attempted"] == 1


def test_knn_and_all_neighbours_agree_on_lattice(oracle):
    """On the bench lattice (spacing 2.5 d_min) the CBF rows of agents beyond the 8 nearest are
    provably redundant, so KNN and all-neighbour (reference) semantics give the same QP optimum."""
    cfg = swarm.config(15)
    p = O.make_params(cfg)
    states, targets = swarm.lattice_swarm(36)
    refs = swarm.refs_from_targets(targets, 15)
    rp, col = swarm.knn_csr(states, 8, 6.0)
    rpa, cola = swarm.all_csr(36)
    for a in (0, 7, 14, 21, 35):
        r1 = oracle.impc_optimize(p, states, a, col[rp[a]:rp[a + 1]], refs[a])
        r2 = oracle.impc_optimize(p, states, a, cola[rpa[a]:rpa[a + 1]], refs[a])
        assert list(r1["status"]) == list(r2["status"])
        np.testing.assert_allclose(r1["obj"], r2["obj"], rtol=1e-8)


def test_slack_mode_all_neighbours_objective_independent_solver(oracle):
    """The oracle's slack-mode objective with every other robot as a neighbour (the reference's
    all-(N-1) lists, ConnectivityIMPCCBF.cpp:59-67,73-119: slack weights slack_cost * decay^rank
    over 11 neighbours, 5e4 down to 5e-6, some slacks positive) against an independent solve of
    the same assembled QP by scipy's trust-constr. This pins the oracle's slack polish
    (oracle.cpp, orc_impc_optimize: v_i = max(0, max row excess) after the dense solve) with a
    solver that shares no code with it or with the GPU."""
    from scipy.optimize import Bounds, LinearConstraint, minimize
    cfg = swarm.config(15, slack_mode=1)
    p = O.make_params(cfg)
    states, targets = swarm.lattice_swarm(12)
    states[:, :2] *= 0.45  # packed: CBF rows active, slacks positive for close neighbours
    refs = swarm.refs_from_targets(targets, 15)
    big = 1e300
    for i in (0, 2):
        nbr = [j for j in range(12) if j != i]
        r = oracle.impc_optimize(p, states, i, nbr, refs[i])
        assert r["status"][0] == O.OPTIMAL
        d = np.hypot(states[nbr, 0] - states[i, 0], states[nbr, 1] - states[i, 1])
        order = sorted(range(len(nbr)), key=lambda k: (d[k], k))
        rank = np.empty(len(nbr), int)
        rank[order] = np.arange(len(nbr))
        w = cfg["slack_cost"] * cfg["slack_decay_rate"] ** rank
        q = oracle.assemble_qp(p, states[i], refs[i], states[nbr], it=0, slack_w=w)
        inf = lambda a, s: np.where(s * a >= big, s * np.inf, a)  # noqa: E731
        H, c, c0 = q["H"], q["c"], q["c0"]
        res = minimize(lambda x: x @ H @ x + c @ x + c0, np.zeros(q["n"]), jac=lambda x: 2 * H @ x + c,
                       hess=lambda x: 2 * H, method="trust-constr",
                       constraints=[LinearConstraint(q["A"], inf(q["lo"], -1), inf(q["hi"], 1))],
                       bounds=Bounds(inf(q["vlo"], -1), inf(q["vhi"], 1)),
                       options=dict(gtol=1e-12, xtol=1e-14, maxiter=20000))
        assert res.constr_violation <= 1e-9
        assert abs(res.fun - r["obj"][0]) <= 1e-6 * max(1.0, abs(r["obj"][0])), (i, res.fun, r["obj"][0])
        if i == 2:  # a case where the slacks carry most of the cost
            assert r["obj"][0] > 1e6
