"""Generic dense-QP boundary (mpccbf_qp_solve_dense*), the path a qpcpp::Solver<double> adapter
uses in place of CPLEXSolver::solve (qpcpp/src/solvers/CPLEX.cpp:35-177).

CPU tests: argument validation happens on the host before any device work, and a valid QP
without a GPU fails loudly (no CPU fallback). GPU tests (the equality elimination runs on the
device): the CPLEXTest toy (qpcpp/tests/CPLEXTest.cpp:28-56), the 42 golden MPC-CBF QPs in their
full (un-condensed) CPLEX form, status cases, rank-deficient and inconsistent equalities, fixed
variables, and random QPs against the oracle's independent dense solver.
"""
import os

import numpy as np
import pytest

INF = np.finfo(np.float64).max  # numeric_limits<double>::max() as qpcpp::Problem uses it
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_qps.npz")


def toy():
    # min x^2 + y^2  s.t.  x + y >= 1   (CPLEXTest.cpp:34-47)
    return dict(H=np.eye(2), c=np.zeros(2), A=np.array([[1.0, 1.0]]), lo=np.array([1.0]),
                hi=np.array([INF]))


def test_one_scan_packer_matches_two_pass_form(tmp_path):
    """The host's one-scan packer (dense_pack.hpp pack_qp_once, the product path) gives the plan,
    the first error and the packed words of the two-pass form (plan_qp, then pack_qp) on seeded
    random QPs covering every branch of the packer (tests/cpp/dense_pack_check.cpp). CPU only."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "dense_pack_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + repo, "-I" + os.path.join(repo, "include"),
                    os.path.join(repo, "tests", "cpp", "dense_pack_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "identical" in out.stdout


def test_dense_invalid_arguments_rejected_on_host(mpclib):
    bad = dict(H=np.eye(2), c=np.array([0.0, np.nan]))
    with pytest.raises(mpclib.MpccbfError, match="non-finite"):
        mpclib.dense_qp_solve_batch([bad])
    bad = dict(H=np.eye(2), c=np.zeros(2), A=np.array([[1.0, 1.0]]), lo=np.array([np.nan]),
               hi=np.array([1.0]))
    with pytest.raises(mpclib.MpccbfError, match="NaN"):
        mpclib.dense_qp_solve_batch([bad])


def test_dense_without_gpu_fails_loudly(mpclib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(mpclib.MpccbfError, match="no HIP device"):
        mpclib.dense_qp_solve_batch([toy()])


@pytest.mark.gpu
def test_dense_fully_determined_needs_no_solve(mpclib):
    # equalities pin x completely: decided by the device elimination, no interior-point solve
    q = dict(H=np.eye(2), c=np.array([1.0, 0.0]), A=np.eye(2), lo=np.array([1.0, 2.0]),
             hi=np.array([1.0, 2.0]))
    st, xs, obj = mpclib.dense_qp_solve_batch([q])
    assert st[0] == mpclib.OPTIMAL
    np.testing.assert_allclose(xs[0], [1.0, 2.0])
    assert abs(obj[0] - (1 + 4 + 1)) < 1e-12
    q["lo"] = np.array([1.0, 2.0])
    q["A"] = np.array([[1.0, 0.0], [1.0, 0.0]])  # x = 1 and x = 2: inconsistent
    st, xs, _ = mpclib.dense_qp_solve_batch([q])
    assert st[0] == mpclib.INFEASIBLE and xs[0] is None


@pytest.mark.gpu
def test_cplex_toy(mpclib):
    st, x, obj = mpclib.dense_qp_solve(**toy())
    assert st == mpclib.OPTIMAL
    np.testing.assert_allclose(x, [0.5, 0.5], atol=1e-6)  # CPLEXTest.cpp:53-54 tolerance
    assert abs(obj - 0.5) < 1e-8


@pytest.mark.gpu
def test_dense_status_cases(mpclib):
    qps = [
        toy(),
        # infeasible: x >= 1 and x <= 0
        dict(H=np.eye(1), c=np.zeros(1), A=np.array([[1.0], [1.0]]), lo=np.array([1.0, -INF]),
             hi=np.array([INF, 0.0])),
        # unbounded LP: min -x, x >= 0
        dict(H=np.zeros((1, 1)), c=np.array([-1.0]), vlo=np.array([0.0]), vhi=np.array([INF])),
        # equality only: min x^2 + y^2 s.t. x + y = 1
        dict(H=np.eye(2), c=np.zeros(2), A=np.array([[1.0, 1.0]]), lo=np.array([1.0]),
             hi=np.array([1.0])),
        # LP with a bounded optimum (P = 0): min x + y, 0 <= x, y <= 3, x + y >= 2
        dict(H=np.zeros((2, 2)), c=np.ones(2), A=np.array([[1.0, 1.0]]), lo=np.array([2.0]),
             hi=np.array([INF]), vlo=np.zeros(2), vhi=np.full(2, 3.0)),
        # variable bounds active: min (x - 5)^2 with x <= 2  -> x = 2, obj = x^2 - 10 x + 25 = 9
        dict(H=np.eye(1), c=np.array([-10.0]), c0=25.0, vlo=np.array([-INF]), vhi=np.array([2.0])),
    ]
    st, xs, obj = mpclib.dense_qp_solve_batch(qps)
    assert list(st) == [mpclib.OPTIMAL, mpclib.INFEASIBLE, mpclib.UNBOUNDED, mpclib.OPTIMAL,
                        mpclib.OPTIMAL, mpclib.OPTIMAL]
    np.testing.assert_allclose(xs[3], [0.5, 0.5], atol=1e-9)
    assert abs(obj[4] - 2.0) < 1e-7 and abs(xs[4].sum() - 2.0) < 1e-7
    np.testing.assert_allclose(xs[5], [2.0], atol=1e-8)
    assert abs(obj[5] - 9.0) < 1e-7
    assert xs[1] is None and xs[2] is None


@pytest.mark.gpu
def test_dense_golden_mpc_qps(mpclib):
    """Every golden MPC-CBF QP in its full CPLEX form (36 variables, 30 equalities, box + CBF
    rows) through the generic path: same optimum as the independent solver + KKT certificate."""
    g = np.load(GOLDEN)
    count = int(g["count"])
    qps = [dict(H=g[f"c{i}_H"], c=g[f"c{i}_c"], A=g[f"c{i}_A"], lo=g[f"c{i}_lo"], hi=g[f"c{i}_hi"])
           for i in range(count)]
    st, xs, obj = mpclib.dense_qp_solve_batch(qps)
    for i in range(count):
        assert st[i] == mpclib.OPTIMAL, (i, st[i])
        ref = float(g[f"c{i}_obj"])
        assert abs(obj[i] - ref) <= 1e-4 * max(1.0, abs(ref)), (i, obj[i], ref)
        assert np.max(np.abs(xs[i] - g[f"c{i}_x"])) <= 1e-5


def _random_qp(rng, n, me, mi, redundant=0, fixed=0):
    """A strictly convex QP with me equalities (redundant copies appended), mi two-sided rows
    and `fixed` fixed variables, feasible by construction around x0."""
    M = rng.standard_normal((n, n))
    H = M @ M.T / n + 0.1 * np.eye(n)
    c = rng.standard_normal(n)
    x0 = rng.standard_normal(n)
    E = rng.standard_normal((me, n))
    if redundant:
        E = np.vstack([E, rng.standard_normal((redundant, me)) @ E])
    G = rng.standard_normal((mi, n))
    gx = G @ x0
    A = np.vstack([E, G])
    lo = np.concatenate([E @ x0, gx - rng.uniform(0.05, 1.0, mi)])
    hi = np.concatenate([E @ x0, gx + rng.uniform(0.05, 1.0, mi)])
    vlo = np.full(n, -INF)
    vhi = np.full(n, INF)
    for i in range(fixed):
        vlo[i] = vhi[i] = x0[i]
    return dict(H=H, c=c, A=A, lo=lo, hi=hi, vlo=vlo, vhi=vhi, c0=0.25)


@pytest.mark.gpu
def test_dense_random_qps_match_oracle(mpclib, oracle):
    """Random strictly convex QPs through the device elimination (Householder QR with column
    pivoting, minimum-norm particular solution, null-space basis) and the interior-point kernel,
    against the oracle's dense solve of the same full-space QP: statuses equal, objectives within
    1e-6 relative, solutions within 1e-5. Covers fixed variables (unit equality rows), up to 64
    variables and 58 equalities, a QP without inequality rows, in one batch (the oracle's KKT solve
    needs independent equalities: dependent ones are tested against their closed form below)."""
    rng = np.random.default_rng(11)
    qps = []
    for n, me, mi, red, fx in ((6, 2, 5, 0, 0), (12, 5, 20, 0, 1), (36, 30, 60, 0, 0), (40, 33, 40, 0, 2),
                               (64, 58, 30, 0, 0), (20, 14, 0, 0, 3)):
        qps.append(_random_qp(rng, n, me, mi, red, fx))
    st, xs, obj = mpclib.dense_qp_solve_batch(qps)
    for k, q in enumerate(qps):
        r = oracle.solve_dense_qp(dict(n=q["c"].shape[0], H=q["H"], c=q["c"], c0=q["c0"], A=q["A"], lo=q["lo"],
                                       hi=q["hi"], vlo=q["vlo"], vhi=q["vhi"]))
        assert st[k] == r["status"] == mpclib.OPTIMAL, (k, st[k], r["status"])
        assert abs(obj[k] - r["obj"]) <= 1e-6 * max(1.0, abs(r["obj"])), (k, obj[k], r["obj"])
        np.testing.assert_allclose(xs[k], r["x"], atol=1e-5)


@pytest.mark.gpu
def test_dense_asymmetric_sparse_h_and_index_edges(mpclib, oracle):
    """The packed form carries Hs = (H + H^T)/2's upper triangle with u16 indices (i << 6 | j) and u8
    columns: an asymmetric H (a random antisymmetric part, entries with H_ij = -H_ji whose Hs entry
    is zero) solves as its symmetric part; a sparse block-diagonal H; the index edges at 64 variables
    (i = j = 63, u8 column 63) with 58 equalities and two fixed variables. Against the oracle's
    dense solve of the same QP with Hs given explicitly."""
    rng = np.random.default_rng(41)
    cases = []
    q = _random_qp(rng, 64, 58, 30, 0, 2)
    K = rng.standard_normal((64, 64))
    q["H"] = q["H"] + (K - K.T)
    cases.append(q)
    q = _random_qp(rng, 20, 14, 12, 0, 0)
    Hs = q["H"].copy()
    Hb = np.zeros_like(Hs)
    for b0 in range(0, 20, 5):  # block-diagonal part of Hs (positive definite blocks)
        Hb[b0:b0 + 5, b0:b0 + 5] = Hs[b0:b0 + 5, b0:b0 + 5]
    A5 = np.zeros_like(Hs)
    A5[0, 19], A5[19, 0] = 3.0, -3.0  # antisymmetric pair: Hs zero there
    q["H"] = Hb + A5
    cases.append(q)
    st, xs, obj = mpclib.dense_qp_solve_batch(cases)
    for k, q in enumerate(cases):
        hs = 0.5 * (q["H"] + q["H"].T)
        r = oracle.solve_dense_qp(dict(n=q["c"].shape[0], H=hs, c=q["c"], c0=q["c0"], A=q["A"], lo=q["lo"],
                                       hi=q["hi"], vlo=q["vlo"], vhi=q["vhi"]))
        assert st[k] == r["status"] == mpclib.OPTIMAL, (k, st[k], r["status"])
        assert abs(obj[k] - r["obj"]) <= 1e-6 * max(1.0, abs(r["obj"])), (k, obj[k], r["obj"])
        np.testing.assert_allclose(xs[k], r["x"], atol=1e-5)


@pytest.mark.gpu
def test_dense_inconsistent_and_dependent_equalities(mpclib):
    """Dependent equalities with consistent right-hand sides are dropped by the pivoted QR's
    rank test; inconsistent ones make the QP INFEASIBLE; more equalities than variables."""
    base = dict(H=np.eye(3), c=np.zeros(3))
    A = np.array([[1.0, 1.0, 0.0], [2.0, 2.0, 0.0], [0.0, 1.0, 1.0], [1.0, 2.0, 1.0]])
    ok = dict(base, A=A, lo=np.array([1.0, 2.0, 1.0, 2.0]), hi=np.array([1.0, 2.0, 1.0, 2.0]))
    bad = dict(base, A=A, lo=np.array([1.0, 2.5, 1.0, 2.0]), hi=np.array([1.0, 2.5, 1.0, 2.0]))
    st, xs, obj = mpclib.dense_qp_solve_batch([ok, bad])
    assert st[0] == mpclib.OPTIMAL and st[1] == mpclib.INFEASIBLE
    x = xs[0]
    np.testing.assert_allclose([x[0] + x[1], x[1] + x[2]], [1.0, 1.0], atol=1e-10)
    # min |x|^2 on the two planes: x = (1/3, 2/3, 1/3)
    np.testing.assert_allclose(x, [1 / 3, 2 / 3, 1 / 3], atol=1e-9)


@pytest.mark.gpu
def test_dense_beyond_device_elimination_capacity(mpclib, oracle):
    """QPs beyond the device elimination's 64 variables / 64 equality rows are reduced on the host
    (host/dense_qp.cpp) and solved by the same device interior-point kernel, in one batch with a
    device-reduced QP: 80 variables with 74 equality rows and 2 fixed variables (reduced dimension
    4), and 40 variables with 70 equality rows of rank 34 (36 consistent combinations: reduced
    dimension 6, the same optimum as its 34 independent rows), against the oracle. Inconsistent
    equalities with a reduced dimension above 8 are INFEASIBLE, not a capacity error (the equality
    decision precedes the capacity checks), on the device path (30 variables) and the host path (90)."""
    rng = np.random.default_rng(29)
    big = _random_qp(rng, 80, 74, 40, 0, 2)
    small = _random_qp(rng, 12, 5, 20, 0, 1)
    indep = _random_qp(rng, 40, 34, 30, 0, 0)
    eq = indep["lo"] == indep["hi"]
    E, b = indep["A"][eq], indep["lo"][eq]
    W = rng.normal(size=(36, E.shape[0]))
    dep = dict(indep, A=np.vstack([indep["A"], W @ E]), lo=np.concatenate([indep["lo"], W @ b]),
               hi=np.concatenate([indep["hi"], W @ b]))
    st, xs, obj = mpclib.dense_qp_solve_batch([big, small, dep])
    for k, q in enumerate((big, small, indep)):
        r = oracle.solve_dense_qp(dict(n=q["c"].shape[0], H=q["H"], c=q["c"], c0=q["c0"], A=q["A"], lo=q["lo"],
                                       hi=q["hi"], vlo=q["vlo"], vhi=q["vhi"]))
        assert st[k] == r["status"] == mpclib.OPTIMAL, (k, st[k], r["status"])
        assert abs(obj[k] - r["obj"]) <= 1e-6 * max(1.0, abs(r["obj"])), (k, obj[k], r["obj"])
        np.testing.assert_allclose(xs[k], r["x"], atol=1e-5)
    # inconsistent equalities (a row repeated with its right-hand side + 1), reduced dimension 20
    for n in (30, 90):
        q = _random_qp(rng, n, 10, 5, 0, 0)
        eqm = q["lo"] == q["hi"]
        row, rhs = q["A"][eqm][0], q["lo"][eqm][0] + 1.0
        extra = 1 if n <= 64 else 60  # (beyond 64 equality rows too on the host path)
        q["A"] = np.vstack([q["A"]] + [row[None, :]] * extra)
        q["lo"] = np.concatenate([q["lo"], np.full(extra, rhs)])
        q["hi"] = np.concatenate([q["hi"], np.full(extra, rhs)])
        st, xs, _ = mpclib.dense_qp_solve_batch([q])
        assert st[0] == mpclib.INFEASIBLE and xs[0] is None, (n, st[0])
    # a violated constant row (an inequality along an equality row, its bounds excluding the
    # equality's value) with a reduced dimension above 8: decided only within capacity, so a
    # capacity error on both paths (the device reduction's order), not INFEASIBLE on one of them
    for n in (30, 90):
        q = _random_qp(rng, n, 10, 5, 0, 0)
        eqm = q["lo"] == q["hi"]
        row, rhs = q["A"][eqm][0], q["lo"][eqm][0]
        q["A"] = np.vstack([q["A"], row[None, :]])
        q["lo"] = np.concatenate([q["lo"], [rhs + 1.0]])
        q["hi"] = np.concatenate([q["hi"], [rhs + 2.0]])
        with pytest.raises(mpclib.MpccbfError, match="capacity|exceeds"):
            mpclib.dense_qp_solve_batch([q])
