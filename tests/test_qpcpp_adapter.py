"""qpcpp::HIPSolver<double> — the C++ drop-in for CPLEXSolver<double> (CPLEX.h:19-24) — driven by
tests/cpp/hipsolver_check.cpp on qpcpp::Problem instances built like the reference's callers.

CPU: the flattening into the CPLEX form (column order = forward_list order, i<=j quadratic
convention, infinite bounds) and the loud failure without a GPU. GPU: CPLEXTest::SolveSimpleQP
(x = y = 0.5 within 1e-6, CPLEXTest.cpp:53-54) and a problem with every row/bound kind.
"""
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "mpc-cbf_amd", "build", "hipsolver_check")
BIG = np.finfo(np.float64).max


def run(mode):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (make -C mpc-cbf_amd)")
    out = subprocess.run([EXE, mode], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]


def test_flatten_matches_cplex_form(mpclib):
    p0, p1 = run("flatten")
    # newest variable first (push_front), like CPLEXSolver's column order
    assert p0["col"] == [1, 0] and p1["col"] == [2, 1, 0]
    assert p0["H"] == [1, 0, 0, 1] and p0["lo"] == [1] and p0["hi"] == [BIG]
    H = np.array(p1["H"]).reshape(3, 3)
    col = p1["col"]
    Hv = H[np.ix_(col, col)]  # in creation order (x, y, z)
    np.testing.assert_array_equal(Hv, [[1, 0, 0.5], [0, 1, 0], [0.5, 0, 1]])  # q_xz = 1 -> 1/2, 1/2
    np.testing.assert_array_equal(np.array(p1["c"])[col], [-2, -4, 0])
    assert p1["c0"] == 8
    np.testing.assert_array_equal(np.array(p1["vlo"])[col], [0, -BIG, -2])
    np.testing.assert_array_equal(np.array(p1["vhi"])[col], [0.25, BIG, BIG])
    # rows: newest first as well (range row, then the equality)
    A = np.array(p1["A"]).reshape(2, 3)[:, col]
    np.testing.assert_array_equal(A, [[1, 0, -1], [1, 1, 1]])
    assert p1["lo"] == [-1, 1] and p1["hi"] == [0.5, 1]


def test_solve_without_gpu_reports_error(mpclib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    for r in run("solve"):
        assert r["status"] == "ERROR" and "no HIP device" in r["error"]


def _problem1_reference():
    from scipy.optimize import minimize
    f = lambda v: (v[0] - 1) ** 2 + (v[1] - 2) ** 2 + v[0] * v[2] + v[2] ** 2 + 3  # noqa: E731
    cons = [{"type": "eq", "fun": lambda v: v[0] + v[1] + v[2] - 1},
            {"type": "ineq", "fun": lambda v: 0.5 - (v[0] - v[2])},
            {"type": "ineq", "fun": lambda v: (v[0] - v[2]) + 1}]
    r = minimize(f, np.zeros(3), method="SLSQP", bounds=[(0, 0.25), (None, None), (-2, None)],
                 constraints=cons, options={"ftol": 1e-14, "maxiter": 500})
    assert r.success
    return r.x, r.fun


@pytest.mark.gpu
def test_hipsolver_solves_on_gpu(mpclib):
    p0, p1 = run("solve")
    assert p0["status"] == "OPTIMAL"
    np.testing.assert_allclose(p0["x"], [0.5, 0.5], atol=1e-6)
    assert p1["status"] == "OPTIMAL"
    x, fun = _problem1_reference()
    np.testing.assert_allclose(p1["x"], x, atol=1e-6)
    assert abs(p1["obj"] - fun) <= 1e-6 * max(1.0, abs(fun))


def test_problem_mirror_passes_reference_problem_tests(mpclib):
    """The reference's qpcpp/tests/ProblemTest.cpp:19-137 (all 11 bookkeeping tests: counts,
    variable limits, hasVariable, solution values, constraint / cost coefficients, symmetric
    quadratic lookup, clear / reset) restated in hipsolver_check against the qpcpp::Problem
    mirror that qpcpp::HIPSolver flattens."""
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (make -C mpc-cbf_amd)")
    out = subprocess.run([EXE, "problemtest"], capture_output=True, text=True, timeout=60)
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    names = [r["test"] for r in lines]
    assert names == ["InitialProblemStateIsEmpty", "AddingVariablesIncreasesCount", "VariableMinMaxLimits",
                     "HasVariableTest", "VariableSolutionValueTest", "AddingConstraintsIncreasesCount",
                     "ConstraintCoefficients", "ClearingConstraints", "CostFunctionLinearTerms",
                     "CostFunctionQuadraticTerms", "ResetProblem"]
    assert all(r["ok"] for r in lines), [r for r in lines if not r["ok"]]
    assert out.returncode == 0
