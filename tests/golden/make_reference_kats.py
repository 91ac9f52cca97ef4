"""Writes reference_kats.json: the known-answer vectors the reference's own tests hold for the
hot path, transcribed as data (inputs + expected outputs, with the tolerance each test uses).

Sources (paths under workspace/lib of ywang760/mpc-cbf @ 2025-08-29):
  cbf/tests/TestInitSafetyCBF.cpp:50-143   collision (safety) CBF Ac/Bc, d_min 0.8, gamma 5
  qpcpp/tests/CPLEXTest.cpp:28-56          min x^2 + y^2 s.t. x + y >= 1 -> x = y = 0.5
  model/tests/DoubleIntegratorXYYawTest.cpp:19-47  applyInput with ts = 0.1
  math/tests/CombinatoricsTest.cpp:17-63   fac / comb / perm
  separating_hyperplanes/tests/VoronoiTest.cpp:10-73  voronoi(p1, p2): normal direction, midpoint
      on the plane, sides, equidistance (the test's own points and sample parameters)
  cbf/tests/TestInitConnectivity.cpp:103-153  connectivity (lambda2) CBF Ac/Bc, d_max 3.0;
      the intermediate values (lambda2, grad h, Hessian, Lf h, Lf^2 h) are the ones the same
      test run printed, cbf/tests/results.log:7-128 (a data file the reference's tests hold)
Run:  python tests/golden/make_reference_kats.py
"""
import json
import os

KATS = {
    "voronoi": {
        "source": "separating_hyperplanes/tests/VoronoiTest.cpp:10-73",
        "tolerance": 1e-10,
        "cases": [
            # ComputeVoronoiHyperplane2D (:10-44): normal = (p2 - p1) / |p2 - p1|; the midpoint on
            # the plane; p1 on the negative side, p2 on the positive side; equal distances
            {"name": "ComputeVoronoiHyperplane2D", "p1": [1.0, 1.0], "p2": [4.0, 5.0],
             "expected_normal": [0.6, 0.8], "midpoint": [2.5, 3.0], "p1_side": "<0", "p2_side": ">0"},
            # EquidistanceProperty (:46-70): points n_perp t - n offset / |n|^2, t = -5 + 10 i / 10,
            # i = 0..9, lie on the plane and are equidistant from p1 and p2
            {"name": "EquidistanceProperty", "p1": [2.5, -1.0], "p2": [-3.0, 4.0],
             "t": [-5.0 + 10.0 * i / 10 for i in range(10)]},
        ],
    },
    "connectivity_cbf": {
        "source": "cbf/tests/TestInitConnectivity.cpp:103-153, cbf/tests/results.log:7-128",
        "d_min": 0.8, "d_max": 3.0, "lambda2_min": 0.1,
        "tolerance_Ac": 1e-6, "Bc_check": "EXPECT_DOUBLE_EQ (4 ulp)",
        "cases": [
            {"name": "Misc", "self": 0,
             "robot_states": [[1.0, 2.0, 0, 0, 0, 0], [1.0, 4.0, 0, 0, 0, 0], [1.0, 6.0, 0, 0, 0, 0]],
             "Ac": [0.0, -2.703392, 0.0], "Bc": 3.4635324630258153,
             "log_lambda2": 0.23854129852103262, "log_grad_h": [0.0, -2.703392],
             "log_hessian": [[0.622855, 0.0], [0.0, 6.990999]], "log_Lfh": 0.0, "log_Lf2h": 0.0},
            {"name": "Misc2", "self": 0,
             "robot_states": [[0.212, 1.592, 0, -0.293, -0.21, 0.0], [1.01, 4.20, 0, -1.2, 0.12, 0],
                              [-1.0, -0.02, 0, -0.2, 0.16, 0]],
             "Ac": [0.061292, 0.201971, 0.0], "Bc": -2.2784138163109593,
             "log_lambda2": 0.030874640699123754, "log_grad_h": [0.061292, 0.201971],
             "log_hessian": [[-0.011820, 0.217050], [0.217050, 0.629234]],
             "log_Lfh": -0.0603724539485257, "log_Lf2h": 0.05344470569620386},
        ],
    },
    "safety_cbf": {
        "source": "cbf/tests/TestInitSafetyCBF.cpp:50-143",
        "d_min": 0.8,
        "tolerance_Bc": 1e-6,
        "cases": [
            {"name": "TwoRobotInSafeRegion", "state": [0, 0, 0, 0, 0, 0],
             "neighbor": [1, 0, 0, 0, 0, 0], "Ac": [-2.0, 0.0, 0.0],
             "Bc": 0.06347497291775989, "sign": ">0"},
            {"name": "TwoRobotInSafeRegionWithHugeVelocity", "state": [0, 0, 0, 100, 100, 0],
             "neighbor": [1, 0, 0, 0, 0, 0], "Ac": [-2.0, 0.0, 0.0],
             "Bc": -39820583.995200224, "sign": "<0"},
            {"name": "TwoRobotOnSafetyBound", "state": [0, 0, 0, 0, 0, 0],
             "neighbor": [0.8, 0, 0, 0, 0, 0], "Ac": [-1.6, 0.0, 0.0], "Bc": 0.0, "sign": "==0"},
            {"name": "TwoRobotInUnsafeRegion", "state": [0, 0, 0, 0, 0, 0],
             "neighbor": [0.5, 0, 0, 0, 0, 0], "Ac": [-1.0, 0.0, 0.0],
             "Bc": -0.13045522572422458, "sign": "<0"},
        ],
    },
    "cplex_toy_qp": {
        "source": "qpcpp/tests/CPLEXTest.cpp:28-56",
        "objective": "x^2 + y^2 (addQuadraticTerm(x,x,1), (y,y,1))",
        "H": [[1.0, 0.0], [0.0, 1.0]], "c": [0.0, 0.0],
        "A": [[1.0, 1.0]], "lo": [1.0], "hi": ["inf"],
        "status": "OPTIMAL", "x": [0.5, 0.5], "tolerance": 1e-6,
    },
    "xyyaw_apply_input": {
        "source": "model/tests/DoubleIntegratorXYYawTest.cpp:19-47",
        "ts": 0.1, "state": [1.0, 2.0, 0.5, 0.1, 0.2, 0.3], "u": [0.5, 0.6, 0.1],
        "expected": [1.0 + 0.1 * 0.1 + 0.5 * 0.5 * 0.01, 2.0 + 0.2 * 0.1 + 0.5 * 0.6 * 0.01,
                     0.5 + 0.3 * 0.1 + 0.5 * 0.1 * 0.01, 0.1 + 0.5 * 0.1, 0.2 + 0.6 * 0.1,
                     0.3 + 0.1 * 0.1],
        "tolerance": 1e-10,
        "prediction_shapes": {"horizon": 10, "A0_pos": [30, 6], "Lambda_pos": [30, 30]},
    },
}


def combinatorics_cases():
    """CombinatoricsTest.cpp:17-63, transcribed (fac(21) must throw; k > n gives 0)."""
    return {
        "source": "math/tests/CombinatoricsTest.cpp:17-63",
        "fac": [[0, 1], [1, 1], [2, 2], [3, 6], [4, 24], [5, 120], [10, 3628800],
                [20, 2432902008176640000]],
        "fac_throws": [21],
        "comb": [[5, 0, 1], [5, 1, 5], [5, 2, 10], [5, 3, 10], [5, 4, 5], [5, 5, 1], [0, 0, 1],
                 [10, 0, 1], [10, 10, 1], [5, 6, 0], [20, 10, 184756]],
        "perm": [[5, 0, 1], [5, 1, 5], [5, 2, 20], [5, 3, 60], [5, 4, 120], [5, 5, 120],
                 [0, 0, 1], [10, 0, 1], [5, 6, 0], [10, 3, 720]],
    }


if __name__ == "__main__":
    KATS["combinatorics"] = combinatorics_cases()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump(KATS, f, indent=1)
    print("wrote", out)
