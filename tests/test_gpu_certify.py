"""GPU solutions certified in the reference's full space (SURVEY.md §8c parity rule).

The GPU solves a condensed QP: equality rows eliminated, exactly redundant box rows removed on
the host, CBF rows implied by the acceleration box dropped in the kernel, or — with the fast start
— no Newton step at all when the unconstrained minimiser is feasible. Here each returned control
point vector x is plugged into the oracle's full-space QP of the same inputs (assemble_qp: every
box row, every CBF row unfiltered, all initial-state and continuity equalities, the reference's
x^T H x + c^T x + c0 objective, CPLEX.cpp:82-107) and must be primal feasible to a scaled
residual of 1e-6 with an objective within 1e-4 of the oracle's optimum — which, being the
minimum over the feasible set, certifies the GPU point as optimal to that tolerance. The kernel's
own reported residuals (mpccbf_batch.primal_res / dual_res) are checked against the same bounds.
"""
import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm

FEAS_TOL = 1e-6
OBJ_TOL = 1e-4
INF = 1e299


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a visible MI355X")
    return torch


def _solve(mpclib, cfg, states, targets, rp, col, torch):
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    out = ctx.alloc_outputs(len(states))
    ctx.impc_solve(torch.tensor(states, device=dev), torch.tensor(rp, device=dev),
                   torch.tensor(col if len(col) else np.zeros(1, np.int32), device=dev),
                   targets=torch.tensor(targets, device=dev), **out)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def _scaled_violation(qp, x):
    """Largest row violation of x in the full QP, each row scaled by 1 + |its bound|."""
    ax = qp["A"] @ x
    lo, hi = qp["lo"], qp["hi"]
    vl = np.where(lo > -INF, (lo - ax) / (1.0 + np.abs(np.where(lo > -INF, lo, 0.0))), 0.0)
    vh = np.where(hi < INF, (ax - hi) / (1.0 + np.abs(np.where(hi < INF, hi, 0.0))), 0.0)
    vb = np.maximum(np.where(qp["vlo"] > -INF, qp["vlo"] - x, 0.0),
                    np.where(qp["vhi"] < INF, x - qp["vhi"], 0.0))
    return max(0.0, float(np.max(vl, initial=0.0)), float(np.max(vh, initial=0.0)), float(np.max(vb)))


def _objective(qp, x):
    return float(x @ qp["H"] @ x + qp["c"] @ x + qp["c0"])


@pytest.mark.gpu
@pytest.mark.parametrize("scale,k_hor", [(0.5, 15), (0.45, 10), (1.0, 15)])
def test_gpu_solutions_certified_in_full_space(mpclib, scale, k_hor):
    torch = _torch()
    cfg2 = swarm.config(k_hor)
    cfg1 = swarm.config(k_hor, impc_iter=1)  # iteration 0 alone: the control points it returns
    states, targets = swarm.lattice_swarm(256, seed=3)
    states[:, :2] *= scale
    rp, col = swarm.knn_csr(states, 8, 3.0 * cfg2["d_min"])
    g1 = _solve(mpclib, cfg1, states, targets, rp, col, torch)
    g2 = _solve(mpclib, cfg2, states, targets, rp, col, torch)
    np.testing.assert_array_equal(g1["status"][:, 0], g2["status"][:, 0])
    p = O.make_params(cfg2)
    refs = swarm.refs_from_targets(targets, k_hor)
    hs = [k * cfg2["h"] for k in range(cfg2["cbf_horizon"])]
    checked = [0, 0]
    for a in range(len(states)):
        nbs = states[col[rp[a]:rp[a + 1]]]
        ref = O.impc_optimize(p, states, a, col[rp[a]:rp[a + 1]], refs[a])
        st = g2["status"][a]
        assert list(st) == list(ref["status"]), (a, st, ref["status"])
        for it in range(2):
            if st[it] == O.INFEASIBLE:
                pr = g2["primal_res"][a, it]
                assert np.isnan(pr) or pr > FEAS_TOL, (a, it, pr)
            if st[it] != O.OPTIMAL:
                continue
            # the QP of this IMPC iteration: iteration 1's CBF rows at the states predicted by
            # iteration 0's curve (ConnectivityIMPCCBF.cpp:158-168), evaluated from the GPU's x0
            pred = None
            if it == 1:
                pred = np.array([np.concatenate([O.eval_curve(p, g1["x"][a], t, 0),
                                                 O.eval_curve(p, g1["x"][a], t, 1)]) for t in hs])
            qp = O.assemble_qp(p, states[a], refs[a], nbs, it=it, pred=pred)
            x = (g1 if it == 0 else g2)["x"][a][:qp["n"]]
            viol = _scaled_violation(qp, x)
            assert viol <= FEAS_TOL, (a, it, viol)
            fo = _objective(qp, x)
            assert abs(fo - ref["obj"][it]) <= OBJ_TOL * max(1.0, abs(ref["obj"][it])), (a, it, fo, ref["obj"][it])
            # the kernel's objective is the condensed form's (same value up to rounding)
            assert abs(fo - g2["obj"][a, it]) <= 1e-6 * max(1.0, abs(fo)), (a, it, fo, g2["obj"][a, it])
            assert 0.0 <= g2["primal_res"][a, it] <= FEAS_TOL and 0.0 <= g2["dual_res"][a, it] <= FEAS_TOL, \
                (a, it, g2["primal_res"][a, it], g2["dual_res"][a, it])
            checked[it] += 1
    assert checked[0] > 100 and checked[1] > 50, checked


def test_objective_convention_of_the_full_qp():
    """x^T H x + c^T x + c0 of the oracle's own optimum is the objective it reports (the
    convention the certificate above relies on; P = 2Q, CPLEX.cpp:82-107)."""
    cfg = swarm.config(15)
    p = O.make_params(cfg)
    states, targets = swarm.lattice_swarm(16, seed=3)
    refs = swarm.refs_from_targets(targets, 15)
    rp, col = swarm.knn_csr(states, 8, 6.0)
    qp = O.assemble_qp(p, states[0], refs[0], states[col[rp[0]:rp[1]]], it=0)
    r = O.solve_dense_qp(qp)
    assert r["status"] == O.OPTIMAL
    assert abs(_objective(qp, r["x"]) - r["obj"]) <= 1e-9 * max(1.0, abs(r["obj"]))
