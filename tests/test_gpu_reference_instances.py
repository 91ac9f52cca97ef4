"""GPU: the reference's own experiment instances through the closed-loop simulator, run as the
reference runs them — base_config.json overlaid (preprocess.py:21), zero start velocity, every other
robot a neighbour, robots updated one after another in index order (Gauss–Seidel,
MPCCBFFormationControl_example.cpp:140-201). 2r/line.json is the example's default and the CI run
(:43-44, ci.yml:112-114); 8r/circle.json starts its robots 1.53 m apart, inside d_min = 2 (the
infeasible-start regime). Every update of the device trace must match the oracle's restatement fed
with the same inputs (the rule of test_gpu_sim.py's Gauss–Seidel test), and every status must be
equal."""
import numpy as np
import pytest

import oracle_lib as O
from mpccbf import instances, sim

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a visible MI355X")
    return torch


# (first OPTIMAL -> INFEASIBLE transition of an iteration-0 QP in the 400-step runs,
# profiles/r06_reference_instances.json: 2r/circle 11, 5r/circle 2, 6r/circle 58, 8r/diverge 194 in
# base mode; 3r/line3 17 and 8r/circle2 19 with their own parameters — slack mode, K = 16, every
# other robot a neighbour, which before round 6 ended in a capacity error)
TRANSITIONS = {("2r/circle", "base"): 11, ("5r/circle", "base"): 2, ("6r/circle", "base"): 58,
               ("8r/diverge", "base"): 194, ("3r/line3", "own"): 17, ("8r/circle2", "own"): 19}


@pytest.mark.parametrize("name,mode,steps", [("2r/line", "base", 120), ("8r/circle", "base", 100),
                                             ("3r/line", "base", 100), ("6r/upward", "base", 100),
                                             ("2r/line", "own", 120), ("8r/circle", "own", 100),
                                             ("2r/circle", "base", 24), ("5r/circle", "base", 16),
                                             ("6r/circle", "base", 70), ("8r/diverge", "base", 200),
                                             ("3r/line3", "own", 30), ("8r/circle2", "own", 30)])
def test_reference_instance_gauss_seidel_matches_oracle(mpclib, name, mode, steps):
    """mode "base": the reference's run (base_config.json overlaid); "own": the instance file's own
    parameters (d_min 0.8, w_u_eff 1, ...), the keys it lacks from the base config."""
    _torch()
    cfg, states, targets, shape, kind, noise = instances.instance(name, preprocess=mode)
    seed = 20251015
    s = sim.Simulator(cfg, states, targets, neighbours="all", order="gauss_seidel", record=False,
                      noise_seed=seed, **noise)
    n = len(states)
    gpu, objs = [s.states.cpu().numpy().copy()], []
    for _ in range(steps):
        s.step()
        gpu.append(s.states.cpu().numpy().copy())
        objs.append(s.out["obj"].cpu().numpy().copy())
    gpu = np.array(gpu)
    one, one_status = O.closed_loop_gauss_seidel(cfg, states, targets, steps, pos_std=noise["pos_std"],
                                                 vel_std=noise["vel_std"], seed=seed, neighbours="all", inputs=gpu)
    np.testing.assert_array_equal(np.array(s.status_log), one_status)
    err = np.max(np.abs(gpu - one), axis=2)
    p = O.make_params(cfg)
    refs = np.tile(np.asarray(targets, dtype=np.float64), (1, cfg["k_hor"]))
    # the rule of test_gpu_sim.py: within 1e-8, or within 1e-6 where the oracle's interior-point
    # optimum of an ill-conditioned QP is off the device's exact one (device objective not worse
    # beyond 1e-8 relative;
    # e.g. 3r/line's first step from rest: the acceleration box active at several samples, the
    # oracle 6e-7 off on all three robots)
    for s1, i in zip(*np.nonzero(err > 1e-8)):
        assert err[s1, i] <= 1e-6, (s1, i, err[s1, i])
        st = s1 - 1
        cur = np.concatenate([gpu[st + 1][:i], gpu[st][i:]])
        nb = np.array([j for j in range(n) if j != i], dtype=np.int32)
        r = O.impc_optimize(p, cur, i, nb, refs[i])
        ok = r["status"] == O.OPTIMAL
        # (not worse beyond the solvers' own tolerance: 1e-8 relative)
        assert np.all(objs[st][i][ok] <= r["obj"][ok] + 1e-8 * np.maximum(1.0, np.abs(r["obj"][ok]))), \
            (st, i, objs[st][i], r["obj"])
    # (each such update checked above; they stay rare: 7 of 600 on 6r/upward)
    assert (err > 1e-8).sum() <= max(2, 0.02 * err.size), np.argwhere(err > 1e-8)
    st = np.array(s.status_log)
    d0 = np.sqrt(((states[:, None, :2] - states[None, :, :2]) ** 2).sum(-1)) + np.diag(np.full(n, np.inf))
    if (name, mode) in TRANSITIONS:
        # the run covers an OPTIMAL -> INFEASIBLE transition (the oracle's statuses confirmed every
        # update above); chaotic closed loops may move it by a few steps with last-bit changes
        tr = np.argwhere((st[:-1, :, 0] == O.OPTIMAL) & (st[1:, :, 0] == O.INFEASIBLE))
        assert len(tr) > 0 and tr[0, 0] + 1 <= TRANSITIONS[(name, mode)] + 5, tr[:3]
    elif mode == "base" and name in ("2r/line", "8r/circle"):
        # started inside d_min = 2 of each other (1.5 / 1.53 m): a CBF row no acceleration
        # satisfies, every QP INFEASIBLE, the robots hold position (example :208-221)
        assert d0.min() < cfg["d_min"] and np.all(st[:, :, 0] == O.INFEASIBLE)
    else:
        # (8r/circle with its own d_min: the robots meet at the centre and the later QPs are
        # INFEASIBLE, as the oracle's; the statuses were compared above)
        assert np.mean(st[:10] == O.OPTIMAL) > 0.5
