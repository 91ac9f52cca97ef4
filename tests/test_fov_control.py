"""Batched CBF-only controller (FovControl::optimize, cbf/src/controller/FovControl.cpp:17-86):
the oracle restatement on CPU, the device kernel against it on the GPU."""
import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm


def _cfg():
    return swarm.fov_config(20)


def _case(n, seed, scale=1.0):
    """Agents with headings, desired controls pointing at their targets, observed neighbours =
    those inside the FoV cone within Rs (positions only, as FovControl receives them)."""
    cfg = _cfg()
    states, targets = swarm.heading_swarm(n, seed=seed)
    states[:, :2] *= scale
    rng = np.random.default_rng(seed)
    desired = np.zeros((n, 3))
    desired[:, :2] = 2.0 * (targets[:, :2] - states[:, :2]) + rng.uniform(-1, 1, (n, 2))
    desired[:, 2] = rng.uniform(-1, 1, n)
    rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
    nb_xy = states[col, :2] if len(col) else np.zeros((0, 2))
    return cfg, states, desired, rp, nb_xy


def test_oracle_without_neighbours_clips_to_the_box():
    cfg = _cfg()
    st = np.array([0.0, 0.0, 0.3, 1.9, -1.5, 0.0])
    ud = np.array([4.0, -9.0, 1.0])
    stt, u, obj = O.fov_control(cfg, st, ud, np.zeros((0, 2)))
    assert stt == O.OPTIMAL
    lo = np.maximum(cfg["a_min"], np.array(cfg["v_min"]) - st[3:])
    hi = np.minimum(cfg["a_max"], np.array(cfg["v_max"]) - st[3:])
    np.testing.assert_allclose(u, np.clip(ud, lo, hi), atol=1e-7)
    assert abs(obj - np.sum((u - ud) ** 2)) < 1e-6


def test_oracle_solution_satisfies_the_fov_rows():
    cfg, states, desired, rp, nb_xy = _case(40, 3, 0.8)
    checked = 0
    for a in range(40):
        nb = nb_xy[rp[a]:rp[a + 1]]
        stt, u, _ = O.fov_control(cfg, states[a], desired[a], nb)
        if stt != O.OPTIMAL:
            continue
        for o in nb:
            A, b, present = O.fov_cbf(states[a], o, cfg["fov_beta"], cfg["fov_Ds"], cfg["fov_Rs"])
            for r in range(4):
                if present[r]:
                    assert -A[r] @ u <= b[r] + 1e-6 * max(1.0, abs(b[r]))
                    checked += 1
    assert checked > 20


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,scale", [(256, 5, 1.0), (256, 6, 0.6)])
def test_gpu_fov_control_matches_oracle(mpclib, n, seed, scale):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg, states, desired, rp, nb_xy = _case(n, seed, scale)
    dev = torch.device("cuda", 0)
    t = lambda v, dt=torch.float64: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    u = torch.empty((n, 3), dtype=torch.float64, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    obj = torch.empty(n, dtype=torch.float64, device=dev)
    mpclib.fov_control_solve(cfg, t(states), t(desired), t(rp, torch.int32),
                             t(nb_xy if len(nb_xy) else np.zeros((1, 2))), u, status=status, obj=obj)
    torch.cuda.synchronize()
    u, status, obj = u.cpu().numpy(), status.cpu().numpy(), obj.cpu().numpy()
    n_opt = 0
    for a in range(n):
        stt, ur, objr = O.fov_control(cfg, states[a], desired[a], nb_xy[rp[a]:rp[a + 1]])
        assert status[a] == stt, (a, status[a], stt)
        if stt == O.OPTIMAL:
            n_opt += 1
            np.testing.assert_allclose(u[a], ur, atol=1e-6, rtol=1e-6)
            assert abs(obj[a] - objr) <= 1e-6 * max(1.0, abs(objr))
    assert n_opt > n // 2


def _slack_cfg(decay=0.5):
    return dict(_cfg(), control_slack_mode=1, slack_cost=1000.0, slack_decay_rate=decay)


def _nb_covs(nb_count, seed):
    rng = np.random.default_rng(seed)
    cov = np.zeros((nb_count, 3))
    for j in range(nb_count):
        L = rng.normal(size=(2, 2)) * 0.4
        c = L @ L.T + 0.01 * np.eye(2)
        cov[j] = (c[0, 0], c[0, 1], c[1, 1]) if j % 4 else (0.1, 0.0, 0.1)
    return cov


def test_oracle_slack_mode_relaxes_the_fov_rows():
    """FovControl slack mode: every QP solves, the relaxation never costs more than the plain QP
    (its objective includes the slack cost), and where a FoV row binds the slack is used."""
    cfg, states, desired, rp, nb_xy = _case(60, 7, 0.3)
    cov = _nb_covs(len(nb_xy), 3)
    scfg = _slack_cfg()
    n_relaxed = 0
    for a in range(60):
        nb = nb_xy[rp[a]:rp[a + 1]]
        st0, u0, o0 = O.fov_control(cfg, states[a], desired[a], nb)
        st1, u1, o1 = O.fov_control(scfg, states[a], desired[a], nb, nb_cov=cov[rp[a]:rp[a + 1]])
        assert st1 == O.OPTIMAL
        if st0 == O.OPTIMAL:
            assert o1 <= o0 + 1e-6 * max(1.0, abs(o0))
            n_relaxed += o1 < o0 - 1e-6
    assert n_relaxed > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,scale,decay", [(256, 5, 1.0, 0.5), (256, 6, 0.3, 0.9)])
def test_gpu_fov_control_slack_matches_oracle(mpclib, n, seed, scale, decay):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg, states, desired, rp, nb_xy = _case(n, seed, scale)
    scfg = _slack_cfg(decay)
    cov = _nb_covs(max(len(nb_xy), 1), seed)
    dev = torch.device("cuda", 0)
    t = lambda v, dt=torch.float64: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    u = torch.empty((n, 3), dtype=torch.float64, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    obj = torch.empty(n, dtype=torch.float64, device=dev)
    mpclib.fov_control_solve(scfg, t(states), t(desired), t(rp, torch.int32),
                             t(nb_xy if len(nb_xy) else np.zeros((1, 2))), u, status=status, obj=obj,
                             nb_cov=t(cov))
    torch.cuda.synchronize()
    u, status, obj = u.cpu().numpy(), status.cpu().numpy(), obj.cpu().numpy()
    for a in range(n):
        stt, ur, objr = O.fov_control(scfg, states[a], desired[a], nb_xy[rp[a]:rp[a + 1]],
                                      nb_cov=cov[rp[a]:rp[a + 1]])
        assert status[a] == stt, (a, status[a], stt)
        if stt == O.OPTIMAL:
            np.testing.assert_allclose(u[a], ur, atol=1e-5, rtol=1e-5)
            assert abs(obj[a] - objr) <= 1e-4 * max(1.0, abs(objr)), (a, obj[a], objr)
    assert np.all(status == O.OPTIMAL)
