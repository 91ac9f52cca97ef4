"""GPU: closed-loop simulator semantics of mpccbf_batch.traj_t (MPCCBFFormationControl_example.cpp
:150-221) — fallback to the last successful trajectory, eval-time bookkeeping, hold-at-rest
without one — checked step by step against the oracle's curve evaluation, plus the
counter-based state noise (math::addRandomNoise)."""
import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _expected_next(p, cfg, x_new, x_prev, t_prev, have, state):
    """The example's per-robot update for one agent: (next state, new eval time)."""
    step = cfg["Ts"] * int(cfg["h"] / cfg["Ts"])
    tmax = cfg["num_pieces"] * cfg["piece_max_parameter"]
    if have:
        t = min(0.0 + step, tmax)
        xs = x_new
    elif t_prev >= 0.0:
        t = min(t_prev + step, tmax)
        xs = x_prev
    else:
        return np.concatenate([state[:3], np.zeros(3)]), t_prev
    return np.concatenate([O.eval_curve(p, xs, t, 0), O.eval_curve(p, xs, t, 1)]), t


@pytest.mark.parametrize("fov", [False, True])
def test_fallback_trajectory_bookkeeping(mpclib, fov):
    torch = _torch()
    if fov:
        cfg = swarm.fov_config(20)
        states, targets = swarm.heading_swarm(96, seed=11)
        states[:, :2] *= 0.5
        radius = cfg["fov_Rs"]
    else:
        cfg = swarm.config(15)
        states, targets = swarm.lattice_swarm(128, seed=11)
        states[:, :2] *= 0.42  # crowded: iteration failures from the first steps on
        radius = 3.0 * cfg["d_min"]
    p = O.make_params(cfg)
    n_ag = len(states)
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    st = torch.tensor(states, device=dev)
    tg = torch.tensor(targets, device=dev)
    out = ctx.alloc_outputs(n_ag)
    out["x"].fill_(float("nan"))
    traj_t = torch.full((n_ag,), -1.0, dtype=torch.float64, device=dev)
    fallback = held = fresh = 0
    for step in range(10):
        x_prev = out["x"].cpu().numpy().copy()
        t_prev = traj_t.cpu().numpy().copy()
        s_now = st.cpu().numpy().copy()
        ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=radius, traj_t=traj_t, **out)
        torch.cuda.synchronize()
        status = out["status"].cpu().numpy()
        x_new = out["x"].cpu().numpy()
        nxt = out["next_states"].cpu().numpy()
        t_new = traj_t.cpu().numpy()
        for a in range(n_ag):
            have = status[a, 0] == O.OPTIMAL
            if not have:
                np.testing.assert_array_equal(x_new[a], x_prev[a])  # x keeps the stored curve
            e, te = _expected_next(p, cfg, x_new[a], x_prev[a], t_prev[a], have, s_now[a])
            np.testing.assert_allclose(nxt[a], e, rtol=1e-12, atol=1e-12, err_msg=f"step {step} agent {a}")
            assert t_new[a] == te, (step, a, t_new[a], te)
            fresh += have
            fallback += (not have) and t_prev[a] >= 0.0
            held += (not have) and t_prev[a] < 0.0
        st.copy_(out["next_states"])
    assert fresh > 0 and fallback > 0, (fresh, fallback, held)


def test_run_steps_fallback_matches_step_by_step(mpclib):
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(256, seed=12)
    states[:, :2] *= 0.45
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    tg = torch.tensor(targets, device=dev)
    kw = dict(knn_k=8, knn_radius=6.0, pos_std=1e-3, vel_std=1e-2, noise_seed=99)
    # step by step
    st = torch.tensor(states, device=dev)
    out = ctx.alloc_outputs(256)
    tt = torch.full((256,), -1.0, dtype=torch.float64, device=dev)
    for s in range(6):
        ctx.impc_solve(st, targets=tg, traj_t=tt, step_index=s, **kw, **out)
        st.copy_(out["next_states"])
    torch.cuda.synchronize()
    # native loop
    a, b = torch.tensor(states, device=dev), torch.empty((256, 6), dtype=torch.float64, device=dev)
    out2 = ctx.alloc_outputs(256)
    tt2 = torch.full((256,), -1.0, dtype=torch.float64, device=dev)
    r = ctx.run_steps(a, b, 6, targets=tg, x=out2["x"], obj=out2["obj"], traj_t=tt2, **kw)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r["final"].cpu().numpy(), st.cpu().numpy())
    np.testing.assert_array_equal(tt2.cpu().numpy(), tt.cpu().numpy())


def test_state_noise_statistics_and_determinism(mpclib):
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(1024, seed=13)
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    st = torch.tensor(states, device=dev)
    tg = torch.tensor(targets, device=dev)

    def run(pos_std, vel_std, seed):
        out = ctx.alloc_outputs(1024)
        ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=6.0, pos_std=pos_std, vel_std=vel_std,
                       noise_seed=seed, step_index=3, **out)
        torch.cuda.synchronize()
        return out["next_states"].cpu().numpy()

    clean = run(0.0, 0.0, 0)
    a = run(1e-3, 1e-2, 5)
    b = run(1e-3, 1e-2, 5)
    c = run(1e-3, 1e-2, 6)
    np.testing.assert_array_equal(a, b)
    assert np.all(a != c)
    for cols, sd in (((0, 1, 2), 1e-3), ((3, 4, 5), 1e-2)):
        z = (a[:, cols] - clean[:, cols]).reshape(-1) / sd
        assert abs(z.mean()) < 4.0 / np.sqrt(z.size)
        assert 0.9 < z.std() < 1.1


@pytest.mark.parametrize("n,variant", [(1024, 0), (4096, 0)])
def test_launch_clock_per_wave(mpclib, n, variant):
    """mpccbf_run::kernel_clock: every wave of every step's IMPC launch writes its (start, end) pair;
    the launch durations (largest end - smallest start) are positive, below the HIP-event time of
    the same steps' kernels, and the clocked run gives the same closed loop as an unclocked one (the
    clock changes no result). A buffer with fewer pairs per step than the launch's waves is refused."""
    torch = _torch()
    from mpccbf._lib import kernel_clock_us
    dev = torch.device("cuda", 0)
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(n, seed=4)
    ctx = mpclib.Context(cfg)
    ctx.set_variant(variant)
    waves = ctx.launch_waves(n)
    assert waves == (n if n <= 1024 else n // 4)  # one agent per wave / four per wave
    tg = torch.tensor(targets, device=dev)
    steps = 20
    finals = []
    for clocked in (True, False):
        a = torch.tensor(states, device=dev)
        b = torch.empty_like(a)
        kc = torch.zeros((steps, waves, 2), dtype=torch.int64, device=dev) if clocked else None
        r = ctx.run_steps(a, b, steps, targets=tg, knn_k=8, knn_radius=6.0, kernel_clock=kc, timing=not clocked)
        torch.cuda.synchronize()
        finals.append(r["final"].cpu().numpy())
        if clocked:
            us = kernel_clock_us(kc.cpu().numpy())
            assert np.all(np.isfinite(us)) and np.all(us > 1.0), us
            written = (kc.cpu().numpy()[..., 1] != 0).sum(axis=1)
            assert np.all(written == waves), written  # (every wave holds an agent at these sizes)
        else:
            ev_us = r["solve_ms"] * 1e3
    assert np.median(us) <= np.median(ev_us) * 1.05, (np.median(us), np.median(ev_us))
    np.testing.assert_array_equal(finals[0], finals[1])
    with pytest.raises(mpclib.MpccbfError, match="kernel_clock_waves"):
        a = torch.tensor(states, device=dev)
        ctx.run_steps(a, torch.empty_like(a), 2, targets=tg, knn_k=8, knn_radius=6.0,
                      kernel_clock=torch.zeros((2, waves - 1, 2), dtype=torch.int64, device=dev))
