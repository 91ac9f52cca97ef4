"""The multi-GPU product path of mpccbf_run_steps on one GPU.

Ranks own equal contiguous agent blocks; each step every rank's IMPC kernel writes its block of
the next state table and inserts those rows into the next step's neighbour table, the blocks are
exchanged (an RCCL all-gather across GPUs), and the other ranks' rows are inserted after the
exchange (grid_insert_kernel). Here the ranks are host threads on one device with the in-process
communicator group (mpccbf_comm_create_local: the all-gather becomes device copies between the
ranks' tables), so the whole N-rank data flow runs — table rotation, exchange, foreign-row
insertion — and must reproduce the single-rank closed loop bit for bit. (An N > 1 run over RCCL
needs several GPUs: the driver's scaling run.)
"""
import threading

import numpy as np
import pytest

from mpccbf import swarm

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a visible MI355X")
    return torch


def _run(mpclib, torch, cfg, states, targets, steps, nranks, cov=None, variant=None, names=None):
    dev = torch.device("cuda", 0)
    n = len(states)
    per = n // nranks
    fov = cfg.get("cbf_mode", 0) == 1
    radius = cfg["fov_Rs"] if fov else 3.0 * cfg["d_min"]
    comms = mpclib.Comm.local_group(nranks, 0) if nranks > 1 else [None]
    results, errors = [None] * nranks, []

    def rank_main(r):
        try:
            stream = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(stream):
                ctx = mpclib.Context(cfg)
                if variant is not None:
                    ctx.set_variant(variant)
                out = ctx.alloc_outputs(per)
                a = torch.tensor(states, device=dev)
                b = torch.empty_like(a)
                tg = torch.tensor(targets[r * per:(r + 1) * per], device=dev)
                traj_t = torch.full((per,), -1.0, dtype=torch.float64, device=dev)
                slog = torch.empty((steps, per, 2), dtype=torch.int32, device=dev)
                ilog = torch.empty((steps, per, 2), dtype=torch.int32, device=dev)
                cv = None if cov is None else torch.tensor(cov, device=dev)
                res = ctx.run_steps(a, b, steps, targets=tg, agent_first=r * per, num_agents=per,
                                    knn_k=8, knn_radius=radius, x=out["x"], obj=out["obj"],
                                    traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=7,
                                    status_log=slog, iters_log=ilog, comm=comms[r], stream=stream, cov=cv)
                stream.synchronize()
                if names is not None:
                    names.append(ctx.kernel_name)
                results[r] = (res["final"].cpu().numpy(), slog.cpu().numpy(), out["x"].cpu().numpy(),
                              ilog.cpu().numpy())
        except Exception as e:  # surfaced in the main thread
            errors.append(e)

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(nranks)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    for c in comms:
        if c is not None:
            c.close()
    assert not errors, errors
    return results


@pytest.mark.parametrize("nranks,n_agents,variant", [(2, 1024, 4), (4, 1024, 0), (8, 8192, 0), (8, 8192, 4)])
def test_local_group_matches_single_rank(mpclib, nranks, n_agents, variant):
    """(8, 8192) is BASELINE config 4's shape: 8 ranks x 1024 agents of an 8192-agent table.
    variant 0 (share-adaptive): every rank's 1024 agents take the one-agent-per-wave kernel, so
    the single-rank loop is run with that kernel forced (variant 5) and the two must agree bit for
    bit; variant 4: the 16-lane kernel on both sides."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(n_agents, seed=13)
    states[:, :2] *= 0.6  # crowded: CBF rows, infeasible QPs, fallback trajectories
    steps = 12
    names = []
    single = _run(mpclib, torch, cfg, states, targets, steps, 1, variant=5 if variant == 0 else variant)[0]
    multi = _run(mpclib, torch, cfg, states, targets, steps, nranks, variant=variant, names=names)
    assert all(nm == ("impc_wide_kernel<256>" if variant == 0 else "impc_sep_kernel<1,1,false,256>")
               for nm in names), names
    per = n_agents // nranks
    for r, (final, slog, x, _) in enumerate(multi):
        # every rank ends with the whole gathered table, equal to the single-rank loop
        np.testing.assert_array_equal(final, single[0])
        np.testing.assert_array_equal(slog, single[1][:, r * per:(r + 1) * per])
        np.testing.assert_array_equal(x, single[2][r * per:(r + 1) * per])
    assert not np.array_equal(single[0], states)
    assert np.any(single[1] == 3), "the crowded swarm should produce INFEASIBLE QPs"


@pytest.mark.parametrize("slack", [False, True])
def test_local_group_fov_config5_shape(mpclib, slack):
    """BASELINE config 5's shape: 4096 FoV agents as 8 ranks x 512 (FovBezierIMPCCBF.cpp:48-223,
    cone-filtered neighbour query over the gathered table, foreign rows inserted after the
    exchange), with and without slack variables: bit-identical to the single-rank closed loop,
    solver-step counts included."""
    torch = _torch()
    over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if slack else {}
    cfg = swarm.fov_config(20, **over)
    states, targets = swarm.heading_swarm(4096)
    cov = np.tile([0.1, 0.0, 0.1], (4096, 1)) if slack else None
    steps = 8
    single = _run(mpclib, torch, cfg, states, targets, steps, 1, cov=cov)[0]
    multi = _run(mpclib, torch, cfg, states, targets, steps, 8, cov=cov)
    per = 512
    for r, (final, slog, x, ilog) in enumerate(multi):
        np.testing.assert_array_equal(final, single[0])
        np.testing.assert_array_equal(slog, single[1][:, r * per:(r + 1) * per])
        np.testing.assert_array_equal(ilog, single[3][:, r * per:(r + 1) * per])
        np.testing.assert_array_equal(x, single[2][r * per:(r + 1) * per])
    assert not np.array_equal(single[0], states)
    assert np.any(single[3] > 0), "some QP should need solver steps"


def test_local_group_rank_failure_does_not_hang(mpclib):
    """A rank whose mpccbf_run_steps disagrees (a different num_steps) or fails aborts the
    in-process group: every rank returns an error instead of waiting at a barrier forever."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(256, seed=3)
    dev = torch.device("cuda", 0)
    comms = mpclib.Comm.local_group(2, 0)
    errors = [None, None]

    def rank_main(r):
        try:
            ctx = mpclib.Context(cfg)
            a = torch.tensor(states, device=dev)
            b = torch.empty_like(a)
            tg = torch.tensor(targets[r * 128:(r + 1) * 128], device=dev)
            ctx.run_steps(a, b, 3 + r, targets=tg, agent_first=r * 128, num_agents=128, knn_k=8,
                          knn_radius=6.0, comm=comms[r])
            torch.cuda.synchronize()
        except mpclib.MpccbfError as e:
            errors[r] = str(e)

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=60)
    assert not any(th.is_alive() for th in threads), "a rank hung in the group barrier"
    for c in comms:
        c.close()
    assert errors[0] is not None and errors[1] is not None, errors
    assert any("num_steps" in e for e in errors), errors
