"""GPU: BASELINE config 5 in the FoV example's slack setting at its per-GPU size — 512 agents
(4096 on 8 GPUs), FovBezierIMPCCBF slack mode (slack_cost 1000, decay 0.9, neighbour covariances
0.1 I, BezierIMPCCBFPFXYYaw_example.cpp:138-142,201-202; weights FovBezierIMPCCBF.cpp:58-81) —
run closed loop for 60 steps with the example's trajectory fallback and state noise. No QP may
end UNKNOWN or ERROR, and at every 10th step the oracle re-solves every agent that is not OPTIMAL
in both IMPC iterations, the 16 agents with the most solver steps (the hard QPs: slack patterns,
the slack PDIP) and a seeded sample of 24: statuses equal, objectives within 1e-4."""
import os

import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm
from test_gpu_parity import OBJ_TOL, _torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fov_slack_closed_loop_512_agents(mpclib):
    torch = _torch()
    n, steps = 512, 60
    cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9)
    p = O.make_params(cfg)
    states, targets = swarm.heading_swarm(n)
    refs = swarm.refs_from_targets(targets, cfg["k_hor"])
    cov_h = np.tile([0.1, 0.0, 0.1], (n, 1))
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    out = ctx.alloc_outputs(n)
    traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    out["x"].fill_(float("nan"))
    cur = torch.tensor(states, device=dev)
    tg = torch.tensor(targets, device=dev)
    cov = torch.tensor(cov_h, device=dev)
    rng = np.random.default_rng(5)
    checked = 0
    hist = np.zeros(7, np.int64)
    for s in range(steps):
        ctx.impc_solve(cur, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], cov=cov, traj_t=traj_t, step_index=s,
                       pos_std=0.001, vel_std=0.01, noise_seed=20251015, **out)
        torch.cuda.synchronize()
        st = out["status"].cpu().numpy()
        it = out["iters"].cpu().numpy()
        attempted = ~((st == O.UNKNOWN) & (it == 0))
        hist += np.bincount(st[attempted], minlength=7)
        failed = attempted & ((st == O.UNKNOWN) | (st == 4))
        if np.any(failed) and os.path.isdir(os.path.join(REPO, "gpurun_out")):  # keep the inputs
            np.savez_compressed(os.path.join(REPO, "gpurun_out", f"fovs_fail_step{s}.npz"), states=cur.cpu().numpy(),
                                targets=targets, agents=np.nonzero(np.any(failed, axis=1))[0], status=st)
        assert not np.any(failed), (s, np.argwhere(failed))
        if s % 10 == 9:
            sh = cur.cpu().numpy()
            rp, col = swarm.fov_csr(sh, 8, cfg["fov_Rs"], cfg["fov_beta"])
            obj = out["obj"].cpu().numpy()
            bad = np.nonzero(np.any(st != O.OPTIMAL, axis=1))[0]
            hard = np.argsort(-it.sum(axis=1))[:16]
            agents = sorted(set(bad.tolist()) | set(hard.tolist()) | set(rng.choice(n, 24, replace=False).tolist()))
            for a in agents:
                r = O.impc_optimize(p, sh, a, col[rp[a]:rp[a + 1]], refs[a], covs=cov_h)
                assert list(st[a]) == list(r["status"]), (s, a, st[a], r["status"])
                for k in range(cfg["impc_iter"]):
                    if r["status"][k] == O.OPTIMAL:
                        ro = r["obj"][k]
                        assert abs(obj[a, k] - ro) <= OBJ_TOL * max(1.0, abs(ro)), (s, a, k, obj[a, k], ro)
            checked += len(agents)
        cur = out["next_states"].clone()
    assert checked >= 6 * 24 and hist[O.OPTIMAL] > 0


@pytest.mark.parametrize("slack", [True, False])
def test_fov_closed_loop_is_deterministic(mpclib, slack):
    """The FoV controller's closed loop (512 agents, 30 steps) run twice from the same swarm,
    with the output buffers pre-filled with different garbage and a different allocation
    history, is bit-identical: no result depends on uninitialised memory or on the order the
    neighbour table's atomics insert agents. The neighbour lists the kernel built its rows from
    (mpccbf_batch.nb_out) are compared too, and at step 0 they are the CPU query's (fov_csr: the
    k nearest inside the cone and range, sorted by index).
    Round 3's step-0 failures of the slack case (1 vs 7-8 solver steps) were a product with 0 of
    LDS the active set had not written (das_wave.hpp, the slack patterns' unbounded loops): NaN /
    Inf left there by an earlier kernel turned the first direction into NaN; reproduced
    deterministically by a NaN LDS-poison build (profiles/r04_lds_poison_nan.log)."""
    torch = _torch()
    n, steps = 512, 30
    over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if slack else {}
    cfg = swarm.fov_config(20, **over)
    states, targets = swarm.heading_swarm(n)
    dev = torch.device("cuda", 0)
    cov = torch.tensor(np.tile([0.1, 0.0, 0.1], (n, 1)), device=dev) if slack else None
    runs = []
    for fill in (float("nan"), 1.0e30):
        junk = torch.full((1 << 22,), fill, dtype=torch.float64, device=dev)  # shifts the allocator
        ctx = mpclib.Context(cfg)
        out = ctx.alloc_outputs(n)
        for k, v in out.items():
            v.fill_(fill if v.dtype == torch.float64 else -7)
        traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        out["x"].fill_(float("nan"))
        cur = torch.tensor(states, device=dev)
        tg = torch.tensor(targets, device=dev)
        log = []
        nb_out = torch.full((n, 16), -5, dtype=torch.int32, device=dev)
        for s in range(steps):
            ctx.impc_solve(cur, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], cov=cov, traj_t=traj_t,
                           step_index=s, pos_std=0.001, vel_std=0.01, noise_seed=20251015, nb_out=nb_out, **out)
            log.append((out["status"].clone(), out["iters"].clone(), out["obj"].clone(), out["next_states"].clone(),
                        nb_out.clone()))
            if s == 0:
                rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
                nbl = nb_out.cpu().numpy()
                for a in range(n):
                    lst = col[rp[a]:rp[a + 1]]
                    assert list(nbl[a, :len(lst)]) == list(lst) and np.all(nbl[a, len(lst):] == -1), (a, nbl[a], lst)
            cur = out["next_states"].clone()
        torch.cuda.synchronize()
        runs.append(log)
        del junk
    for s in range(steps):
        for a, b, name in zip(runs[0][s], runs[1][s], ("status", "iters", "obj", "next_states", "nb_out")):
            same = torch.equal(a, b) if name != "obj" else bool(torch.all((a == b) | (torch.isnan(a) & torch.isnan(b))))
            if not same:
                idx = torch.nonzero(a != b)[:4].tolist()
                vals = [(i, a[tuple(i)].item(), b[tuple(i)].item(),
                         [runs[r][s][0][i[0]].tolist() for r in (0, 1)]) for i in idx]
            assert same, (s, name, vals if not same else None)
