"""GPU parity: libmpccbf (HIP, gfx950) against the CPU oracle on identical seeded inputs.

Parity rule: status must match; for OPTIMAL QPs
|obj_gpu - obj_ref| <= 1e-4 * max(1, |obj_ref|) (north-star tolerance), and we additionally
hold the control points to 1e-5 (inf-norm) to catch a wrong-but-close optimum.
"""
import numpy as np
import pytest

import oracle_lib as O
from mpccbf import swarm

pytestmark = pytest.mark.gpu

OBJ_TOL = 1e-4
X_TOL = 1e-5


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a visible MI355X")
    return torch


def run_gpu(ctx, states, targets, row_ptr, col, torch, cov=None):
    dev = torch.device("cuda", 0)
    st = torch.tensor(states, dtype=torch.float64, device=dev)
    tg = torch.tensor(targets, dtype=torch.float64, device=dev)
    rp = torch.tensor(row_ptr, dtype=torch.int32, device=dev)
    cl = torch.tensor(col if len(col) else np.zeros(1, np.int32), dtype=torch.int32, device=dev)
    out = ctx.alloc_outputs(len(states))
    cv = None if cov is None else torch.tensor(cov, dtype=torch.float64, device=dev)
    ctx.impc_solve(st, rp, cl, targets=tg, cov=cv, **out)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def run_oracle(cfg, states, targets, row_ptr, col, agents, cov=None):
    p = O.make_params(cfg)
    refs = swarm.refs_from_targets(targets, cfg["k_hor"])
    res = []
    for a in agents:
        res.append(O.impc_optimize(p, states, a, col[row_ptr[a]:row_ptr[a + 1]], refs[a], covs=cov))
    return res


def compare(cfg, g, ref, agents):
    n = g["x"].shape[1]
    worst = 0.0
    for i, a in enumerate(agents):
        r = ref[i]
        assert list(g["status"][a]) == list(r["status"]), (a, g["status"][a], r["status"])
        for it in range(cfg["impc_iter"]):
            if r["status"][it] == O.OPTIMAL:
                ro = r["obj"][it]
                err = abs(g["obj"][a, it] - ro) / max(1.0, abs(ro))
                worst = max(worst, err)
                assert err <= OBJ_TOL, (a, it, g["obj"][a, it], ro)
        last = [it for it in range(cfg["impc_iter"]) if r["status"][it] == O.OPTIMAL]
        if last:
            xr = r["x"][last[-1]][:n]
            assert np.max(np.abs(g["x"][a] - xr)) <= X_TOL, (a, np.max(np.abs(g["x"][a] - xr)))
    return worst


@pytest.mark.parametrize("k_hor,n_agents", [(10, 256), (15, 64)])
def test_impc_knn_matches_oracle(mpclib, k_hor, n_agents):
    torch = _torch()
    cfg = swarm.config(k_hor)
    states, targets = swarm.lattice_swarm(n_agents)
    rp, col = swarm.knn_csr(states, 8, 3 * cfg["d_min"])
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    agents = list(range(n_agents))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)


def test_impc_all_neighbours_reference_semantics(mpclib):
    """Every other robot as a neighbour (ConnectivityIMPCCBF.cpp:59-67), closer spacing so some
    CBF rows are active."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(36, seed=7)
    states[:, :2] *= 0.5  # 2.5 m lattice: neighbours at ~d_min
    rp, col = swarm.all_csr(len(states))
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    agents = list(range(len(states)))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)


def test_config1_single_agent_static_obstacle(mpclib):
    """BASELINE config 1: 1 agent, K=10, one static obstacle 3 m ahead."""
    torch = _torch()
    cfg = swarm.config(10)
    states = np.array([[0.0, 0.0, 0.0, 0.8, 0.0, 0.0], [3.0, 0.0, 0.0, 0.0, 0.0, 0.0]])
    targets = np.array([[6.0, 0.0, 0.0], [3.0, 0.0, 0.0]])
    rp = np.array([0, 1, 2], np.int32)
    col = np.array([1, 0], np.int32)
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    ref = run_oracle(cfg, states, targets, rp, col, [0])
    compare(cfg, g, ref, [0])


def test_infeasible_initial_velocity(mpclib):
    """v0 outside the velocity box: the k=0 velocity row equals the initial-velocity equality,
    so the QP is infeasible and the IMPC loop stops after iteration 0 (:208-211)."""
    torch = _torch()
    cfg = swarm.config(10)
    states = np.array([[0.0, 0.0, 0.0, 2.5, 0.0, 0.0]])
    targets = np.array([[5.0, 0.0, 0.0]])
    rp = np.array([0, 0], np.int32)
    col = np.zeros(0, np.int32)
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    ref = run_oracle(cfg, states, targets, rp, col, [0])
    assert ref[0]["status"][0] == O.INFEASIBLE
    compare(cfg, g, ref, [0])
    assert np.all(np.isnan(g["x"][0]))


def test_next_state_is_curve_at_h(mpclib):
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(16)
    rp, col = swarm.knn_csr(states, 8, 6.0)
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    p = O.make_params(cfg)
    for a in range(16):
        pos = O.eval_curve(p, g["x"][a], cfg["h"], 0)
        vel = O.eval_curve(p, g["x"][a], cfg["h"], 1)
        np.testing.assert_allclose(g["next_states"][a], np.concatenate([pos, vel]), atol=1e-9)


def test_device_knn_matches_cpu(mpclib):
    torch = _torch()
    cfg = swarm.config(15)
    states, _ = swarm.lattice_swarm(1000)
    rp_ref, col_ref = swarm.knn_csr(states, 8, 6.0)
    ctx = mpclib.Context(cfg)
    dev = torch.device("cuda", 0)
    st = torch.tensor(states, dtype=torch.float64, device=dev)
    rp = torch.empty(len(states) + 1, dtype=torch.int32, device=dev)
    col = torch.empty(len(states) * 8, dtype=torch.int32, device=dev)
    ctx.build_neighbors(st, 0, len(states), 8, 6.0, rp, col)
    torch.cuda.synchronize()
    rp_h = rp.cpu().numpy()
    np.testing.assert_array_equal(rp_h, rp_ref)
    np.testing.assert_array_equal(col.cpu().numpy()[: rp_h[-1]], col_ref)


def test_grid_neighbours_match_csr(mpclib):
    """Fused device neighbour query (spatial hash + in-kernel 3x3 cells) == CSR path with the CPU
    k-nearest lists, on a swarm where several CBF rows are active."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(400, seed=11)
    states[:, :2] *= 0.55  # 2.75 m spacing: close neighbours, non-redundant CBF rows
    rp, col = swarm.knn_csr(states, 8, 6.0)
    ctx = mpclib.Context(cfg)
    g_csr = run_gpu(ctx, states, targets, rp, col, torch)
    dev = torch.device("cuda", 0)
    out = ctx.alloc_outputs(len(states))
    ctx.impc_solve(torch.tensor(states, device=dev), targets=torch.tensor(targets, device=dev),
                   knn_k=8, knn_radius=6.0, **out)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in out.items()}
    np.testing.assert_array_equal(g["status"], g_csr["status"])
    ok = g["status"] == 0
    np.testing.assert_allclose(g["obj"][ok], g_csr["obj"][ok], rtol=1e-10, atol=1e-9)
    # and against the oracle on a sample of agents
    agents = list(range(0, 400, 13))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)


def test_separable_and_dense_layouts_agree(mpclib):
    """variant 0 (separable x/y/yaw layout, pdip_sep.hpp) and variant 3 (dense 6x6 layout,
    pdip.hpp) solve the same QPs: same statuses, objectives within solver tolerance."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(1024, seed=3)
    states[:, :2] *= 0.55
    rp, col = swarm.knn_csr(states, 8, 6.0)
    res = {}
    for variant in (0, 3):
        ctx = mpclib.Context(cfg)
        ctx.set_variant(variant)
        res[variant] = run_gpu(ctx, states, targets, rp, col, torch)
    np.testing.assert_array_equal(res[0]["status"], res[3]["status"])
    ok = res[0]["status"] == 0
    assert ok.sum() > 1000
    err = np.abs(res[0]["obj"][ok] - res[3]["obj"][ok]) / np.maximum(1.0, np.abs(res[3]["obj"][ok]))
    assert err.max() <= 1e-8, err.max()
    assert np.nanmax(np.abs(res[0]["x"] - res[3]["x"])) <= 1e-6


@pytest.mark.parametrize("scale,steps", [(1.0, 25), (0.55, 12), (0.42, 6)])
def test_wide_and_16lane_layouts_agree(mpclib, scale, steps):
    """The share-adaptive default picks the one-agent-per-wave kernel (variant 5) up to one agent
    per SIMD and the 16-lane kernel (variant 4) beyond, so the same QPs must not depend on the
    layout: on a closed-loop-evolved 1024-agent table (both layouts run from the same states),
    equal statuses, objectives within 1e-7 relative and control points within 1e-6 (the two
    layouts' active-set paths can differ — float-keyed vs double candidate scores — and reach the
    same optimum through different factor updates: measured up to 1.6e-8)."""
    torch = _torch()
    dev = torch.device("cuda", 0)
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(1024, seed=21)
    states[:, :2] *= scale
    tg = torch.tensor(targets, device=dev)
    # evolve the table with the default kernel (the bench's noise), then solve it with both layouts
    ctx = mpclib.Context(cfg)
    cur = torch.tensor(states, device=dev)
    alt = torch.empty_like(cur)
    out = ctx.alloc_outputs(len(states))
    traj_t = torch.full((len(states),), -1.0, dtype=torch.float64, device=dev)
    r = ctx.run_steps(cur, alt, steps, targets=tg, knn_k=8, knn_radius=6.0, x=out["x"], obj=out["obj"],
                      traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=7)
    table = r["final"].clone()
    res, names = {}, {}
    for variant in (4, 5):
        c = mpclib.Context(cfg)
        c.set_variant(variant)
        o = c.alloc_outputs(len(states))
        c.impc_solve(table, targets=tg, knn_k=8, knn_radius=6.0, **o)
        torch.cuda.synchronize()
        res[variant] = {k: v.cpu().numpy() for k, v in o.items()}
        names[variant] = c.kernel_name
    assert names == {4: "impc_sep_kernel<1,1,false,256>", 5: "impc_wide_kernel<256>"}, names
    a, b = res[4], res[5]
    np.testing.assert_array_equal(a["status"], b["status"])
    ok = a["status"] == 0
    assert ok.sum() > 0
    err = np.abs(a["obj"][ok] - b["obj"][ok]) / np.maximum(1.0, np.abs(a["obj"][ok]))
    assert err.max() <= 1e-7, err.max()
    assert np.nanmax(np.abs(a["x"] - b["x"])) <= 1e-6, np.nanmax(np.abs(a["x"] - b["x"]))
    if scale < 1.0:  # (the crowded tables have active CBF rows: the solves are not all fast starts)
        assert np.count_nonzero(a["iters"] > 0) > 10


def test_nb_out_written_by_every_collision_kernel(mpclib):
    """mpccbf_batch.nb_out (the neighbour list each agent's QPs were built from) from the generic
    dense-layout kernel (variant 3) equals the separable kernels' (variants 4 and 5) on the same
    grid query: every entry written (no sentinel left), same sets."""
    torch = _torch()
    dev = torch.device("cuda", 0)
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(512, seed=5)
    states[:, :2] *= 0.6
    st = torch.tensor(states, device=dev)
    tg = torch.tensor(targets, device=dev)
    res = {}
    for variant in (3, 4, 5):
        ctx = mpclib.Context(cfg)
        ctx.set_variant(variant)
        out = ctx.alloc_outputs(len(states))
        nbo = torch.full((len(states), 16), -5, dtype=torch.int32, device=dev)
        ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=6.0, nb_out=nbo, **out)
        torch.cuda.synchronize()
        res[variant] = nbo.cpu().numpy()
        assert not np.any(res[variant] == -5), variant
    ref = [sorted(v for v in row if v >= 0) for row in res[4]]
    assert sum(len(r) for r in ref) > 3 * len(states)
    for variant in (3, 5):
        assert [sorted(v for v in row if v >= 0) for row in res[variant]] == ref, variant


def _manual_loop(ctx, st0, tg, steps, first, count, torch):
    a = st0.clone()
    b = st0.clone()
    out = ctx.alloc_outputs(count)
    for _ in range(steps):
        b.copy_(a)  # rows outside the batch carry over
        ctx.impc_solve(a, targets=tg, agent_first=first, num_agents=count, knn_k=8, knn_radius=6.0,
                       x=out["x"], status=out["status"], obj=out["obj"], iters=out["iters"],
                       next_states=b[first:first + count])
        a, b = b, a
    torch.cuda.synchronize()
    return a.cpu().numpy(), out["status"].cpu().numpy()


@pytest.mark.parametrize("first,count", [(0, 512), (0, 500), (12, 488)])
def test_run_steps_matches_step_by_step(mpclib, first, count):
    """mpccbf_run_steps (native closed loop, ping-pong tables) == the same steps issued one by
    one through mpccbf_impc_solve; agents outside the batch stay where they are."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(512, seed=5)
    states[:, :2] *= 0.6
    dev = torch.device("cuda", 0)
    st0 = torch.tensor(states, device=dev)
    tg = torch.tensor(targets[first:first + count], device=dev)
    ctx = mpclib.Context(cfg)
    ref_states, ref_status = _manual_loop(ctx, st0, tg, 7, first, count, torch)
    a, b = st0.clone(), torch.empty_like(st0)
    out = ctx.alloc_outputs(count)
    logs = torch.empty((7, count, 2), dtype=torch.int32, device=dev)
    r = ctx.run_steps(a, b, 7, targets=tg, agent_first=first, num_agents=count, knn_k=8,
                      knn_radius=6.0, x=out["x"], obj=out["obj"], status_log=logs, timing=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r["final"].cpu().numpy(), ref_states)
    np.testing.assert_array_equal(logs[-1].cpu().numpy(), ref_status)
    assert np.all(r["step_ms"] > 0) and np.all(r["solve_ms"] > 0)
    assert np.all(r["solve_ms"] <= r["step_ms"] + 1e-3)
    if count < 512:
        keep = np.ones(512, bool)
        keep[first:first + count] = False
        np.testing.assert_array_equal(ref_states[keep], states[keep])


@pytest.mark.parametrize("first,count", [(0, 512), (12, 488)])
def test_run_steps_continuation_matches_one_call(mpclib, first, count):
    """mpccbf_run::continue_tables (ABI 12): 3 + 4 + 5 steps in three calls, each continuing the
    previous call's neighbour-table rotation, == 12 steps in one call (bit-identical states and
    statuses); a continuation whose states are not the previous call's final table, or after an
    mpccbf_impc_solve in grid mode, rebuilds the table and gives the same result."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(512, seed=6)
    states[:, :2] *= 0.6
    dev = torch.device("cuda", 0)
    st0 = torch.tensor(states, device=dev)
    tg = torch.tensor(targets[first:first + count], device=dev)
    common = dict(targets=tg, agent_first=first, num_agents=count, knn_k=8, knn_radius=6.0)
    ctx = mpclib.Context(cfg)
    out = ctx.alloc_outputs(count)
    a, b = st0.clone(), torch.empty_like(st0)
    log1 = torch.empty((12, count, 2), dtype=torch.int32, device=dev)
    r = ctx.run_steps(a, b, 12, x=out["x"], obj=out["obj"], status_log=log1, **common)
    torch.cuda.synchronize()
    ref, ref_log = r["final"].cpu().numpy(), log1.cpu().numpy()
    for mode in ("continue", "interrupted"):
        c = mpclib.Context(cfg)
        o = c.alloc_outputs(count)
        a, b = st0.clone(), torch.empty_like(st0)
        log2 = torch.empty((12, count, 2), dtype=torch.int32, device=dev)
        s = 0
        for k in (3, 4, 5):
            if mode == "interrupted" and s == 7:  # a grid-mode solve between the calls
                c.impc_solve(a, **common)
            r = c.run_steps(a, b, k, x=o["x"], obj=o["obj"], status_log=log2[s:s + k], step_index=s,
                            continue_tables=s > 0, **common)
            if r["final"] is not a:
                a, b = b, a
            s += k
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.cpu().numpy(), ref)
        np.testing.assert_array_equal(log2.cpu().numpy(), ref_log)


def test_run_steps_with_single_rank_communicator(mpclib):
    """The RCCL exchange path (in-place all-gather after every step) with one rank equals the
    single-process loop."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(256, seed=9)
    dev = torch.device("cuda", 0)
    st0 = torch.tensor(states, device=dev)
    tg = torch.tensor(targets, device=dev)
    ctx = mpclib.Context(cfg)
    ref_states, _ = _manual_loop(ctx, st0, tg, 5, 0, 256, torch)
    comm = mpclib.Comm(mpclib.comm_unique_id(), 1, 0, 0)
    a, b = st0.clone(), torch.empty_like(st0)
    r = ctx.run_steps(a, b, 5, targets=tg, knn_k=8, knn_radius=6.0, comm=comm)
    torch.cuda.synchronize()
    comm.close()
    np.testing.assert_array_equal(r["final"].cpu().numpy(), ref_states)


@pytest.mark.parametrize("scale,n_agents", [(1.0, 64), (0.7, 100)])
def test_fov_controller_matches_oracle(mpclib, scale, n_agents):
    """BASELINE config 5 (FovBezierIMPCCBF): FoV + Voronoi rows, 15 free variables, MFMA
    Newton matrix (impc_fov_kernel) against the oracle on the same observed-neighbour lists."""
    torch = _torch()
    cfg = swarm.fov_config(20)
    states, targets = swarm.heading_swarm(n_agents, seed=2)
    states[:, :2] *= scale
    rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
    ctx = mpclib.Context(cfg)
    assert ctx.kernel_name == "impc_fov_kernel<false>"
    g = run_gpu(ctx, states, targets, rp, col, torch)
    agents = list(range(n_agents))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)


def test_fov_controller_matches_oracle_after_closed_loop(mpclib):
    """Config 5 on states the closed loop produced (40 device steps of a crowded swarm): observed
    neighbours close in, so the batch mixes optimal solves with FoV/Voronoi-infeasible ones, each
    checked against the oracle."""
    torch = _torch()
    cfg = swarm.fov_config(20)
    states, targets = swarm.heading_swarm(100, seed=3)
    states[:, :2] *= 0.6
    targets[:, :2] *= 0.6
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    a, b = torch.tensor(states, device=dev), torch.empty((100, 6), dtype=torch.float64, device=dev)
    r = ctx.run_steps(a, b, 40, targets=torch.tensor(targets, device=dev), knn_k=8,
                      knn_radius=cfg["fov_Rs"])
    torch.cuda.synchronize()
    evolved = r["final"].cpu().numpy()
    rp, col = swarm.fov_csr(evolved, 8, cfg["fov_Rs"], cfg["fov_beta"])
    g = run_gpu(ctx, evolved, targets, rp, col, torch)
    agents = list(range(100))
    ref = run_oracle(cfg, evolved, targets, rp, col, agents)
    compare(cfg, g, ref, agents)
    assert np.any(g["status"] == O.INFEASIBLE) and np.any(g["status"][:, 0] == O.OPTIMAL)


def test_fov_grid_neighbours_match_csr(mpclib):
    """Device FoV neighbour query (grid + field-of-view cone) == the CPU observed-neighbour lists."""
    torch = _torch()
    cfg = swarm.fov_config(20)
    states, targets = swarm.heading_swarm(400, seed=6)
    states[:, :2] *= 0.7
    rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
    ctx = mpclib.Context(cfg)
    g_csr = run_gpu(ctx, states, targets, rp, col, torch)
    dev = torch.device("cuda", 0)
    out = ctx.alloc_outputs(len(states))
    ctx.impc_solve(torch.tensor(states, device=dev), targets=torch.tensor(targets, device=dev),
                   knn_k=8, knn_radius=cfg["fov_Rs"], **out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), g_csr["status"])
    ok = g_csr["status"] == 0
    np.testing.assert_allclose(out["obj"].cpu().numpy()[ok], g_csr["obj"][ok], rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("scale", [1.0, 0.6, 0.45])
def test_fov_dual_active_set_matches_pdip(mpclib, scale):
    """Config 5: the dual active-set solve (default first attempt, das_wave.hpp) and the PDIP alone
    (mpccbf_options.dual_as_steps < 0) give the same statuses — INFEASIBLE included (an unreachable candidate
    goes to phase 1 directly) — and the same optima to the PDIP's tolerance, except where the
    PDIP alone fails (UNKNOWN): there the active-set result is checked against the oracle."""
    torch = _torch()
    cfg = swarm.fov_config(20)
    states, targets = swarm.heading_swarm(256, seed=4)
    states[:, :2] *= scale
    rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
    pdip = run_gpu(mpclib.Context(cfg, dual_as_steps=-1), states, targets, rp, col, torch)
    das = run_gpu(mpclib.Context(cfg), states, targets, rp, col, torch)
    mism = np.nonzero(np.any(pdip["status"] != das["status"], axis=1))[0]
    assert len(mism) <= 0.02 * len(states), mism
    if len(mism):
        assert np.all(np.any(pdip["status"][mism] == O.UNKNOWN, axis=1)), (pdip["status"][mism], das["status"][mism])
        ref = run_oracle(cfg, states, targets, rp, col, list(mism))
        sub = {k: v[mism] for k, v in das.items()}
        compare(cfg, sub, ref, list(range(len(mism))))
    same = np.ones(len(states), dtype=bool)
    same[mism] = False
    ok = (pdip["status"] == 0) & same[:, None]
    assert ok[:, 0].sum() > 50
    err = np.abs(pdip["obj"][ok] - das["obj"][ok]) / np.maximum(1.0, np.abs(pdip["obj"][ok]))
    assert err.max() <= 1e-7, err.max()
    assert np.nanmax(np.abs(pdip["x"][same] - das["x"][same])) <= 1e-5
    assert np.all(das["dual_res"][ok] <= 1e-9) and np.all(das["primal_res"][ok] <= 1e-9)


@pytest.mark.parametrize("scale,k_hor", [(0.42, 15), (0.6, 10)])
def test_slack_mode_matches_oracle(mpclib, scale, k_hor):
    """slack_mode (ConnectivityIMPCCBF.cpp:73-119, MPCCBFQPGeneratorBase.cpp:28-130): one
    nonnegative slack per neighbour on its CBF rows, linear cost slack_cost * decay^rank by
    distance; the kernel eliminates the slacks per lane (Schur complement). A crowded swarm whose
    plain CBF QPs are partly infeasible solves to optimality, with the oracle's objective (slack
    cost included) and curve."""
    torch = _torch()
    cfg = swarm.config(k_hor, slack_mode=1)
    states, targets = swarm.lattice_swarm(64, seed=21)
    states[:, :2] *= scale
    rp, col = swarm.knn_csr(states, 8, 6.0)
    ctx = mpclib.Context(cfg)
    assert ctx.kernel_name == "impc_sep_kernel<1,2,true,256>"
    g = run_gpu(ctx, states, targets, rp, col, torch)
    agents = list(range(64))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)
    plain = run_oracle(swarm.config(k_hor), states, targets, rp, col, agents)
    if scale < 0.5:  # without slack some of these QPs are infeasible; with slack none is
        assert any(r["status"][0] == O.INFEASIBLE for r in plain)
    assert np.all(g["status"][:, 0] == O.OPTIMAL)


@pytest.mark.parametrize("n,scale", [(20, 1.0), (30, 1.0)])
def test_slack_mode_all_neighbours(mpclib, n, scale):
    """Slack mode with the reference's neighbour semantics — every other robot
    (ConnectivityIMPCCBF.cpp:59-67), far more than the 16 lanes of a group: per IMPC iteration the
    neighbours with a live CBF row are compacted into the lanes (a slack without rows is 0 at the
    optimum), weights ranked over all of them. No ERROR; parity with the oracle."""
    torch = _torch()
    cfg = swarm.config(15, slack_mode=1)
    states, targets = swarm.lattice_swarm(n, seed=23)
    states[:, :2] *= scale
    rp, col = swarm.all_csr(n)
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    assert not np.any(g["status"] == O.ERROR)
    agents = list(range(n))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    # the oracle's dense PDIP does not always converge with ~40 slack variables of linear cost
    # (UNKNOWN): those QPs have no verdict to compare with and are left out
    sure = [i for i in agents if O.UNKNOWN not in list(ref[i]["status"])]
    assert len(sure) >= 0.8 * n, len(sure)
    compare(cfg, {k: v[sure] for k, v in g.items()}, [ref[i] for i in sure], list(range(len(sure))))


def test_very_crowded_swarm_statuses_match_oracle(mpclib):
    """Agents 1.5 m apart (below d_min): most QPs are infeasible and their phase-1 LPs end at
    degenerate vertices where the normal matrix loses its pivots; the certificate still agrees
    with the oracle's, and the feasible ones match it."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(64, seed=21)
    states[:, :2] *= 0.3
    rp, col = swarm.knn_csr(states, 8, 6.0)
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    agents = list(range(64))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)
    assert np.sum(g["status"][:, 0] == O.INFEASIBLE) > 16


def _estimate_covs(n, seed):
    """Per-agent position covariances (cxx, cxy, cyy) of the neighbours' estimates: the FoV
    example's 0.1 I for a third, random anisotropic ones for the rest, a few unknown (inf)."""
    rng = np.random.default_rng(seed)
    cov = np.zeros((n, 3))
    for j in range(n):
        if j % 3 == 0:
            cov[j] = (0.1, 0.0, 0.1)
        elif j % 11 == 5:
            cov[j] = (np.inf, 0.0, np.inf)
        else:
            L = rng.normal(size=(2, 2)) * 0.4
            c = L @ L.T + 0.01 * np.eye(2)
            cov[j] = (c[0, 0], c[0, 1], c[1, 1])
    return cov


@pytest.mark.parametrize("scale,decay", [(1.0, 0.5), (0.6, 0.9)])
def test_fov_slack_mode_matches_oracle(mpclib, scale, decay):
    """FovBezierIMPCCBF in slack mode (the FoV example's setting: slack_cost 1000): one slack per
    observed neighbour relaxes its FoV rows; weights ordered by distanceToEllipse with the
    reference's idx[i] indexing; the kernel eliminates each slack in its 8-lane segment through
    the centred-row Schur form (impc_fov_kernel<true>)."""
    torch = _torch()
    cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=decay)
    n = 100
    states, targets = swarm.heading_swarm(n, seed=2)
    states[:, :2] *= scale
    cov = _estimate_covs(n, 5)
    rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
    ctx = mpclib.Context(cfg)
    assert ctx.kernel_name == "impc_fov_kernel<true>"
    g = run_gpu(ctx, states, targets, rp, col, torch, cov=cov)
    agents = list(range(n))
    ref = run_oracle(cfg, states, targets, rp, col, agents, cov=cov)
    compare(cfg, g, ref, agents)
    assert np.mean(g["status"][:, 0] == O.OPTIMAL) > 0.9


def test_fov_slack_mode_crowded_closed_loop(mpclib):
    """Slack mode on closed-loop-evolved crowded states (device neighbour query, 30 steps), where
    the plain FoV QPs are often infeasible: the slack QPs solve, and match the oracle."""
    torch = _torch()
    cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.7)
    n = 100
    states, targets = swarm.heading_swarm(n, seed=3)
    states[:, :2] *= 0.6
    targets[:, :2] *= 0.6
    cov = _estimate_covs(n, 9)
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    a, b = torch.tensor(states, device=dev), torch.empty((n, 6), dtype=torch.float64, device=dev)
    r = ctx.run_steps(a, b, 30, targets=torch.tensor(targets, device=dev), knn_k=8,
                      knn_radius=cfg["fov_Rs"], cov=torch.tensor(cov, device=dev))
    torch.cuda.synchronize()
    evolved = r["final"].cpu().numpy()
    rp, col = swarm.fov_csr(evolved, 8, cfg["fov_Rs"], cfg["fov_beta"])
    g = run_gpu(ctx, evolved, targets, rp, col, torch, cov=cov)
    agents = list(range(n))
    ref = run_oracle(cfg, evolved, targets, rp, col, agents, cov=cov)
    compare(cfg, g, ref, agents)
    plain = run_oracle(swarm.fov_config(20), evolved, targets, rp, col, agents)
    n_inf_plain = sum(r_["status"][0] == O.INFEASIBLE for r_ in plain)
    assert np.sum(g["status"][:, 0] == O.OPTIMAL) >= n - n_inf_plain


def test_fov_slack_grid_neighbours_match_csr(mpclib):
    """Slack weights from the device FoV neighbour query equal the CSR path's (same lists)."""
    torch = _torch()
    cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.5)
    states, targets = swarm.heading_swarm(300, seed=6)
    states[:, :2] *= 0.7
    cov = _estimate_covs(300, 1)
    rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
    ctx = mpclib.Context(cfg)
    g_csr = run_gpu(ctx, states, targets, rp, col, torch, cov=cov)
    dev = torch.device("cuda", 0)
    out = ctx.alloc_outputs(len(states))
    ctx.impc_solve(torch.tensor(states, device=dev), targets=torch.tensor(targets, device=dev),
                   knn_k=8, knn_radius=cfg["fov_Rs"], cov=torch.tensor(cov, device=dev), **out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), g_csr["status"])
    ok = g_csr["status"] == 0
    np.testing.assert_allclose(out["obj"].cpu().numpy()[ok], g_csr["obj"][ok], rtol=1e-10, atol=1e-9)


def test_grid_neighbours_large_table(mpclib):
    """A state table of 12000 agents (the multi-GPU bench gathers 8 x 4096) in the fixed-capacity
    bucket table: a window of agents solved against the whole table matches the CSR path with the
    CPU k-nearest lists."""
    torch = _torch()
    cfg = swarm.config(15)
    n, first, count = 12000, 5000, 512
    states, targets = swarm.lattice_swarm(n, seed=17)
    states[:, :2] *= 0.6
    p = states[:, :2]
    rows = []
    for i in range(first, first + count):
        d2 = np.sum((p - p[i]) ** 2, axis=1)
        d2[i] = np.inf
        cand = np.nonzero(d2 <= 36.0)[0]
        rows.append(np.sort(cand[np.lexsort((cand, d2[cand]))[:8]]))
    rp = np.zeros(count + 1, dtype=np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    dev = torch.device("cuda", 0)
    st = torch.tensor(states, device=dev)
    tg = torch.tensor(targets[first:first + count], device=dev)
    ctx = mpclib.Context(cfg)
    o_csr = ctx.alloc_outputs(count)
    ctx.impc_solve(st, torch.tensor(rp, device=dev), torch.tensor(col, device=dev), targets=tg,
                   agent_first=first, num_agents=count, **o_csr)
    o_grid = ctx.alloc_outputs(count)
    ctx.impc_solve(st, targets=tg, agent_first=first, num_agents=count, knn_k=8, knn_radius=6.0, **o_grid)
    torch.cuda.synchronize()
    s_csr, s_grid = o_csr["status"].cpu().numpy(), o_grid["status"].cpu().numpy()
    np.testing.assert_array_equal(s_grid, s_csr)
    ok = s_csr == 0
    assert ok.sum() > count // 2
    np.testing.assert_allclose(o_grid["obj"].cpu().numpy()[ok], o_csr["obj"].cpu().numpy()[ok],
                               rtol=1e-10, atol=1e-9)


def test_grid_bucket_overflow_falls_back_to_full_scan(mpclib):
    """70 agents in one hash cell (two tight clusters at opposite corners, each agent with 34
    others in range) overflow the 64-slot bucket: the agents that read it scan the whole table,
    so the grid path still equals the CSR path with the CPU k-nearest lists, in the standalone
    solve and after native closed-loop steps."""
    torch = _torch()
    cfg = swarm.config(15)
    n = 300
    states = np.zeros((n, 6))
    g = np.arange(35)
    states[:35, 0], states[:35, 1] = 0.05 + 0.1 * (g % 6), 0.05 + 0.1 * (g // 6)  # cell (0, 0)
    states[35:70, 0], states[35:70, 1] = 5.95 - 0.1 * (g % 6), 5.95 - 0.1 * (g // 6)  # > 6 apart
    m = np.arange(n - 70)
    states[70:, 0], states[70:, 1] = 40.0 + 7.0 * (m % 20), 40.0 + 7.0 * (m // 20)
    targets = states[:, :3].copy()
    targets[:, 0] += 1.0
    dev = torch.device("cuda", 0)
    tg = torch.tensor(targets, device=dev)
    ctx = mpclib.Context(cfg)
    for it in range(2):
        rp, col = swarm.knn_csr(states, 8, 6.0)
        st = torch.tensor(states, device=dev)
        o_csr, o_grid = ctx.alloc_outputs(n), ctx.alloc_outputs(n)
        ctx.impc_solve(st, torch.tensor(rp, device=dev), torch.tensor(col, device=dev), targets=tg, **o_csr)
        ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=6.0, **o_grid)
        torch.cuda.synchronize()
        s_csr, s_grid = o_csr["status"].cpu().numpy(), o_grid["status"].cpu().numpy()
        np.testing.assert_array_equal(s_grid, s_csr)
        assert np.all(s_csr[70:, 0] == O.OPTIMAL)
        ok = s_csr == 0
        np.testing.assert_allclose(o_grid["obj"].cpu().numpy()[ok], o_csr["obj"].cpu().numpy()[ok],
                                   rtol=1e-10, atol=1e-9)
        if it == 0:  # evolve with the native loop (grid tables rotated by the kernel), then recheck
            a, b = st.clone(), torch.empty_like(st)
            r = ctx.run_steps(a, b, 4, targets=tg, knn_k=8, knn_radius=6.0)
            torch.cuda.synchronize()
            states = r["final"].cpu().numpy()
            ref, _ = _manual_loop(ctx, st, tg, 4, 0, n, torch)
            np.testing.assert_array_equal(states, ref)


@pytest.mark.parametrize("scale", [0.55, 0.42, 0.3])
def test_iteration1_warm_start_matches_cold_start(mpclib, scale):
    """IMPC iteration 1 warm-started from iteration 0's primal-dual point (the default,
    mpccbf_options.warm_delta = 0 -> 0.3) and cold-started (warm_delta < 0) reach the same
    optima: statuses equal (also on the very crowded 0.3 lattice, where breakdowns and infeasible
    QPs occur), objectives within solver tolerance; the warm start saves Newton steps. The PDIP
    path alone (dual active-set solve off), which is the one the warm start feeds."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(1024, seed=5)
    states[:, :2] *= scale
    rp, col = swarm.knn_csr(states, 8, 6.0)
    cold = run_gpu(mpclib.Context(cfg, warm_delta=-1.0, dual_as_steps=-1), states, targets, rp, col, torch)
    warm = run_gpu(mpclib.Context(cfg, dual_as_steps=-1), states, targets, rp, col, torch)
    np.testing.assert_array_equal(cold["status"], warm["status"])
    ok = cold["status"] == 0
    if scale < 0.4:  # very crowded: iteration 1 is never reached OPTIMAL; statuses are the check
        return
    assert ok[:, 1].sum() > 100
    err = np.abs(cold["obj"][ok] - warm["obj"][ok]) / np.maximum(1.0, np.abs(cold["obj"][ok]))
    assert err.max() <= 1e-7, err.max()
    assert np.nanmax(np.abs(cold["x"] - warm["x"])) <= 1e-5
    hard = ok[:, 1] & (cold["iters"][:, 1] > 0)  # QPs the fast start does not settle
    if scale > 0.4:
        assert warm["iters"][hard, 1].mean() < cold["iters"][hard, 1].mean()


@pytest.mark.parametrize("scale", [0.3, 0.45, 0.55, 1.0])
def test_dual_active_set_matches_pdip(mpclib, scale):
    """The dual active-set solve (default first attempt) and the PDIP alone (MPCCBF_DUAL_AS=0)
    give the same statuses — INFEASIBLE included: a QP the active-set method finds unreachable is
    certified by phase 1 as before — and the same optima to the PDIP's tolerance; the active-set
    solve takes fewer steps than the PDIP takes Newton steps on the QPs the fast start does not
    settle."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(1024, seed=5)
    states[:, :2] *= scale
    rp, col = swarm.knn_csr(states, 8, 6.0)
    pdip = run_gpu(mpclib.Context(cfg, dual_as_steps=-1), states, targets, rp, col, torch)
    das = run_gpu(mpclib.Context(cfg), states, targets, rp, col, torch)
    np.testing.assert_array_equal(pdip["status"], das["status"])
    ok = pdip["status"] == 0
    if scale < 0.4:  # very crowded: mostly infeasible QPs; statuses are the check
        assert (pdip["status"][:, 0] == 3).sum() > 100
        return
    assert ok[:, 0].sum() > 100
    err = np.abs(pdip["obj"][ok] - das["obj"][ok]) / np.maximum(1.0, np.abs(pdip["obj"][ok]))
    assert err.max() <= 1e-7, err.max()
    assert np.nanmax(np.abs(pdip["x"] - das["x"])) <= 1e-5
    hard = ok[:, 0] & (pdip["iters"][:, 0] > 0)
    if hard.sum() > 10:
        assert das["iters"][hard, 0].mean() < pdip["iters"][hard, 0].mean()


def test_solver_env_vars_have_no_effect(mpclib, monkeypatch):
    """The release library's solver path comes from mpccbf_options alone: the diagnostics build's
    tuning variables (MPCCBF_DUAL_AS, ...) set in the caller's environment change nothing, while
    the same setting through the options does (the PDIP alone takes other solver steps)."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(512, seed=5)
    states[:, :2] *= 0.55
    rp, col = swarm.knn_csr(states, 8, 6.0)
    ref = run_gpu(mpclib.Context(cfg), states, targets, rp, col, torch)
    for k, v in (("MPCCBF_DUAL_AS", "0"), ("MPCCBF_EARLY_IT", "1"), ("MPCCBF_FAST_START", "0"),
                 ("MPCCBF_LEAN", "1"), ("MPCCBF_DAS_WARM", "0"), ("MPCCBF_WARM_DELTA", "0.3x")):
        monkeypatch.setenv(k, v)
    env = run_gpu(mpclib.Context(cfg), states, targets, rp, col, torch)
    for k in ("status", "iters", "obj"):
        np.testing.assert_array_equal(env[k], ref[k])
    opt = run_gpu(mpclib.Context(cfg, dual_as_steps=-1), states, targets, rp, col, torch)
    np.testing.assert_array_equal(opt["status"], ref["status"])
    assert not np.array_equal(opt["iters"], ref["iters"])


@pytest.mark.parametrize("n_ring,radius,v0", [(20, 1.99, (0.2, 0.1)), (40, 1.98, (0.1, 0.3))])
def test_capacity_fallback_many_live_rows(mpclib, n_ring, radius, v0):
    """An agent with more live CBF rows than the default kernel's 16 slots: n_ring static
    neighbours on a half circle just inside d_min, all passed as its neighbours (the reference
    passes every other robot, ConnectivityIMPCCBF.cpp:59-67,135-141). The agent is deferred to the
    128-row fallback launch in the same call: no ERROR, parity with the oracle. The ring robots
    themselves (each other's neighbours, all N-1 semantics) are solved too."""
    torch = _torch()
    cfg = swarm.config(15)
    n = n_ring + 1
    states = np.zeros((n, 6))
    states[0, 3:5] = v0
    ang = np.linspace(0.05, np.pi - 0.05, n_ring)
    states[1:, 0] = radius * np.cos(ang)
    states[1:, 1] = radius * np.sin(ang)
    targets = np.zeros((n, 3))
    targets[:, 1] = -2.0
    targets[1:, :2] = states[1:, :2]
    rp, col = swarm.all_csr(n)
    live = _live_cbf_rows(cfg, states, rp, col)
    assert live[0] > 16, live[0]
    ctx = mpclib.Context(cfg)
    g = run_gpu(ctx, states, targets, rp, col, torch)
    assert not np.any(g["status"] == O.ERROR), np.argwhere(g["status"] == O.ERROR)[:5]
    assert g["status"][0, 0] == O.OPTIMAL
    agents = list(range(n))
    ref = run_oracle(cfg, states, targets, rp, col, agents)
    compare(cfg, g, ref, agents)


def _live_cbf_rows(cfg, states, rp, col):
    """Iteration-0 CBF rows per agent that the exact box filter keeps (b < max_u -a^T u)."""
    amax = np.array(cfg["a_max"])
    amin = np.array(cfg["a_min"])
    out = np.zeros(len(states), dtype=int)
    for i in range(len(states)):
        for j in col[rp[i]:rp[i + 1]]:
            a, b = O.safety_cbf(states[i], states[j], cfg["d_min"])
            bmax = np.sum(np.maximum(-a * amin, -a * amax))
            out[i] += int(b < bmax)
    return out


@pytest.mark.parametrize("what", ["neighbour", "target", "state"])
def test_non_finite_inputs_are_never_optimal(mpclib, what):
    """A NaN neighbour state, target or own state must not come back OPTIMAL (the dual
    active-set scan treats a NaN row as satisfied; it gives up instead and the PDIP's finiteness
    checks decide). Agents packed so the affected agent has live CBF rows; the other agents'
    statuses and optima are unchanged against the oracle on the finite inputs."""
    torch = _torch()
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(64)
    states[:, :2] *= 0.5
    rp, col = swarm.knn_csr(states, 8, 3 * cfg["d_min"])
    bad = 27
    nb = int(col[rp[bad]])
    st, tg = states.copy(), targets.copy()
    if what == "neighbour":
        st[nb, 0] = np.nan  # agent `bad` sees it; so does every other agent with nb in its list
        hit = [a for a in range(64) if nb in col[rp[a]:rp[a + 1]]] + [nb]
    elif what == "target":
        tg[bad, 1] = np.nan
        hit = [bad]
    else:
        st[bad, 3] = np.inf
        hit = [bad]
    # agents that see the bad state (an infinite velocity may give an infinite, dropped row)
    skip = set(hit) | {a for a in range(64) if (nb if what == "neighbour" else bad) in col[rp[a]:rp[a + 1]]}
    ctx = mpclib.Context(cfg)
    for dual_res in (True, False):  # the solver's acceptance must not depend on dual_res
        dev = torch.device("cuda", 0)
        out = ctx.alloc_outputs(64)
        if not dual_res:
            out["dual_res"] = None
        ctx.impc_solve(torch.tensor(st, device=dev), torch.tensor(rp, device=dev), torch.tensor(col, device=dev),
                       targets=torch.tensor(tg, device=dev), **out)
        torch.cuda.synchronize()
        status = out["status"].cpu().numpy()
        for a in hit:
            assert status[a, 0] != O.OPTIMAL, (what, a, status[a])
            assert status[a, 1] != O.OPTIMAL, (what, a, status[a])
    g = {k: v.cpu().numpy() for k, v in out.items() if v is not None}
    others = [a for a in range(64) if a not in skip][:24]
    compare(cfg, g, run_oracle(cfg, states, targets, rp, col, others), others)


@pytest.mark.parametrize("fov", [False, True])
def test_grid_neighbours_crowd_beyond_candidate_capacity(mpclib, fov):
    """More than 64 agents within the query radius of every agent (a 12 x 12 block at 0.45 m
    spacing, radius 6 m: up to 143 candidates): the query switches to its uncapped streaming form
    (grid_neighbors_stream) instead of reporting ERROR, and the k nearest it keeps equal the CPU
    lists: grid path == CSR path (statuses, objectives), collision and FoV controllers."""
    torch = _torch()
    n = 144
    g = np.arange(n)
    states = np.zeros((n, 6))
    states[:, 0], states[:, 1] = 0.45 * (g % 12), 0.45 * (g // 12)
    states[:, 2] = 0.3 * np.sin(g)  # yaw (FoV cones differ per agent)
    targets = states[:, :3].copy()
    targets[:, 0] += 1.5
    if fov:
        cfg = swarm.fov_config(20)
        radius = cfg["fov_Rs"]
        rp, col = swarm.fov_csr(states, 8, radius, cfg["fov_beta"])
    else:
        cfg = swarm.config(15)
        radius = 6.0
        rp, col = swarm.knn_csr(states, 8, radius)
    d2 = np.sum((states[:, None, :2] - states[None, :, :2]) ** 2, axis=-1)
    assert np.all(np.sum(d2 <= radius * radius, axis=1) - 1 > 64)  # every agent: > 64 in range
    dev = torch.device("cuda", 0)
    ctx = mpclib.Context(cfg)
    st, tg = torch.tensor(states, device=dev), torch.tensor(targets, device=dev)
    o_csr, o_grid = ctx.alloc_outputs(n), ctx.alloc_outputs(n)
    ctx.impc_solve(st, torch.tensor(rp, device=dev), torch.tensor(col, device=dev), targets=tg, **o_csr)
    ctx.impc_solve(st, targets=tg, knn_k=8, knn_radius=radius, **o_grid)
    torch.cuda.synchronize()
    s_csr, s_grid = o_csr["status"].cpu().numpy(), o_grid["status"].cpu().numpy()
    assert not np.any(s_grid[:, 0] == O.ERROR)
    np.testing.assert_array_equal(s_grid, s_csr)
    ok = s_csr == 0
    np.testing.assert_allclose(o_grid["obj"].cpu().numpy()[ok], o_csr["obj"].cpu().numpy()[ok], rtol=1e-10, atol=1e-9)
