"""Benchmark: batched MPC-CBF QP solves on MI355X (BASELINE.json metric).

A step = one IMPC control step of ConnectivityIMPCCBF::optimize for every agent
(mpc_cbf/src/controller/ConnectivityIMPCCBF.cpp:47-215): state exchange (RCCL all-gather over
xGMI when --gpus > 1), neighbour lists, two dependent QP solves per agent (fused HIP kernel), and
the closed-loop state update. value = QPs solved by all ranks / wall time.

Default workload (N=1): BASELINE config 3 — 4096 agents, horizon 15, pairwise collision CBF,
8 nearest neighbours within 3 d_min, base_config.json parameters. Multi-GPU (N > 1): BASELINE
config 4 — 8192 agents in total sharded over the N GPUs (1024 per GPU at N = 8), strong scaling;
--weak keeps 4096 agents per GPU instead. FoV (--workload fov): config 5's 512-agent per-GPU
share at N = 1, its 4096 agents in total at N > 1.

    python bench.py [--gpus N --steps K --warmup W]      (N > 1: relaunches itself as N ranks)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Timing: the timed pass runs warm-up + K steps with nothing else on the stream (barrier +
synchronize on both sides, max over ranks); an identical replay of the same steps (same initial
swarm and counter-based noise) records HIP events around every step and every IMPC kernel for the
p99 step latency and the kernel's average duration (roofline).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= matrix) peak, vendor spec
HBM_PEAK_GBS = 8000.0
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 4  # wave64 VALU instructions / s: 1024 SIMDs, one per 4 cycles at 2.4 GHz


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", choices=["collision", "fov", "dense"], default="collision",
                    help="collision: BASELINE config 3/4 (ConnectivityIMPCCBF); fov: config 5 "
                         "(FovBezierIMPCCBF, horizon 20, 4 Bezier pieces); dense: the generic "
                         "qpcpp::Solver path (mpccbf_qp_solve_dense_batch) on the golden QPs")
    ap.add_argument("--agents-per-gpu", type=int, default=0,
                    help="default 4096 (collision), 512 (fov: config 5 = 4096 agents on 8 GPUs)")
    ap.add_argument("--agents-total", type=int, default=0,
                    help="strong scaling: fixed total (default at --gpus > 1: 8192 collision = config 4, "
                         "4096 fov = config 5)")
    ap.add_argument("--weak", action="store_true",
                    help="--gpus > 1: weak scaling, --agents-per-gpu agents on every GPU")
    ap.add_argument("--rank-share", type=int, default=0,
                    help="one GPU times rank 0's share of an N-rank run: agents-total / N agents of "
                         "the agents-total table, the other rows carried over and inserted into the "
                         "next step's neighbour table every step (the all-gather itself excluded)")
    ap.add_argument("--k-hor", type=int, default=0, help="default 15 (collision), 20 (fov)")
    ap.add_argument("--knn", type=int, default=8)
    ap.add_argument("--slack", action="store_true",
                    help="slack_mode (one slack per neighbour on its CBF rows): the FoV example's "
                         "setting (slack_cost 1000, neighbour covariances 0.1 I, "
                         "BezierIMPCCBFPFXYYaw_example.cpp:138-142,201-202)")
    ap.add_argument("--slack-decay", type=float, default=0.9)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--das-warm", type=int, default=0,
                    help="mpccbf_options.das_warm_steps (0 = default 3; < 0 = no IMPC iteration-1 warm start)")
    ap.add_argument("--lean", action="store_true",
                    help="diagnostics: mpccbf_options.lean (main launch without the PDIP; a fallback launch per step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--loop", choices=["native", "python"], default="native",
                    help="native: mpccbf_run_steps (C++ loop, RCCL); python: one call per step")
    ap.add_argument("--neighbours", choices=["grid", "csr", "all"], default="grid",
                    help="grid: fused in-kernel spatial-hash query; csr: separate KNN kernels; all: "
                         "every other robot as a neighbour (the reference's own lists, "
                         "ConnectivityIMPCCBF.cpp:59-67), fixed CSR lists in the native loop")
    ap.add_argument("--crowded", action="store_true",
                    help="collision workload on a crowded lattice (0.6 x the spacing: 3 m, jitter +-0.3 m), "
                         "where the dual active set and the interior-point fallback do the work")
    ap.add_argument("--no-trace", action="store_true",
                    help="skip the closed-loop safety metrics pass (collision_check.py on the trace)")
    ap.add_argument("--dump", default="",
                    help="write the timed pass's per-step status / solver-step logs (rank 0) to this .npz")
    return ap.parse_args(argv)


def flops_per_qp(iters: np.ndarray, rows: np.ndarray, nz: int) -> float:
    """Algorithmic FP64 flops of the dense-layout condensed Mehrotra PDIP (impc_kernel), one QP:
    per iteration and row: residual 2nz, normal matrix nz(nz+1), rhs 2nz, two step directions
    2*2nz, step/update ~20; per iteration: Cholesky nz^3/3, four triangular solves 4nz^2,
    P y 2nz^2. (roofline uses min(canonical, executed); executed is smaller.)"""
    per_row = 2 * nz + nz * (nz + 1) + 2 * nz + 4 * nz + 20
    per_it = nz ** 3 / 3 + 6 * nz * nz
    return float(np.sum(iters * (rows * per_row + per_it)))


def flops_per_qp_sep(iters: np.ndarray, rows: int) -> float:
    """Algorithmic FP64 flops of the separable-layout solver (impc_sep_kernel), one QP: `iters`
    counts its steps — dual active-set steps, then PDIP Newton steps for the rare QPs the
    active-set solve hands on. Priced as active-set steps, a lower bound for either: per step
    and box row (2 nonzeros, both sides) ~10 flops of violation scan, per step ~500 flops of the
    k x k (k <= 6) factorisation, the multiplier and primal directions and the step lengths; CBF
    rows (4 nonzeros) not counted. (A PDIP Newton step is ~60 flops per box row + 100.)"""
    return float(np.sum(iters * (rows * 10 + 500)))


STATUS_NAMES = {0: "OPTIMAL", 3: "INFEASIBLE", 4: "ERROR", 5: "UNKNOWN"}


def spawn_ranks(args) -> None:
    """`--gpus N` outside torch.distributed.run: relaunch this command as N ranks (one process per
    GPU, torch.distributed.run on 127.0.0.1) before anything touches the GPU, and exit with the
    launcher's code. A torchrun environment whose WORLD_SIZE differs from --gpus is an error."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def algorithmic_bytes_per_agent(n: int, knn: int, impc_iter: int, cov: bool) -> int:
    """HBM bytes one agent-step must move: state 48 + target 24 + knn neighbour
    states (px, py, vx, vy: 32 each) + the kept curve x (8 n) + per-iteration status, iterations
    and objective (16 each) + next state 48 + trajectory time read / write 16 (+ 24 per neighbour
    covariance in FoV slack mode)."""
    return 48 + 24 + 32 * knn + 8 * n + 16 * impc_iter + 48 + 16 + (24 * knn if cov else 0)


def run_dense(args) -> None:
    """--workload dense: the generic path a qpcpp::Solver<double> adapter calls in place of
    CPLEXSolver::solve (qpcpp/src/solvers/CPLEX.cpp:35-177) — mpccbf_qp_solve_dense_batch on the
    42 golden MPC-CBF QPs in their full CPLEX form (36 variables, 30 equalities, box + CBF rows),
    replicated to --agents-per-gpu QPs per call (default 4096). The boundary takes host arrays, so
    the rate includes the transfers both ways and the host-side validation and packing; the
    mpccbf_dense_qp structs (pointers to the caller's arrays) are marshalled once, outside the
    timed calls, as a C++ caller holds them. Also reported: the
    single-QP latency (mpccbf_qp_solve_dense, one synchronous call) and the CPU oracle's dense
    solve of the same QPs. Replicas only: no multi-GPU form."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        sys.exit("bench.py --workload dense: single GPU only")
    import torch
    from mpccbf import _lib as L
    torch.cuda.set_device(0)
    g = np.load(os.path.join(REPO, "tests", "golden", "golden_qps.npz"))
    count = int(g["count"])
    qps = [dict(H=g[f"c{i}_H"], c=g[f"c{i}_c"], A=g[f"c{i}_A"], lo=g[f"c{i}_lo"], hi=g[f"c{i}_hi"])
           for i in range(count)]
    ref = np.array([float(g[f"c{i}_obj"]) for i in range(count)])
    batch = args.agents_per_gpu if args.agents_per_gpu > 0 else 4096
    big = [qps[i % count] for i in range(batch)]
    # the caller's QP structs (pointers to its arrays) are built once, as a C++ caller holds them;
    # the timed region is the C-ABI call: validation, packing, transfers both ways, the kernels
    call = L.DenseBatchCall(big)
    for _ in range(args.warmup):
        call.run_raw()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call.run_raw()
    dt = time.perf_counter() - t0
    st, xs, obj = call.run()
    refb = ref[np.arange(batch) % count]
    rel = np.abs(obj - refb) / np.maximum(1.0, np.abs(refb))
    single = []
    for q in qps:
        t1 = time.perf_counter()
        s1, _, o1 = L.dense_qp_solve(**q)
        single.append(time.perf_counter() - t1)
    hist = {STATUS_NAMES.get(int(k), str(int(k))): int(v) for k, v in zip(*np.unique(st, return_counts=True))}
    line = {"metric": "dense_qps_per_sec", "value": batch * args.steps / dt, "unit": "QP/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "replicas",
            "vs_baseline": None, "dtype": "f64", "data": "golden QPs (tests/golden/golden_qps.npz)",
            "config": {"workload": f"generic dense path: {batch} QPs per call ({count} golden MPC-CBF QPs "
                                   "replicated), n=36, 30 equalities, host arrays in/out"},
            "status_hist": hist, "max_rel_obj_err_vs_golden": float(rel.max()),
            "single_qp_latency_ms": {"median": 1e3 * float(np.median(single)),
                                     "max": 1e3 * float(np.max(single))}}
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib as O
        big_ = np.finfo(np.float64).max
        oqs = [dict(n=q["c"].shape[0], H=q["H"], c=q["c"], A=q["A"], lo=q["lo"], hi=q["hi"],
                    vlo=np.full(q["c"].shape[0], -big_), vhi=np.full(q["c"].shape[0], big_)) for q in qps]
        n_cpu, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < 5.0:
            for q in oqs:
                O.solve_dense_qp(q)
            n_cpu += len(oqs)
        tc = time.perf_counter() - t1
        line["cpu_baseline"] = {"value": n_cpu / tc, "unit": "QP/s", "cores": 1, "kind": "port",
                                "sample": f"{n_cpu} solves of the {count} golden QPs (oracle dense "
                                          "Mehrotra PDIP + active-set polish)"}
    print(json.dumps(line), flush=True)


def workload_sizes(args, world: int, rank: int) -> tuple[int, int, int]:
    """Agents in total, agents per rank and this rank's first agent; fills in the defaults of
    --agents-total / --agents-per-gpu / --k-hor on args. N = 1: config 3 (4096 agents, horizon 15)
    or config 5's 512-agent per-GPU share (FoV, horizon 20). N > 1: config 4 (8192 agents in total)
    / config 5 (4096 FoV agents) sharded evenly over the ranks, unless --weak (per-GPU size kept)
    or an explicit size is given. --rank-share S times one rank's 1/S share on one GPU."""
    fov = args.workload == "fov"
    if world > 1 and not args.weak and args.agents_total <= 0 and args.agents_per_gpu <= 0:
        # BASELINE config 4 (8192 agents sharded over the node's GPUs) / config 5 (4096 FoV agents);
        # a rank count that does not divide it (3, 5, 6, 7) runs weak scaling at the per-GPU size
        cfg_total = 4096 if fov else 8192
        if cfg_total % world == 0:
            args.agents_total = cfg_total
        else:
            print(f"bench: {cfg_total} agents do not divide over {world} ranks; weak scaling at the "
                  "per-GPU size (give --agents-total for a strong-scaling line)", file=sys.stderr)
    if args.agents_per_gpu <= 0:
        args.agents_per_gpu = 512 if fov else 4096
    if args.k_hor <= 0:
        args.k_hor = 20 if fov else 15
    total = args.agents_total if args.agents_total > 0 else args.agents_per_gpu * world
    shares = world
    if args.rank_share > 0:
        assert world == 1, "--rank-share runs on one GPU"
        shares = args.rank_share
    per = total // shares
    assert per * shares == total, "agents must divide evenly over ranks"
    return total, per, rank * per


def main():
    args = parse()
    spawn_ranks(args)
    if args.workload == "dense":
        run_dense(args)
        return
    import torch
    import torch.distributed as dist
    from mpccbf import swarm, Context, Comm, comm_unique_id
    from mpccbf._lib import COMM_ID_BYTES
    from mpccbf.dist import SwarmShard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    fov = args.workload == "fov"
    total, per, first = workload_sizes(args, world, rank)
    slack = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=args.slack_decay) if args.slack else {}
    if fov:
        cfg = swarm.fov_config(args.k_hor, **slack)
        radius = cfg["fov_Rs"]  # observed neighbours: inside the FoV cone and the sensing range
        states_h, targets_h = swarm.heading_swarm(total)
        # 5 m lattice, sensing range 6 m: 1-3 observed neighbours per agent, steady closed loop
    else:
        cfg = swarm.config(args.k_hor, **slack)
        radius = 3.0 * cfg["d_min"]
        states_h, targets_h = swarm.lattice_swarm(total, spacing_scale=0.6 if args.crowded else 1.0)
    # neighbour-estimate covariances (FoV slack weights): the FoV example's 0.1 I for everyone
    cov_h = np.tile([0.1, 0.0, 0.1], (total, 1)) if (fov and args.slack) else None
    cov = None if cov_h is None else torch.tensor(cov_h, dtype=torch.float64, device=dev)
    ctx = Context(cfg, device=local, das_warm_steps=args.das_warm, lean=args.lean)
    ctx.set_variant(args.variant)

    targets = torch.tensor(targets_h[first:first + per], dtype=torch.float64, device=dev)
    out = ctx.alloc_outputs(per, device=dev)
    out.pop("next_states")  # written straight into the next state table
    nsteps = args.steps
    logs = [(torch.empty((nsteps, per, cfg["impc_iter"]), dtype=torch.int32, device=dev),
             torch.empty((nsteps, per, cfg["impc_iter"]), dtype=torch.int32, device=dev))
            for _ in range(2)]
    full0 = torch.tensor(states_h, dtype=torch.float64, device=dev)

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    replay_same = None
    trace_res = None
    nb_lists = {}
    if args.neighbours == "all":  # every other robot, as the reference hands them to optimize()
        rp_all = np.arange(per + 1, dtype=np.int32) * (total - 1)
        col_all = np.array([j for a in range(first, first + per) for j in range(total) if j != a], dtype=np.int32)
        nb_lists = dict(nb_row_ptr=torch.tensor(rp_all, device=dev), nb_col=torch.tensor(col_all, device=dev))
    if args.loop == "native" and args.neighbours in ("grid", "all"):
        # the whole closed loop in libmpccbf (mpccbf_run_steps): per step the fused IMPC kernel
        # (neighbour query, both IMPC QPs, next-step neighbour table) and, across ranks, one
        # in-place RCCL all-gather of agent states
        comm = None
        if world > 1:
            uid = torch.zeros(COMM_ID_BYTES, dtype=torch.uint8, device=dev)
            if rank == 0:
                uid.copy_(torch.tensor(list(comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(uid, 0)
            comm = Comm(bytes(uid.cpu().tolist()), world, rank, local)

        kc_waves = ctx.launch_waves(per)
        kclock = torch.zeros((nsteps, max(kc_waves, 1), 2), dtype=torch.int64, device=dev) if kc_waves else None

        def closed_loop(log, timing):
            """warm-up + nsteps control steps from the initial swarm; returns (seconds, run dict).
            timing=False: nothing but the steps on the stream (the throughput pass);
            timing=True: HIP events around every step and every IMPC kernel (the replay)."""
            tables = [full0.clone(), torch.empty_like(full0)]
            # the example's closed loop: fallback to the last successful trajectory, state noise
            # pos_std / vel_std of base_config.json physical_limits (example :150-221)
            traj_t = torch.full((per,), -1.0, dtype=torch.float64, device=dev)
            out["x"].fill_(float("nan"))
            nbsel = nb_lists or dict(knn_k=args.knn, knn_radius=radius)
            common = dict(targets=targets, agent_first=first, num_agents=per, x=out["x"], obj=out["obj"],
                          comm=comm, traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=20251015,
                          cov=cov, **nbsel)
            r = ctx.run_steps(tables[0], tables[1], args.warmup, status=out["status"],
                              iters=out["iters"], reserve_steps=nsteps, **common)
            if r["final"] is not tables[0]:
                tables.reverse()
            # (the timed steps continue the warm-up's closed loop: its last step's neighbour table
            # is the first timed step's, mpccbf_run::continue_tables). Their arguments are
            # marshalled here, before the timed region, which holds the C call alone — the
            # library's own host work (checks, table setup, launches) and the steps
            run = ctx.prepare_run_steps(tables[0], tables[1], nsteps, status_log=log[0], iters_log=log[1],
                                        timing=timing, solve_stride=1, step_index=args.warmup,
                                        kernel_clock=kclock if timing else None, continue_tables=True,
                                        **common)
            barrier_sync()
            t0 = time.perf_counter()
            e0.record()  # torch's current stream: the one run_steps launches on
            r = run()
            e1.record()
            barrier_sync()
            return time.perf_counter() - t0, r

        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        elapsed, _ = closed_loop(logs[0], timing=False)
        # device time of the timed region by HIP events at its two ends (no event between launches)
        region_ms = e0.elapsed_time(e1)
        # replay of the identical steps (same initial swarm, counter-based noise keyed by the step
        # index) with HIP events on the launch stream: per-step device time (p99), the events around
        # every IMPC launch, and each launch's own duration on the device clock (first-wave start to
        # last-wave end, s_memrealtime 100 MHz, mpccbf_run::kernel_clock; collision kernels only: the
        # FoV kernels carry none) — the clock's per-wave stores cost ~0.6 us per launch, so the
        # throughput pass carries neither
        _, rr = closed_loop(logs[1], timing=True)
        launch_us = None
        if kclock is not None:
            from mpccbf._lib import kernel_clock_us
            launch_us = kernel_clock_us(kclock.cpu().numpy())
            launch_us = launch_us if np.all(np.isfinite(launch_us)) else None
        step_ms, kern_ms = rr["step_ms"].astype(np.float64), rr["solve_ms"].astype(np.float64)
        replay_same = bool(torch.equal(logs[0][0], logs[1][0]) and torch.equal(logs[0][1], logs[1][1]))
        if world == 1 and not args.no_trace and args.rank_share <= 0:
            # the same closed loop once more, one step per call, every step's state table kept:
            # the trace the reference's collision_check.py scores (outside the timed region)
            tables = [full0.clone(), torch.empty_like(full0)]
            traj_t = torch.full((per,), -1.0, dtype=torch.float64, device=dev)
            out["x"].fill_(float("nan"))
            nt = args.warmup + nsteps
            trace_dev = torch.empty((nt + 1, total, 6), dtype=torch.float64, device=dev)
            trace_dev[0].copy_(tables[0])
            nbsel = nb_lists or dict(knn_k=args.knn, knn_radius=radius)
            common = dict(targets=targets, agent_first=first, num_agents=per, x=out["x"], obj=out["obj"],
                          traj_t=traj_t, pos_std=0.001, vel_std=0.01, noise_seed=20251015, cov=cov,
                          status=out["status"], iters=out["iters"], **nbsel)
            last_status = None
            for s in range(nt):
                r = ctx.run_steps(tables[0], tables[1], 1, step_index=s, **common)
                if r["final"] is not tables[0]:
                    tables.reverse()
                trace_dev[s + 1].copy_(tables[0])
                if s == nt - 1:
                    last_status = out["status"].clone()
            trace_h = trace_dev.cpu().numpy()
            trace_res = dict(traj=np.transpose(trace_h, (1, 0, 2)), last_status=last_status.cpu().numpy())
            del trace_dev
        if comm is not None:
            comm.close()
    else:
        # host-driven loop (one mpccbf_impc_solve per step; torch.distributed all-gather)
        shard = SwarmShard(full0, world, rank)
        nb_rp = torch.empty(per + 1, dtype=torch.int32, device=dev)
        nb_col = torch.empty(per * max(args.knn, 1), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream()

        def neighbours(states):
            if args.neighbours == "csr":
                ctx.build_neighbors(states, first, per, args.knn, radius, nb_rp, nb_col)
                return dict(nb_row_ptr=nb_rp, nb_col=nb_col)
            return dict(knn_k=args.knn, knn_radius=radius)

        def step(slot, kev_pair=None):
            states = shard.full
            nb = neighbours(states)
            st = logs[0][0][slot] if slot is not None else out["status"]
            it = logs[0][1][slot] if slot is not None else out["iters"]
            if kev_pair is not None:
                kev_pair[0].record(stream)
            ctx.impc_solve(states, targets=targets, agent_first=first, num_agents=per,
                           x=out["x"], status=st, obj=out["obj"], iters=it,
                           next_states=shard.next_out, cov=cov, **nb)
            if kev_pair is not None:
                kev_pair[1].record(stream)
            shard.publish()

        for _ in range(args.warmup):
            step(None)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(nsteps + 1)]
        kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(nsteps)]
        barrier_sync()
        t0 = time.perf_counter()
        ev[0].record(stream)
        for i in range(nsteps):
            step(i, kev[i])
            ev[i + 1].record(stream)
        barrier_sync()
        elapsed = time.perf_counter() - t0
        step_ms = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(nsteps)])
        kern_ms = np.array([a.elapsed_time(b) for a, b in kev])
        region_ms = None
        launch_us = None

    status = logs[0][0].cpu().numpy()
    iters = logs[0][1].cpu().numpy()
    if args.dump and rank == 0:
        extra = {}
        if trace_res is not None:  # every step's state table (warm-up steps first)
            extra = dict(traj=trace_res["traj"], warmup=args.warmup)
        np.savez_compressed(args.dump, status=status, iters=iters, kernel_ms=np.asarray(kern_ms), **extra)
    attempted = ~((status == 5) & (iters == 0))  # UNKNOWN with 0 steps: iteration not attempted
    hist = {name: int(np.sum((status == code) & attempted)) for code, name in STATUS_NAMES.items()}
    hist["not_attempted"] = int(np.sum(~attempted))
    rows = ctx.shared_rows  # CBF rows are few (filtered); counted as shared rows only
    kname = ctx.kernel_name
    if kname.startswith("impc_sep_kernel") or kname.startswith("impc_wide_kernel"):
        flops = flops_per_qp_sep(iters.reshape(-1), rows)
    else:
        flops = flops_per_qp(iters.reshape(-1), np.full(iters.size, rows), ctx.nz)
    # Newton steps per QP over the step index (the first steps from the lattice are the transient)
    att_it = np.where(attempted, iters, 0)
    newton_mean = att_it.sum(axis=(1, 2)) / np.maximum(attempted.sum(axis=(1, 2)), 1)
    newton_max = att_it.max(axis=(1, 2))

    vals = [elapsed, float(hist["OPTIMAL"]), float(hist["INFEASIBLE"]), float(hist["UNKNOWN"]),
            float(hist["ERROR"]), float(hist["not_attempted"]), flops, float(np.mean(kern_ms)),
            float(np.percentile(step_ms, 99)), float(np.max(kern_ms)), float(bool(replay_same) or replay_same is None),
            float(np.mean(launch_us)) if launch_us is not None else -1.0,
            float(np.max(launch_us)) if launch_us is not None else -1.0]
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        mn = t.clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        elapsed, kern_avg, p99, kern_max = float(mx[0]), float(mx[7]), float(mx[8]), float(mx[9])
        launch_avg, launch_max = float(mx[11]), float(mx[12])
        for i, k in enumerate(("OPTIMAL", "INFEASIBLE", "UNKNOWN", "ERROR", "not_attempted")):
            hist[k] = int(sm[1 + i])
        flops_rank0 = float(t[6])
        replay_same = bool(mn[10] > 0.5) if replay_same is not None else None
    else:
        kern_avg, p99, kern_max = vals[7], vals[8], vals[9]
        launch_avg, launch_max = vals[11], vals[12]
        flops_rank0 = flops
    nbk = total - 1 if args.neighbours == "all" else args.knn  # neighbours per agent (at most)
    # the dominant kernel's average duration per launch, in this order: the waves' own clock of the
    # timed pass (collision kernels: first wave start to last wave end); else, when a step is that
    # one launch (FoV on one GPU: no fallback, no foreign rows), the timed region per step (the
    # launches back to back); else HIP events around every launch of the replay. The events around
    # a launch hold its dispatch too (+4-5 us on config 3: kernel_event_bracket_avg_us)
    region_avg = (region_ms / nsteps) if region_ms is not None else None
    kern_bracket = kern_avg
    kern_src = "events"
    # (every other robot as a neighbour: the main launch defers nearly every agent to the capacity
    # launch, so the events around both are the step's kernel time)
    fb_launch = args.neighbours == "all"
    if launch_avg > 0 and not fb_launch:
        kern_avg, kern_max = launch_avg * 1e-3, launch_max * 1e-3
        kern_src = "clock"
    elif region_avg is not None and world == 1 and args.rank_share <= 0 and not fb_launch and \
            not kname.startswith("impc_wide_kernel"):
        kern_avg = region_avg
        kern_src = "region"

    if rank == 0:
        solved = hist["OPTIMAL"] + hist["INFEASIBLE"]
        attempted_n = solved + hist["UNKNOWN"] + hist["ERROR"]
        qps = solved / elapsed
        # roofline of the dominant kernel on rank 0: executed algorithmic flops per launch /
        # average launch time (HIP events on the launch stream, every step of the replay)
        flops_per_launch = flops_rank0 / nsteps
        achieved_tf = flops_per_launch / (kern_avg * 1e-3) / 1e12
        wl = ("fovs" if args.slack else "fov") if fov else "collision"
        traffic, traffic_src = pmc_traffic(kname, wl)
        # VALU issue: the kernel is bound by dependent-instruction latency at one wave per SIMD;
        # wave-level VALU instructions per launch (PMC SQ_INSTS_VALU) / launch time against the
        # issue peak (every SIMD one wave64 VALU op per 4 cycles: 1024 SIMDs x 2.4 GHz / 4)
        valu_insts, valu_src = pmc_lookup(kname, wl, "SQ_INSTS_VALU")
        abytes = algorithmic_bytes_per_agent(ctx.n, nbk, cfg["impc_iter"], cov is not None) * per
        # every IMPC kernel is bound by its agents' dependent instruction chains (latency at one or
        # a few waves per SIMD), not by MFMA, VALU throughput or HBM (the fractions below say how far)
        bound = "latency"
        res = {
            "metric": "QP solves/sec (whole node) + p99 step latency, N-agent horizon-15 MPC-CBF",
            "value": qps,
            "unit": "QP/s",
            "n_gpus": world,
            "steps": nsteps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / nsteps * 1e3,
            "p99_step_ms": p99,
            "higher_is_better": True,
            "scaling": "weak" if args.agents_total <= 0 else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (jittered-lattice swarm, seed 20251015); closed loop with the "
                     "example's trajectory fallback and state noise (pos 1e-3, vel 1e-2)"
                     if args.loop == "native" and args.neighbours in ("grid", "all") else
                     "synthetic (jittered-lattice swarm, seed 20251015); closed loop"),
            "config": {
                "workload": (
                    (f"config5: {total} agents ({per}/GPU), FoV 120 deg + Voronoi CBF, horizon "
                     f"{cfg['k_hor']}, 4 Bezier pieces, {args.knn} nearest observed within {radius:g} m"
                     if fov else
                     f"{'config4' if (world > 1 and total == 8192) else 'config3'}"
                     f"{' crowded (0.6 x spacing)' if args.crowded else ''}: {total} agents"
                     f"{f' sharded {world}xMI355X' if world > 1 else ''}, horizon "
                     f"{cfg['k_hor']}, pairwise collision CBF, "
                     + (f"every other robot as a neighbour ({total - 1}, fixed CSR lists)" if args.neighbours == "all"
                        else f"knn{args.knn} r={radius:g}m ({args.neighbours})"))
                    + (f", slack_mode (cost 1000, decay {args.slack_decay:g})" if args.slack else "")
                    + ", base_config.json; 2 IMPC QPs/agent/step"
                    + ("" if world == 1 else f"; {per}/GPU, RCCL all-gather of states")
                    + (f"; rank 0's share of {args.rank_share} ranks ({per} of {total} agents; the other rows carried "
                       "over and inserted into the neighbour table every step, the all-gather excluded)"
                       if args.rank_share > 0 else "")),
                "agents_total": total,
                "agents_per_gpu": per,
                "k_hor": cfg["k_hor"],
                "qp": {"n": ctx.n, "nz": ctx.nz, "shared_rows": ctx.shared_rows},
                "parallelism": f"dp{world}",
            },
            # value counts OPTIMAL and INFEASIBLE QPs (the latter certified by phase 1 and
            # oracle-confirmed on this workload, tests/test_gpu_status_parity.py); UNKNOWN / ERROR
            # are attempted but not counted
            "qps_solved": solved,
            "qps_attempted": attempted_n,
            "qps_optimal_frac": hist["OPTIMAL"] / max(attempted_n, 1),
            "status_hist": hist,
            "newton_steps_per_qp": ({"mean_by_step": [round(float(v), 3) for v in newton_mean],
                                     "max_by_step": [int(v) for v in newton_max],
                                     "kernel_us_by_step": [round(float(v) * 1e3, 1) for v in kern_ms]}
                                    if nsteps <= 64 else
                                    {"mean": float(np.mean(newton_mean)), "max": int(np.max(newton_max))}),
            "roofline": {
                "bound": bound,
                "achieved": achieved_tf,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / FP64_PEAK_TFLOPS,
                "traffic": traffic,
                "traffic_unit": "bytes/launch (HBM, PMC FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "traffic_source": traffic_src,
                "kernel": kname,
                "kernel_avg_us": kern_avg * 1e3,
                "kernel_max_us": kern_max * 1e3,
                "kernel_timing": {
                    "clock": "the waves themselves on every launch of an identical replay of the timed steps, "
                             "first wave start to last wave end (stores drained), s_memrealtime per wave "
                             "(mpccbf_run::kernel_clock): the launch without its dispatch and end-of-kernel "
                             "write-back, which rocprof's duration adds",
                    "region": "the timed region per step: one launch per step, back to back",
                    "events": "HIP events around every IMPC launch (they hold its dispatch too)"}[kern_src],
                "kernel_event_bracket_avg_us": kern_bracket * 1e3,
                "step_region_avg_us": None if region_avg is None else region_avg * 1e3,
                "step_region_timing": "HIP events at the two ends of the timed region divided by the steps "
                                      "(kernel + fallback / insert launches + dispatch gaps)",
                "replay_statuses_identical": bool(replay_same) if replay_same is not None else None,
                "flops_per_launch": flops_per_launch,
                "flops_model": "executed solver steps (dual active-set + PDIP Newton) x the FP64 flops "
                               "of an active-set step (bench.py flops_per_qp_sep, a lower bound); QPs "
                               "solved by the fast start count 0",
                "valu_issue": (None if valu_insts is None else {
                    "insts_per_launch": valu_insts,
                    "achieved_per_s": valu_insts / (kern_avg * 1e-3),
                    "peak_per_s": VALU_ISSUE_PEAK,
                    "frac": valu_insts / (kern_avg * 1e-3) / VALU_ISSUE_PEAK,
                    "source": valu_src}),
                "hbm": {"algorithmic_bytes_per_launch": abytes,
                        "achieved_gbs": abytes / (kern_avg * 1e-3) / 1e9,
                        "peak_gbs": HBM_PEAK_GBS,
                        "frac": abytes / (kern_avg * 1e-3) / 1e9 / HBM_PEAK_GBS},
            },
            "cpu_baseline": None,
        }
        if replay_same is False:
            res["roofline"]["kernel_timing"] += " (WARNING: replay statuses differ)"
        occ, occ_src = resource_lookup(kname, "occupancy")
        sq_wait, _ = pmc_lookup(kname, wl, "SQ_WAIT_ANY")
        sq_cyc, sq_src = pmc_lookup(kname, wl, "SQ_WAVE_CYCLES")
        res["roofline"]["occupancy_waves_per_simd"] = occ
        res["roofline"]["occupancy_source"] = occ_src
        res["roofline"]["sq_wait_frac"] = (sq_wait / sq_cyc) if (sq_wait is not None and sq_cyc) else None
        res["roofline"]["sq_wait_source"] = sq_src
        # FP64 the kernel issued (PMC: FMA x 2 + MUL + ADD + TRANS wave instructions x 64 lanes per
        # launch) against the vector FP64 peak over the launch: what the hardware executed,
        # assembly and outputs included, where `frac` counts the solver's algorithmic flops only
        f64 = [pmc_lookup(kname, wl, c)[0] for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                                      "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")]
        if all(v is not None for v in f64):
            issued = (2 * f64[0] + f64[1] + f64[2] + f64[3]) * 64
            res["roofline"]["fp64_issued"] = {
                "flops_per_launch": issued, "achieved_tflops": issued / (kern_avg * 1e-3) / 1e12,
                "frac": issued / (kern_avg * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                "source": pmc_lookup(kname, wl, "SQ_INSTS_VALU_FMA_F64")[1]}
        # the launch against its longest agent chain (stamps build: setup .. outputs of the slowest
        # agent, tools/stamp_profile.py): what a latency-bound launch cannot go below
        cp = critical_path_lookup(kname, wl, per)
        if cp is not None:
            res["roofline"]["critical_path"] = cp
        if trace_res is not None:
            res["closed_loop"] = closed_loop_metrics(trace_res, targets_h, cfg, fov)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(cfg, states_h, targets_h, args, radius, cov_h, trace_res)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_lookup(kname: str, workload: str, field: str):
    """Counter-derived `field` of kernel `kname` under `workload` ("collision", "fov", "fovs") from
    the newest committed PMC summary (profiles/r*_pmc_summary.json: rocprofv3 --pmc passes of
    this bench, gfx950-corrected by tools/pmc_summary.py). The counters cannot be read inside a
    timed run, so the value comes from the separate counter passes of the same command; the
    kernel's own name may carry defaulted template arguments (", false>"). (None, None) if absent."""
    import glob
    key = kname.replace(" ", "")

    def norm(n):
        return n.replace(" ", "").replace("void", "").replace("mpccbf::dev::", "")

    def match(name):
        n = norm(name)
        return n == key or (n.startswith(key[:-1] + ",") and n.endswith(">") and key.endswith(">"))

    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        tables = [d[workload]] if isinstance(d.get(workload), dict) else [d]
        for t in tables:
            for name, v in t.items():
                if isinstance(v, dict) and match(name) and field in v:
                    return float(v[field]), os.path.relpath(f, REPO)
    return None, None


def resource_lookup(kname: str, field: str):
    """`field` (vgpr, agpr, scratch, lds, occupancy) of kernel `kname` from the newest committed
    resource table (profiles/r*_resource_usage.txt, tools/resource_usage.py: hipcc
    -Rpass-analysis=kernel-resource-usage of the same sources). (None, None) if absent."""
    import glob
    cols = {"vgpr": 1, "agpr": 2, "scratch": 3, "lds": 4, "occupancy": 5}
    key = kname.replace(" ", "")
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_resource_usage.txt")), reverse=True):
        for ln in open(f):
            parts = ln.split()
            if len(parts) < 6:
                continue
            name = "".join(parts[:-5]).replace(" ", "")
            rest = name[len(key) - 1:-1].split(",")[1:] if key.endswith(">") and name.startswith(key[:-1] + ",") else None
            # exact, or the kernel's own name with defaulted template arguments (", false>")
            if name == key or (rest is not None and all(r == "false" for r in rest)):
                return int(parts[-6 + cols[field]]), os.path.relpath(f, REPO)
    return None, None


def closed_loop_metrics(tr, targets_h, cfg, fov):
    """The reference's post-processing checks (collision_check.py:48-80, mpccbf.metrics, shape =
    base_config.json's aligned_box [0.2, 0.2], goal radius 1 m) on the closed-loop trace (every
    control step of warm-up + timed steps), the smallest pair distance, and whether the last step's
    INFEASIBLE QPs are controller semantics: agents that entered the step within d_min of a
    neighbour (a CBF row no acceleration satisfies, ConnectivityIMPCCBF.cpp:199-211)."""
    from scipy.spatial import cKDTree
    from mpccbf import metrics
    traj = tr["traj"]
    ok, makespan, hit = metrics.instance_success_sparse(traj, targets_h, 1.0, [0.2, 0.2], "box")
    last_in = traj[:, -2, :2]  # the states the last step's QPs were built from
    d1, _ = cKDTree(last_in).query(last_in, k=2)
    within = d1[:, 1] < cfg["d_min"]
    infeas = tr["last_status"][:, 0] == 3
    return {
        "steps_traced": int(traj.shape[1] - 1),
        "instance_success": bool(ok),
        "makespan_steps": (None if makespan == float("inf") else int(makespan)),
        "first_collision": (None if hit is None else {"step": hit[0], "i": hit[1], "j": hit[2]}),
        "min_pair_distance_m": metrics.min_pair_distance_sparse(traj),
        "final_goal_reached_frac": float(np.mean(metrics.reach_goal_area(traj[:, -1, :2], targets_h[:, :2], 1.0))),
        "last_step_infeasible_agents": int(infeas.sum()),
        "last_step_infeasible_within_dmin": int((infeas & within).sum()),
        "last_step_agents_within_dmin": int(within.sum()),
        "shape": "box [0.2, 0.2] (base_config.json robot_params.collision_shape), goal radius 1 m",
    }


def critical_path_lookup(kname: str, workload: str, agents: int):
    """The slowest agent's stamped chain and the span of the stamped launch for `kname` at this
    agent count, from the newest committed profiles/r*_critical_path.json (tools/stamp_profile.py
    --json). None if absent."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_critical_path.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for e in d.get("entries", []):
            if e.get("kernel") == kname and e.get("workload", "collision") == workload and e.get("agents") == agents:
                return {"slowest_agent_chain_us": e["agent_wall_max_us"], "stamped_span_us": e["span_us"],
                        "agent_chain_mean_us": e["agent_wall_mean_us"], "phases_mean_us": e.get("phases_mean_us"),
                        "source": os.path.relpath(f, REPO)}
    return None


def pmc_traffic(kname: str, workload: str):
    """HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, KiB -> bytes) from the PMC summary."""
    return pmc_lookup(kname, workload, "hbm_bytes_per_launch_corrected")


def cpu_threads() -> tuple[int, int]:
    """(threads used, CPUs in this process's affinity set): the affinity set, capped by
    OMP_NUM_THREADS when set (the GPU box sets it to the job's CPU share, while its affinity set and
    os.cpu_count() show the whole machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, omp) if omp > 0 else aff), aff


def cpu_baseline(cfg, states_h, targets_h, args, radius, cov_h=None, trace=None):
    """The oracle (CPU restatement of the reference assembly + dense QP solve, standing in for
    CPLEX which cannot run here) timed on the states of the GPU's own timed steps: the closed-loop
    trace's state tables at up to 6 step indices spread over the timed range (its first and last
    step included), the whole swarm per sampled step on a thread pool (one agent per task, CPLEX
    Threads=1 per solve, CPLEX.cpp:118) — per-step wall times give the p99 step latency — plus one
    bounded single-thread sample (~5 s) of the first timed step. Without a trace (--no-trace,
    multi-rank shares) the initial swarm stands in and the line says so."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    from mpccbf import swarm
    p = O.make_params(cfg)
    refs = swarm.refs_from_targets(targets_h, cfg["k_hor"])
    n = len(states_h)

    def lists(st):
        if cfg.get("cbf_mode", 0) == 1:
            return swarm.fov_csr(st, args.knn, radius, cfg["fov_beta"])
        if args.neighbours == "all":
            rp_ = np.arange(n + 1, dtype=np.int32) * (n - 1)
            col_ = np.array([j for a in range(n) for j in range(n) if j != a], dtype=np.int32)
            return rp_, col_
        return swarm.knn_csr(st, args.knn, radius)

    # the timed steps' state tables: trace index s = the state the QPs of control step s are built from
    if trace is not None:
        nt = trace["traj"].shape[1] - 1
        first_t = args.warmup
        idx = sorted({int(round(v)) for v in np.linspace(first_t, nt - 1, num=min(6, nt - first_t))})
        tables = [(s, np.ascontiguousarray(trace["traj"][:, s, :])) for s in idx]
        src = f"states of timed control steps {idx} (closed-loop trace; timed range {first_t}..{nt - 1})"
    else:
        tables = [(0, np.ascontiguousarray(states_h))]
        src = "the initial swarm (no closed-loop trace in this run)"
    threads, aff = cpu_threads()
    step_ms, solved, total_s = [], 0, 0.0
    for s, st in tables:
        rp, col = lists(st)
        t = time.perf_counter()
        r = O.impc_batch(p, st, refs, rp, col, 0, n, threads, covs=cov_h)
        dt = time.perf_counter() - t
        step_ms.append(1e3 * dt)
        solved += r["solved"]
        total_s += dt
    # one thread on the first sampled step: a bounded sample sized for ~5 s
    s0, st0 = tables[0]
    rp, col = lists(st0)
    t = time.perf_counter()
    O.impc_batch(p, st0, refs, rp, col, 0, min(n, 32), 1, covs=cov_h)
    per = (time.perf_counter() - t) / min(n, 32)
    count = int(min(n, max(64, 5.0 / max(per, 1e-6))))
    t = time.perf_counter()
    r1 = O.impc_batch(p, st0, refs, rp, col, 0, count, 1, covs=cov_h)
    dt1 = time.perf_counter() - t
    model = ""
    try:
        model = next(ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": solved / total_s, "unit": "QP/s", "cores": threads, "kind": "port",
            "affinity_cpus": aff,
            "p99_step_ms": float(np.percentile(step_ms, 99)),
            "step_ms": [round(v, 2) for v in step_ms],
            "steps_sampled": [s for s, _ in tables],
            "single_core_value": r1["solved"] / dt1,
            "cpu": model,
            "sample": f"all {n} agents at each sampled step, {solved} QPs: {total_s:.2f} s on {threads} threads "
                      f"(one agent per task); {src}; 1 thread: first {count} agents of step {s0}, "
                      f"{r1['solved']} QPs in {dt1:.1f} s (oracle/ CPU restatement; CPLEX unavailable)"}


if __name__ == "__main__":
    main()
