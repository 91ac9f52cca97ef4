"""World-size-2 CPU rehearsal of the multi-GPU path (gloo backend, two processes).

The swarm is sharded in contiguous agent blocks (mpccbf.dist.SwarmShard); each control step
all-gathers the agent states, each rank solves its own block, and the closed-loop update writes
its local states. The solver here is the CPU oracle (test infrastructure) in place of the GPU
kernel: what is under test is the sharding / exchange logic that bench.py runs over RCCL, which
must reproduce the single-process closed loop bit for bit.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

import oracle_lib as O
from mpccbf import swarm
from mpccbf.dist import SwarmShard, shard

TOTAL = 48
STEPS = 3


def _oracle_solver(cfg, targets):
    p = O.make_params(cfg)
    refs = swarm.refs_from_targets(targets, cfg["k_hor"])

    def solve(full, first, count, out):
        S = full.numpy().copy()
        rp, col = swarm.knn_csr(S, 8, 3 * cfg["d_min"])
        r = O.impc_batch(p, S, refs, rp, col, first, count, 1)
        nxt = S[first:first + count].copy()
        for i in range(count):
            if np.any(r["status"][i] == O.OPTIMAL):  # closed-loop update: kept curve at t = h
                nxt[i, :3] = O.eval_curve(p, r["x_last"][i], cfg["h"], 0)
                nxt[i, 3:] = O.eval_curve(p, r["x_last"][i], cfg["h"], 1)
        out.copy_(torch.tensor(nxt))

    return solve


def _run(world, rank):
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(TOTAL)
    states[:, :2] *= 0.6  # close spacing: CBF rows active, some agents infeasible
    sh = SwarmShard(torch.tensor(states), world, rank)
    solve = _oracle_solver(cfg, targets)
    for _ in range(STEPS):
        sh.step(solve)
    return sh.full.numpy().copy()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = _run(world, rank)
        q.put((rank, full))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_ranges():
    assert [shard(8192, 8, r) for r in (0, 7)] == [(0, 1024), (7168, 1024)]
    with pytest.raises(ValueError):
        shard(10, 4, 0)


def test_two_rank_closed_loop_matches_single_process():
    ref = _run(1, 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, full = q.get(timeout=240)
        got[r] = full
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank ends with the same gathered table, equal to the single-process loop
    np.testing.assert_array_equal(got[0], got[1])
    np.testing.assert_array_equal(got[0], ref)
    assert not np.array_equal(ref, swarm.lattice_swarm(TOTAL)[0])  # the swarm actually moved
