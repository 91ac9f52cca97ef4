"""bench.py's workload sizing on CPU (no GPU, no library): the BASELINE configs each `--gpus N`
line runs. N = 1 -> config 3 (4096 agents) / config 5's 512-agent FoV share; N > 1 -> config 4
(8192 agents in total) / config 5 (4096 FoV agents) sharded evenly, strong scaling; --weak keeps
the per-GPU size; --rank-share S times one rank's share on one GPU."""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_sizes", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_collision_defaults(bench, world):
    a = bench.parse([])
    total, per, first = bench.workload_sizes(a, world, world - 1)
    assert a.k_hor == 15
    if world == 1:
        assert (total, per, first) == (4096, 4096, 0)
    else:
        assert total == 8192 and per == 8192 // world and first == (world - 1) * per


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_fov_defaults(bench, world):
    a = bench.parse(["--workload", "fov"])
    total, per, first = bench.workload_sizes(a, world, 0)
    assert a.k_hor == 20
    assert (total, per) == ((512, 512) if world == 1 else (4096, 4096 // world))


def test_weak_and_explicit_sizes(bench):
    a = bench.parse(["--weak"])
    assert bench.workload_sizes(a, 4, 2) == (16384, 4096, 8192)
    a = bench.parse(["--agents-per-gpu", "1000"])
    assert bench.workload_sizes(a, 2, 1) == (2000, 1000, 1000)
    a = bench.parse(["--agents-total", "6000"])
    assert bench.workload_sizes(a, 3, 2) == (6000, 2000, 4000)


def test_rank_share_and_uneven(bench):
    a = bench.parse(["--agents-total", "8192", "--rank-share", "8"])
    assert bench.workload_sizes(a, 1, 0) == (8192, 1024, 0)
    with pytest.raises(AssertionError):
        bench.workload_sizes(bench.parse(["--agents-total", "8192", "--rank-share", "8"]), 2, 0)
    with pytest.raises(AssertionError):
        bench.workload_sizes(bench.parse(["--agents-total", "1000"]), 3, 0)


@pytest.mark.parametrize("world", [3, 5, 6, 7])
def test_default_uneven_world_falls_back_to_weak(bench, world):
    a = bench.parse([])
    total, per, first = bench.workload_sizes(a, world, 1)
    assert (total, per, first) == (4096 * world, 4096, 4096) and a.agents_total <= 0
    a = bench.parse(["--workload", "fov"])
    assert bench.workload_sizes(a, world, 0)[:2] == (512 * world, 512)


def test_cpu_baseline_samples_timed_steps(bench, monkeypatch):
    """cpu_baseline times the oracle on the trace's state tables of the timed steps (first and last
    included), reports the per-step wall times, their p99 and the threads actually used."""
    import numpy as np
    from mpccbf import swarm
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(16)
    traj = np.repeat(states[:, None, :], 9, axis=1)  # warm-up 3 + 5 timed steps (+ the initial table)
    traj[:, :, 0] += np.arange(9)[None, :] * 0.01
    a = bench.parse(["--warmup", "3", "--steps", "5"])
    bench.workload_sizes(a, 1, 0)
    cb = bench.cpu_baseline(cfg, states, targets, a, 3.0 * cfg["d_min"], None, dict(traj=traj))
    assert cb["steps_sampled"][0] == 3 and cb["steps_sampled"][-1] == 7
    assert len(cb["step_ms"]) == len(cb["steps_sampled"])
    assert cb["cores"] == min(2, cb["affinity_cpus"])
    assert cb["p99_step_ms"] <= max(cb["step_ms"]) + 1e-9 and cb["value"] > 0
