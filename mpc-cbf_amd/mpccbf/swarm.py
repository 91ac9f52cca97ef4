"""Synthetic agent swarms and the reference parameter set.

Parameters follow workspace/experiments/config/base_config.json (the only effective config:
experiments/python/preprocess.py:21 overwrites every other section with it), with k_hor
overridden per BASELINE.json config. Swarm shape follows BASELINE.md / SURVEY.md §8(d):
agents on a jittered square lattice (spacing 2.5*d_min, jitter U(+-0.25*d_min)), planar
velocities U(-0.5, 0.5) m/s, yaw and yaw rate 0, targets = position + U(disk of radius 3 m)
replicated over the horizon (MPCCBFFormationControl_example.cpp:143-144).
"""
from __future__ import annotations

import math

import numpy as np

SEED = 20251015

BASE_CONFIG = dict(
    h=0.1, Ts=0.01, k_hor=16, w_pos_err=10.0, w_u_eff=10.0, spd_f=8,
    v_min=[-2.0, -2.0, -2.6179938779914944], v_max=[2.0, 2.0, 2.6179938779914944],
    a_min=[-5.0, -5.0, -3.141592653589793], a_max=[5.0, 5.0, 3.141592653589793],
    d_min=2.0, cbf_horizon=2, impc_iter=2, slack_mode=0, slack_cost=50000.0,
    slack_decay_rate=0.1, num_pieces=3, num_control_points=4, piece_max_parameter=0.5,
    continuity_upto_degree=3,
    # FoV controller (BASELINE config 5): FovBezierIMPCCBF with fov 120 deg, Ds = aligned_box[0],
    # Rs = 3 d_min, robot box half extents (0.2, 0.2, 0)
    cbf_mode=0, fov_beta=2.0 * math.pi / 3.0, fov_Ds=0.2, fov_Rs=6.0, bbox=[0.2, 0.2, 0.0],
)


def fov_config(k_hor: int = 20, **over) -> dict:
    """BASELINE config 5: FoV controller, horizon 20 over 4 Bezier pieces (K h <= 4 x 0.5 s)."""
    return config(k_hor, cbf_mode=1, num_pieces=4, **over)


def config(k_hor: int, **over) -> dict:
    """base_config.json with k_hor overridden; validated like common/parsing.hpp:37-214."""
    cfg = dict(BASE_CONFIG)
    cfg["k_hor"] = int(k_hor)
    cfg.update(over)
    validate(cfg)
    return cfg


def validate(cfg: dict) -> None:
    h, Ts, K = cfg["h"], cfg["Ts"], cfg["k_hor"]
    if Ts > h:
        raise ValueError("Control timestep Ts must be <= MPC timestep h")
    if h <= 0 or Ts <= 0:
        raise ValueError("Time parameters h and Ts must be positive")
    if abs(h / Ts - round(h / Ts)) > 1e-10:
        raise ValueError("MPC timestep h must be an integer multiple of control timestep Ts")
    if cfg["spd_f"] > K:
        raise ValueError("Speed factor spd_f must be <= prediction horizon k_hor")
    if cfg["spd_f"] < 1:
        raise ValueError("Speed factor spd_f must be at least 1")
    if K < 1:
        raise ValueError("Prediction horizon k_hor must be at least 1")
    if cfg["cbf_horizon"] < 1:
        raise ValueError("CBF horizon must be at least 1")
    if cfg["impc_iter"] < 1:
        raise ValueError("IMPC iterations must be at least 1")
    if cfg["slack_mode"] and cfg["slack_cost"] <= 0:
        raise ValueError("Slack cost must be positive when slack_mode is enabled")
    if cfg["slack_mode"] and not (0 < cfg["slack_decay_rate"] <= 1):
        raise ValueError("Slack decay rate must be in (0,1] when slack_mode is enabled")
    if cfg["cbf_horizon"] > K:
        raise ValueError("CBF horizon must be <= MPC prediction horizon k_hor")
    if (K - 1) * h > cfg["num_pieces"] * cfg["piece_max_parameter"]:
        raise ValueError("MPC sampling range exceeds Bezier curve parameter range")


def lattice_swarm(n_agents: int, d_min: float = 2.0, seed: int = SEED, v_range: float = 0.5,
                  target_radius: float = 3.0, spacing_scale: float = 1.0):
    """Returns states (N, 6) = [px, py, yaw, vx, vy, vyaw] and targets (N, 3). Lattice spacing
    2.5 d_min and jitter +-0.25 d_min, both times spacing_scale (< 1: a crowded swarm)."""
    rng = np.random.default_rng(seed)
    side = int(math.ceil(math.sqrt(n_agents)))
    spacing = 2.5 * d_min * spacing_scale
    idx = np.arange(n_agents)
    gx = (idx % side).astype(np.float64) * spacing
    gy = (idx // side).astype(np.float64) * spacing
    jit = rng.uniform(-0.25 * d_min * spacing_scale, 0.25 * d_min * spacing_scale, size=(n_agents, 2))
    states = np.zeros((n_agents, 6))
    states[:, 0] = gx + jit[:, 0]
    states[:, 1] = gy + jit[:, 1]
    states[:, 3:5] = rng.uniform(-v_range, v_range, size=(n_agents, 2))
    r = target_radius * np.sqrt(rng.uniform(0, 1, n_agents))
    th = rng.uniform(0, 2 * math.pi, n_agents)
    targets = np.zeros((n_agents, 3))
    targets[:, 0] = states[:, 0] + r * np.cos(th)
    targets[:, 1] = states[:, 1] + r * np.sin(th)
    return states, targets


def refs_from_targets(targets: np.ndarray, k_hor: int) -> np.ndarray:
    """target.replicate(k_hor, 1) per agent (MPCCBFFormationControl_example.cpp:143-144)."""
    return np.tile(targets, (1, k_hor))


def knn_csr(states: np.ndarray, k: int, radius: float):
    """CPU reference neighbour lists: the k nearest (planar) within radius, excluding self.
    Ties broken by index. Returns (row_ptr, col) int32."""
    p = states[:, :2]
    n = len(p)
    rows = []
    for i in range(n):
        d2 = np.sum((p - p[i]) ** 2, axis=1)
        d2[i] = np.inf
        cand = np.nonzero(d2 <= radius * radius)[0]
        order = np.lexsort((cand, d2[cand]))[:k]
        rows.append(np.sort(cand[order]))
    row_ptr = np.zeros(n + 1, dtype=np.int32)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32) if row_ptr[-1] else np.zeros(0, np.int32)
    return row_ptr, col


def fov_csr(states: np.ndarray, k: int, radius: float, fov: float):
    """Neighbour lists for the FoV controller: the k nearest agents (planar) within `radius` whose
    bearing lies strictly inside the ego's field of view (|bearing - yaw| < fov / 2), i.e. the
    robots it can observe. Ties by index; rows sorted by index. Returns (row_ptr, col)."""
    p = states[:, :2]
    n = len(p)
    rows = []
    for i in range(n):
        d = p - p[i]
        d2 = np.sum(d ** 2, axis=1)
        d2[i] = np.inf
        bearing = np.arctan2(d[:, 1], d[:, 0]) - states[i, 2]
        off = np.abs(np.angle(np.exp(1j * bearing)))
        cand = np.nonzero((d2 <= radius * radius) & (off < 0.5 * fov))[0]
        order = np.lexsort((cand, d2[cand]))[:k]
        rows.append(np.sort(cand[order]))
    row_ptr = np.zeros(n + 1, dtype=np.int32)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32) if row_ptr[-1] else np.zeros(0, np.int32)
    return row_ptr, col


def heading_swarm(n_agents: int, d_min: float = 2.0, seed: int = SEED, speed: float = 0.3,
                  target_dist: float = 3.0):
    """Swarm for the FoV controller: lattice positions as lattice_swarm, every agent with a random
    heading, moving along it at `speed`, with its target ahead (within +-30 deg of the heading,
    up to `target_dist`), so the robots it observes can stay in view while it travels."""
    states, targets = lattice_swarm(n_agents, d_min, seed)
    rng = np.random.default_rng(seed + 1)
    yaw = rng.uniform(-math.pi, math.pi, n_agents)
    states[:, 2] = yaw
    states[:, 3] = speed * np.cos(yaw)
    states[:, 4] = speed * np.sin(yaw)
    ang = yaw + rng.uniform(-math.pi / 6, math.pi / 6, n_agents)
    r = target_dist * np.sqrt(rng.uniform(0.25, 1.0, n_agents))
    targets[:, 0] = states[:, 0] + r * np.cos(ang)
    targets[:, 1] = states[:, 1] + r * np.sin(ang)
    targets[:, 2] = yaw
    return states, targets


def all_csr(n: int):
    """Reference semantics: every other agent is a neighbour (ConnectivityIMPCCBF.cpp:59-67)."""
    row_ptr = (np.arange(n + 1) * (n - 1)).astype(np.int32)
    col = np.concatenate([np.delete(np.arange(n), i) for i in range(n)]).astype(np.int32) \
        if n > 1 else np.zeros(0, np.int32)
    return row_ptr, col
