"""Safety / goal metrics of a closed-loop run: the checks of the reference's post-processing script
(workspace/experiments/python/metrics/collision_check.py:11-80), restated on numpy arrays with the
same semantics, so a trace from mpccbf.sim (or the example's states.json) is scored as the
reference scores it.
"""
from __future__ import annotations

import numpy as np


def rectangles_collide(xA, yA, wA, hA, xB, yB, wB, hB):
    """Overlap of two axis-aligned rectangles given by a corner and extents (:11-20)."""
    return (xA < xB + wB) & (xA + wA > xB) & (yA < yB + hB) & (yA + hA > yB)


def collision_check(x1, y1, x2, y2, collision_shape, shape_type):
    """(:22-41) circle: centres within two radii; box: the script's rectangle test (corner at
    centre - half / 2, extent 2 x half). Vectorised over array arguments."""
    if shape_type == "circle":
        return np.hypot(x2 - x1, y2 - y1) <= 2 * collision_shape
    if shape_type == "box":
        cx, cy = collision_shape[0], collision_shape[1]
        return rectangles_collide(x1 - cx / 2, y1 - cy / 2, 2 * cx, 2 * cy,
                                  x2 - cx / 2, y2 - cy / 2, 2 * cx, 2 * cy)
    raise ValueError(f"Unknown shape_type: {shape_type}")


def reach_goal_area(pos, goal, radius=1.0):
    """(:44-46) planar distance to the goal within radius."""
    return np.linalg.norm(np.asarray(pos) - np.asarray(goal), axis=-1) <= radius


def instance_success(traj, goals, radius, collision_shape, shape_type):
    """(:48-80) traj: [n_robot, ts, >= 3]. Walks the time steps: returns (True, max(0, t - 1)) at
    the first step where every robot has reached its goal area, (False, inf) at the first
    colliding pair, else (True, ts). Returns also the first collision (t, i, j) or None."""
    traj = np.asarray(traj, dtype=np.float64)
    goals = np.asarray(goals, dtype=np.float64)
    n, ts = traj.shape[0], traj.shape[1]
    reached = np.zeros(n, dtype=bool)
    iu, ju = np.triu_indices(n, k=1)
    for t in range(ts):
        if reached.all():
            return True, max(0, t - 1), None
        p = traj[:, t, :2]
        reached |= reach_goal_area(p, goals[:, :2], radius)
        hit = collision_check(p[iu, 0], p[iu, 1], p[ju, 0], p[ju, 1], collision_shape, shape_type)
        if np.any(hit):
            k = int(np.argmax(hit))  # first pair in the script's (i, j) order
            return False, float("inf"), (t, int(iu[k]), int(ju[k]))
    return True, ts, None


def instance_success_sparse(traj, goals, radius, collision_shape, shape_type):
    """instance_success for large swarms: the same walk and the same result, with each step's
    colliding pairs found among the pairs a k-d tree returns within the largest distance at which
    the shape test can hold (circle: 2 r; box: centre offsets below 2 x half on both axes, so
    within 2 |half|), so a step costs
    O(n log n) instead of the script's O(n^2)."""
    from scipy.spatial import cKDTree
    traj = np.asarray(traj, dtype=np.float64)
    goals = np.asarray(goals, dtype=np.float64)
    n, ts = traj.shape[0], traj.shape[1]
    if shape_type == "circle":
        reach = 2.0 * float(collision_shape) * (1.0 + 1e-12)
    else:
        reach = 2.0 * float(np.hypot(collision_shape[0], collision_shape[1])) * (1.0 + 1e-12)
    reached = np.zeros(n, dtype=bool)
    for t in range(ts):
        if reached.all():
            return True, max(0, t - 1), None
        p = traj[:, t, :2]
        reached |= reach_goal_area(p, goals[:, :2], radius)
        pairs = cKDTree(p).query_pairs(reach, output_type="ndarray")
        if len(pairs):
            i, j = pairs.min(axis=1), pairs.max(axis=1)
            hit = collision_check(p[i, 0], p[i, 1], p[j, 0], p[j, 1], collision_shape, shape_type)
            if np.any(hit):
                k = np.lexsort((j[hit], i[hit]))[0]  # first pair in the script's (i, j) order
                return False, float("inf"), (t, int(i[hit][k]), int(j[hit][k]))
    return True, ts, None


def min_pair_distance_sparse(traj):
    """min_pair_distance through a k-d tree per step (large swarms)."""
    from scipy.spatial import cKDTree
    traj = np.asarray(traj, dtype=np.float64)
    best = np.inf
    for t in range(traj.shape[1]):
        d, _ = cKDTree(traj[:, t, :2]).query(traj[:, t, :2], k=2)
        best = min(best, float(d[:, 1].min()))
    return best


def min_pair_distance(traj):
    """Smallest planar distance between two robots over the run (a safety margin summary)."""
    traj = np.asarray(traj, dtype=np.float64)
    best = np.inf
    for t in range(traj.shape[1]):
        p = traj[:, t, :2]
        d = np.sqrt(np.sum((p[:, None, :] - p[None, :, :]) ** 2, axis=-1))
        np.fill_diagonal(d, np.inf)
        best = min(best, float(d.min()))
    return best


def trajectories_from_states_json(states_json: dict) -> np.ndarray:
    """[n_robot, ts, 6] from a states.json (collision_check.py:94)."""
    robots = states_json["robots"]
    return np.array([robots[str(i)]["states"] for i in range(len(robots))])
