"""The collision / goal metrics restated from collision_check.py:11-80 (mpccbf.metrics), on
hand-built trajectories whose outcome is known."""
import numpy as np

from mpccbf import metrics


def _traj(paths):
    return np.array(paths, dtype=np.float64)


def test_circle_and_box_collision_rules():
    # circle: centres within 2 r
    assert metrics.collision_check(0.0, 0.0, 0.39, 0.0, 0.2, "circle")
    assert not metrics.collision_check(0.0, 0.0, 0.41, 0.0, 0.2, "circle")
    # box (the script's rectangle: corner at centre - half/2, extent 2 x half): overlap iff the
    # centre offset is below 2 x half on both axes
    assert metrics.collision_check(0.0, 0.0, 0.39, 0.39, [0.2, 0.2], "box")
    assert not metrics.collision_check(0.0, 0.0, 0.41, 0.0, [0.2, 0.2], "box")
    assert not metrics.collision_check(0.0, 0.0, 0.0, 0.40, [0.2, 0.2], "box")


def test_instance_success_reaches_goals_without_collision():
    # two robots walking to their goals on parallel lines 2 m apart
    t = np.linspace(0.0, 1.0, 11)
    r0 = np.stack([5 * t, 0 * t, 0 * t], axis=1)
    r1 = np.stack([5 * t, 0 * t + 2.0, 0 * t], axis=1)
    ok, makespan, hit = metrics.instance_success(_traj([r0, r1]), [[5, 0, 0], [5, 2, 0]], 1.0, 0.2, "circle")
    assert ok and hit is None
    # both inside the 1 m goal area from step 8 (x = 4.0, distance 1.0 <= 1): the all-reached
    # test at the start of step 9 returns 9 - 1
    assert makespan == 8


def test_instance_success_reports_first_collision():
    t = np.linspace(0.0, 1.0, 11)
    r0 = np.stack([4 * t, 0 * t, 0 * t], axis=1)
    r1 = np.stack([4 - 4 * t, 0 * t, 0 * t], axis=1)  # head-on: they meet at t = 0.5
    r2 = np.stack([0 * t, 0 * t + 9.0, 0 * t], axis=1)
    ok, makespan, hit = metrics.instance_success(_traj([r0, r1, r2]), [[4, 0, 0], [0, 0, 0], [0, 9, 0]],
                                                 1.0, [0.2, 0.2], "box")
    assert not ok and makespan == float("inf")
    assert hit == (5, 0, 1)
    assert metrics.min_pair_distance(_traj([r0, r1])) == 0.0


def test_goal_not_reached_runs_to_the_end():
    t = np.linspace(0.0, 1.0, 5)
    r0 = np.stack([t, 0 * t, 0 * t], axis=1)
    ok, makespan, _ = metrics.instance_success(_traj([r0]), [[9, 9, 0]], 1.0, 0.2, "circle")
    assert ok and makespan == 5


def test_sparse_metrics_equal_the_script_form():
    """instance_success_sparse / min_pair_distance_sparse (k-d tree pairs, used on bench-size
    swarms) return exactly what the script-form O(n^2) walk returns, for both shapes, on random
    crowded trajectories with and without collisions."""
    rng = np.random.default_rng(3)
    for trial in range(12):
        n, ts = 40, 15
        start = rng.uniform(0, 6, (n, 2))
        goal = rng.uniform(0, 6, (n, 2))
        w = np.linspace(0.0, 1.0, ts)[None, :, None]
        traj = np.concatenate([start[:, None, :] * (1 - w) + goal[:, None, :] * w, np.zeros((n, ts, 1))], axis=2)
        goals = np.concatenate([goal, np.zeros((n, 1))], axis=1)
        for shape, kind in ((0.2, "circle"), ([0.2, 0.2], "box"), ([0.05, 0.3], "box")):
            a = metrics.instance_success(traj, goals, 1.0, shape, kind)
            b = metrics.instance_success_sparse(traj, goals, 1.0, shape, kind)
            assert a == b, (trial, kind, a, b)
        assert metrics.min_pair_distance(traj) == metrics.min_pair_distance_sparse(traj)
