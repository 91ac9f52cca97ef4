"""Closed-loop safety of the two update orders (diagnostics, GPU): the bench's lattice swarm (256
agents by default, knn 8 within 6 m, noise as the bench) run for S control steps with the batched
Jacobi sweep (the product path) and with the reference example's Gauss-Seidel order
(MPCCBFFormationControl_example.cpp:140-201, one launch per robot), scored by the reference's
collision_check.py metrics (mpccbf.metrics) — whether the collisions of the bench trace are the
controller's or the ordering's.

    python tools/order_compare.py [agents] [steps] [out.json] [--crowded]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-cbf_amd"))
from mpccbf import metrics, sim, swarm  # noqa: E402


def run(order, n, steps, crowded):
    cfg = swarm.config(15)
    states, targets = swarm.lattice_swarm(n, spacing_scale=0.6 if crowded else 1.0)
    s = sim.Simulator(cfg, states, targets, knn_k=8, knn_radius=6.0, pos_std=0.001, vel_std=0.01,
                      noise_seed=20251015, record=False, order=order)
    tr = [s.states.cpu().numpy().copy()]
    for _ in range(steps):
        s.step()
        tr.append(s.states.cpu().numpy().copy())
    traj = np.transpose(np.array(tr), (1, 0, 2))
    st = np.array(s.status_log)
    ok, makespan, hit = metrics.instance_success_sparse(traj, targets, 1.0, [0.2, 0.2], "box")
    return {"order": order, "agents": n, "steps": steps, "crowded": crowded,
            "instance_success": bool(ok),
            "first_collision": None if hit is None else {"step": int(hit[0]), "i": int(hit[1]), "j": int(hit[2])},
            "min_pair_distance_m": float(metrics.min_pair_distance_sparse(traj)),
            "final_goal_reached_frac": float(np.mean(metrics.reach_goal_area(traj[:, -1, :2], targets[:, :2], 1.0))),
            "infeasible_qps": int(np.sum(st == 3)), "optimal_qps": int(np.sum(st == 0)),
            "last_step_infeasible_agents": int(np.sum(st[-1, :, 0] == 3))}


if __name__ == "__main__":
    av = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(av[0]) if av else 256
    steps = int(av[1]) if len(av) > 1 else 300
    crowded = "--crowded" in sys.argv
    res = [run(o, n, steps, crowded) for o in ("jacobi", "gauss_seidel")]
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(av) > 2:
        open(av[2], "w").write(txt)
