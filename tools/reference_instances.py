"""Run the reference's 16 baseline instances (tests/golden/reference_instances.json) through the
closed-loop simulator as the reference runs them (base_config.json overlay, zero start velocity,
every other robot a neighbour, Gauss–Seidel order, the example's sim_runtime default of 40 s =
400 control steps) and score each trace with the reference's collision_check.py metrics
(mpccbf.metrics: instance_success with the aligned box, goal radius 1). Writes one JSON object.

usage: python tools/reference_instances.py [--runtime 40] [--out profiles/r05_reference_instances.json]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-cbf_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runtime", type=float, default=40.0)
    ap.add_argument("--order", default="gauss_seidel")
    ap.add_argument("--out", default="")
    ap.add_argument("--modes", default="base,own")
    ap.add_argument("--only", default="", help="comma-separated instance names (default: all 16)")
    args = ap.parse_args()
    from mpccbf import instances, metrics, sim

    res = {"runtime_s": args.runtime, "order": args.order, "neighbours": "all N-1",
           "modes": {"base": "base_config.json overlaid (preprocess.py:21): the reference's runs",
                     "own": "the instance file's own parameters, missing keys from the base config"},
           "instances": {}}
    names = args.only.split(",") if args.only else instances.names()
    for mode, name in [(m, nm) for m in args.modes.split(",") for nm in names]:
        cfg, states, targets, shape, kind, noise = instances.instance(name, preprocess=mode)
        t0 = time.perf_counter()
        try:
            s = sim.Simulator(cfg, states, targets, neighbours="all", order=args.order, record=True,
                              noise_seed=20251015, **noise)
            s.run(args.runtime)
        except Exception as e:  # (a parameter set outside the kernels' capacity: recorded, not run)
            res["instances"][f"{name} ({mode})"] = {"robots": len(states), "error": str(e),
                                                    "params": {k: cfg[k] for k in ("k_hor", "num_pieces",
                                                                                   "num_control_points", "cbf_horizon",
                                                                                   "d_min")}}
            print(name, mode, "error:", e, flush=True)
            continue
        wall = time.perf_counter() - t0
        traj = metrics.trajectories_from_states_json(s.states_json())
        ok, makespan, hit = metrics.instance_success(traj, targets, 1.0, shape, kind)
        st = np.array(s.status_log)
        fin = np.linalg.norm(traj[:, -1, :2] - targets[:, :2], axis=1)
        # first step at which some robot's iteration-0 QP turns from OPTIMAL to INFEASIBLE
        tr = np.argwhere((st[:-1, :, 0] == 0) & (st[1:, :, 0] == 3))
        r = {"robots": len(states), "steps": len(st), "success": bool(ok),
             "first_opt_to_infeasible_step": int(tr[0, 0] + 1) if len(tr) else None,
             "makespan_records": None if not np.isfinite(makespan) else int(makespan),
             "first_collision": hit, "min_pair_distance_m": metrics.min_pair_distance(traj),
             "goals_reached_at_end": int(np.sum(fin <= 1.0)), "max_final_goal_dist_m": float(fin.max()),
             "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
             "wall_s": round(wall, 2)}
        res["instances"][f"{name} ({mode})"] = r
        print(name, mode, json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
