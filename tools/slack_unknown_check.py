"""Oracle verdict on the non-OPTIMAL QPs of the all-neighbour slack stress line (diagnostics, CPU):
reads a `bench.py --neighbours all --crowded --slack --dump f.npz` dump (statuses of the timed
steps and every step's state table), re-solves every agent-step whose IMPC statuses are not all
OPTIMAL with the CPU oracle on the same states (every other robot as a neighbour), and prints
both verdicts side by side.

    python tools/slack_unknown_check.py gpurun_out/all256s.npz [--agents 256] [--decay 0.9]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--agents", type=int, default=256)
    ap.add_argument("--decay", type=float, default=0.9)
    a = ap.parse_args()
    import oracle_lib as O
    from mpccbf import swarm
    d = np.load(a.npz)
    status, traj, warm = d["status"], d["traj"], int(d["warmup"])
    cfg = swarm.config(15, slack_mode=1, slack_cost=1000.0, slack_decay_rate=a.decay)
    p = O.make_params(cfg)
    _, targets = swarm.lattice_swarm(a.agents, spacing_scale=0.6)
    refs = swarm.refs_from_targets(targets, cfg["k_hor"])
    bad = np.argwhere(np.any(status != 0, axis=2))
    print(f"{len(bad)} agent-steps not OPTIMAL in every IMPC iteration")
    for s, ag in bad:
        states = traj[:, warm + s, :]
        nb = np.array([j for j in range(a.agents) if j != ag], dtype=np.int32)
        r = O.impc_optimize(p, states, int(ag), nb, refs[ag])
        print(f"step {s} agent {ag}: GPU {status[s, ag].tolist()}  oracle {r['status'].tolist()} "
              f"obj {r['obj'].tolist()}", flush=True)


if __name__ == "__main__":
    main()
