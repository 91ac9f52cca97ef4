"""Appends the FoV slack-mode failures captured by tools/fov_status_check.py (MPCCBF_CHECK_SLACK=1,
1000 closed-loop steps of 512 agents; the run's .npz holds each mismatching step's state table) to
regress_cases.json: ego state + its observed neighbours (fov_csr, the oracle's list) + target.
Round 2's records (profiles/r02_fovs_status.log) and this round's capture show the same two
agent-steps: iteration 1 UNKNOWN on the GPU (slack-pattern active set and slack PDIP alike), the
oracle OPTIMAL with a slack of ~10 (cost 1000) on one neighbour.

    python tests/golden/add_fov_slack_regressions.py gpurun_out/<tag>/fovs_status.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "mpc-cbf_amd"))
from mpccbf import swarm  # noqa: E402

CASES = [(6, 223), (8, 83)]


def main(path):
    d = np.load(path)
    cfg = swarm.fov_config(20, slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9)
    out = json.load(open(os.path.join(HERE, "regress_cases.json")))
    names = {c["name"] for c in out["cases"]}
    for step, a in CASES:
        name = f"config5_slack_step{step}_agent{a}"
        if name in names:
            continue
        states = d[f"states_{step}"]
        rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
        nb = [int(j) for j in col[rp[a]:rp[a + 1]]]
        out["cases"].append({
            "name": name, "controller": "fov_slack", "k_hor": 20,
            "slack_cost": 1000.0, "slack_decay_rate": 0.9, "cov": [0.1, 0.0, 0.1],
            "note": (f"FoV slack closed loop (tools/fov_status_check.py, 512 agents, heading swarm) step "
                     f"{step}: IMPC iteration 1 UNKNOWN on the GPU, OPTIMAL in the oracle with one neighbour's "
                     "slack near 10 (cost 1000); row 0 = ego, rows 1.. = its observed neighbours"),
            "states": [states[a].tolist()] + [states[j].tolist() for j in nb],
            "target": d["targets"][a].tolist(),
        })
    json.dump(out, open(os.path.join(HERE, "regress_cases.json"), "w"), indent=1)
    print("cases:", [c["name"] for c in out["cases"]])


if __name__ == "__main__":
    main(sys.argv[1])
