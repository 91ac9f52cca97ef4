"""Appends the two all-neighbour slack QPs that ended UNKNOWN in round 3 to regress_cases.json
(collision controller, slack_mode, every other robot as a neighbour): step 100 agent 87 and step 143
agent 52 of `bench.py --neighbours all --crowded --slack --steps 200 --warmup 20 --dump all256s.npz`
(256 agents; the dump's state table of that step). Row 0 = the ego, rows 1.. = every other robot in
index order (its neighbour list). Round 3: GPU [OPTIMAL, UNKNOWN], oracle [UNKNOWN, UNKNOWN]; the
oracle's exact presolves (box-implied slack rows dropped, idle slack columns fixed at 0) solve both.

    python tests/golden/add_slack_all_regressions.py gpurun_out/all256s.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "mpc-cbf_amd"))
from mpccbf import swarm  # noqa: E402

d = np.load(sys.argv[1])
traj, warm = d["traj"], int(d["warmup"])
_, targets = swarm.lattice_swarm(256, spacing_scale=0.6)
path = os.path.join(HERE, "regress_cases.json")
js = json.load(open(path))
names = {c["name"] for c in js["cases"]}
for s, ag in ((100, 87), (143, 52)):
    name = f"all256_slack_step{s}_agent{ag}"
    if name in names:
        continue
    st = traj[:, warm + s, :]
    order = [ag] + [j for j in range(256) if j != ag]
    js["cases"].append({
        "name": name, "controller": "collision_slack", "k_hor": 15, "slack_cost": 1000.0,
        "slack_decay_rate": 0.9,
        "note": f"--neighbours all --crowded --slack stress line, step {s}: agent {ag} against every other "
                "robot (255 slack variables, weights 1000 * 0.9^rank down to ~2e-9). Round 3: GPU "
                "[OPTIMAL, UNKNOWN], oracle [UNKNOWN, UNKNOWN].",
        "states": st[order].tolist(), "target": targets[ag].tolist()})
json.dump(js, open(path, "w"), indent=1)
print(len(js["cases"]), "cases")
