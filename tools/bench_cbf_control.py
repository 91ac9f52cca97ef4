"""Throughput of the batched CBF-only controllers (not a BASELINE metric; reported in DESIGN.md):
FovControl (4096 agents, 8 observed neighbours max, plain and slack) and ConnectivityControl
(1024 teams of 8 robots, plain and slack). Device time per launch from HIP events.

    python tools/bench_cbf_control.py [reps]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import mpccbf  # noqa: E402
from mpccbf import swarm  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
t = lambda v, dt=torch.float64: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731


def timed(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = {}
# FovControl
n = 4096
cfg = swarm.fov_config(20)
states, targets = swarm.heading_swarm(n)
rng = np.random.default_rng(1)
desired = np.zeros((n, 3))
desired[:, :2] = 2.0 * (targets[:, :2] - states[:, :2]) + rng.uniform(-1, 1, (n, 2))
rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
nb_xy = states[col, :2]
cov = np.tile([0.1, 0.0, 0.1], (max(len(col), 1), 1))
u = torch.empty((n, 3), dtype=torch.float64, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
args = (t(states), t(desired), t(rp, torch.int32), t(nb_xy))
for slack in (False, True):
    c = dict(cfg, control_slack_mode=int(slack), slack_cost=1000.0, slack_decay_rate=0.9)
    ms = timed(lambda: mpccbf.fov_control_solve(c, *args, u, status=st, nb_cov=t(cov)))
    out[f"fov_control{'_slack' if slack else ''}"] = {
        "agents": n, "mean_neighbours": float(np.diff(rp).mean()), "ms_per_launch": ms,
        "QP_per_s": n / (ms * 1e-3), "optimal_frac": float((st == 0).float().mean())}
# ConnectivityControl: 1024 teams of 8
teams, size = 1024, 8
S = np.zeros((teams * size, 6))
for k in range(teams):
    S[k * size:(k + 1) * size, :2] = rng.uniform(-1.5, 1.5, (size, 2)) * (1.0 if k % 2 else 3.0)
    S[k * size:(k + 1) * size, 3:5] = rng.uniform(-0.3, 0.3, (size, 2))
ud = rng.uniform(-1, 1, (teams * size, 3))
ptr = np.arange(teams + 1, dtype=np.int32) * size
R = teams * size
u = torch.empty((R, 3), dtype=torch.float64, device=dev)
st = torch.empty(R, dtype=torch.int32, device=dev)
l2 = torch.empty(teams, dtype=torch.float64, device=dev)
cargs = (t(ptr, torch.int32), t(S), t(ud))
for slack in (False, True):
    c = dict(d_min=0.8, d_max=3.0, v_min=[-1, -1, -2.618], v_max=[1, 1, 2.618],
             control_slack_mode=int(slack), slack_cost=1e5, slack_decay_rate=0.1)
    ms = timed(lambda: mpccbf.connectivity_control_solve(c, *cargs, u, status=st, lambda2=l2))
    out[f"connectivity_control{'_slack' if slack else ''}"] = {
        "teams": teams, "robots_per_team": size, "ms_per_launch": ms, "QP_per_s": R / (ms * 1e-3),
        "optimal_frac": float((st == 0).float().mean()),
        "lambda2_branch_frac": float((l2 > 0.1).float().mean())}
print(json.dumps(out, indent=1))
