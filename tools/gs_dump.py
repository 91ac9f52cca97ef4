"""Gauss-Seidel closed loop of tests/test_gpu_sim.py::test_gauss_seidel_trace_matches_oracle on the
device, dumped for a CPU-side look at single updates: the state trace, statuses, control points and
objectives of every step.   python tools/gs_dump.py <knn|all> out.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-cbf_amd"))
from mpccbf import sim, swarm  # noqa: E402

nb = sys.argv[1]
cfg = swarm.config(15)
n, steps = (64, 30) if nb == "knn" else (24, 20)
states, targets = swarm.lattice_swarm(n, seed=21)
states[:, :2] *= 0.6
kw = dict(pos_std=1e-3, vel_std=1e-2, noise_seed=77)
s = sim.Simulator(cfg, states, targets, neighbours=nb, knn_k=8, knn_radius=6.0, order="gauss_seidel",
                  record=False, **kw)
tr, xs, objs = [s.states.cpu().numpy().copy()], [], []
for _ in range(steps):
    s.step()
    tr.append(s.states.cpu().numpy().copy())
    xs.append(s.out["x"].cpu().numpy().copy())
    objs.append(s.out["obj"].cpu().numpy().copy())
np.savez(sys.argv[2], trace=np.array(tr), status=np.array(s.status_log), x=np.array(xs), obj=np.array(objs),
         states0=states, targets=targets)
print("saved", sys.argv[2])
