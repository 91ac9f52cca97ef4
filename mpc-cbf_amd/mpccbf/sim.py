"""Closed-loop swarm simulator with the reference example's outputs.

The loop of MPCCBFFormationControl_example.cpp:131-231 on the device: every control step each
robot re-plans (ConnectivityIMPCCBF::optimize -> mpccbf_impc_solve), keeps its last successful
trajectory when a step fails (:150-165), and integrates int(h / Ts) control sub-steps of the kept
curve with state noise (:188-207), or holds its position at zero velocity when it never had a
curve (:208-221). Two update orders:
  order="jacobi" (default, the batched product path): all robots in one launch, every robot
      re-planning from the states of the previous step;
  order="gauss_seidel" (the reference's own order, for parity at small N): robots in index order
      (:140), each solved alone (one launch per robot) from the current table and its next state
      written back in place (:201) before the next robot plans, so robot i sees robots < i at
      their new states.
The states.json trace is written in the example's shape (:127-129, :166-205, :229-231):

    {"dt": h, "Ts": Ts, "robots": {"<i>": {"pred_curve": [[[x, y, z], ...]] per step,
                                           "states": [[px, py, pz, vx, vy, vz], ...] per sub-step}}}

pred_curve: the kept curve's positions at traj_eval_t + 0.05 k, k = 0.. while 0.05 k <= the curve's
parameter range (clamped to it), or the current position when there is no curve.
"""
from __future__ import annotations

import json
import math

import numpy as np

from . import swarm
from ._lib import Context


def bezier_positions(cfg: dict, x: np.ndarray, ts) -> np.ndarray:
    """Positions of the piecewise Bezier curve with control points x ([piece][dim][cp],
    BezierQPOperations.cpp:20-43) at parameters ts (SingleParameterPiecewiseCurve::eval,
    SingleParameterPiecewiseCurve.cpp:94-127: the first piece whose cumulative parameter reaches
    t, local parameter clamped to the piece)."""
    P, C, T = cfg["num_pieces"], cfg["num_control_points"], cfg["piece_max_parameter"]
    deg = C - 1
    cps = np.asarray(x).reshape(P, 3, C)
    out = []
    for t in ts:
        piece = 0
        while piece < P - 1 and (piece + 1) * T < t:
            piece += 1
        u = t if piece == 0 else min(T, t - piece * T)
        s = u / T
        basis = np.array([math.comb(deg, i) * s ** i * (1.0 - s) ** (deg - i) for i in range(C)])
        out.append(cps[piece] @ basis)
    return np.array(out)


class Simulator:
    """Closed-loop simulation of a swarm on one GPU, recording the example's states.json.

    neighbours: "knn" (the knn_k nearest within knn_radius, found on the device) or "all" (every
    other robot, the reference's semantics, ConnectivityIMPCCBF.cpp:59-67)."""

    def __init__(self, cfg: dict, states: np.ndarray, targets: np.ndarray, *, neighbours="knn",
                 knn_k=8, knn_radius=None, pos_std=0.0, vel_std=0.0, noise_seed=0, device=0,
                 record=True, order="jacobi"):
        import torch
        if order not in ("jacobi", "gauss_seidel"):
            raise ValueError("order must be 'jacobi' or 'gauss_seidel'")
        self.order = order
        self.torch = torch
        self.cfg = dict(cfg)
        self.dev = torch.device("cuda", device)
        self.ctx = Context(cfg, device=device)
        n = len(states)
        self.n = n
        self.states = torch.tensor(states, dtype=torch.float64, device=self.dev)
        self.next = torch.empty_like(self.states)
        self.targets = torch.tensor(targets, dtype=torch.float64, device=self.dev)
        self.traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=self.dev)
        self.out = self.ctx.alloc_outputs(n, device=self.dev)
        self.out["x"].fill_(float("nan"))
        self.nsub = int(cfg["h"] / cfg["Ts"])
        self.substeps = torch.empty((n, self.nsub, 6), dtype=torch.float64, device=self.dev)
        self.nb = {}
        self.csr = neighbours == "all"
        if self.csr:
            rp, col = swarm.all_csr(n)
            self.nb = dict(nb_row_ptr=torch.tensor(rp, device=self.dev),
                           nb_col=torch.tensor(col if len(col) else np.zeros(1, np.int32), device=self.dev))
        else:
            self.nb = dict(knn_k=knn_k, knn_radius=knn_radius or 3.0 * cfg["d_min"])
        self.gs_next = torch.empty((1, 6), dtype=torch.float64, device=self.dev)
        self.noise = dict(pos_std=pos_std, vel_std=vel_std, noise_seed=noise_seed)
        self.step_index = 0
        self.sim_t = 0.0
        self.record = record
        self.rec = {str(i): {"pred_curve": [], "states": []} for i in range(n)} if record else None
        self.status_log = []

    def step(self):
        """One control step for every robot (the body of the example's while loop)."""
        torch = self.torch
        t_before = self.traj_t.cpu().numpy() if self.record else None
        o = self.out
        if self.order == "jacobi":
            self.ctx.impc_solve(self.states, targets=self.targets, x=o["x"], status=o["status"], obj=o["obj"],
                                iters=o["iters"], next_states=self.next, traj_t=self.traj_t,
                                substeps=self.substeps, step_index=self.step_index, **self.nb, **self.noise)
        else:
            # robot by robot (:140), each from the table as the robots before it left it (:201)
            self.next.copy_(self.states)  # (the states the robots re-plan from, for the record)
            for i in range(self.n):
                sl = slice(i, i + 1)
                nb = dict(self.nb)
                if self.csr:
                    nb["nb_row_ptr"] = self.nb["nb_row_ptr"][i:i + 2]
                self.ctx.impc_solve(self.states, targets=self.targets[sl], agent_first=i, num_agents=1,
                                    x=o["x"][sl], status=o["status"][sl], obj=o["obj"][sl], iters=o["iters"][sl],
                                    next_states=self.gs_next, traj_t=self.traj_t[sl], substeps=self.substeps[sl],
                                    step_index=self.step_index, **nb, **self.noise)
                self.states[i].copy_(self.gs_next[0])
            self.states, self.next = self.next, self.states  # (swapped back below)
        torch.cuda.synchronize()
        status = o["status"].cpu().numpy()
        self.status_log.append(status.copy())
        if self.record:
            self._record(t_before, status)
        self.states, self.next = self.next, self.states
        self.step_index += 1
        self.sim_t += self.cfg["h"]
        return status

    def _record(self, t_before, status):
        cfg = self.cfg
        horizon = cfg["num_pieces"] * cfg["piece_max_parameter"]
        x = self.out["x"].cpu().numpy()
        sub = self.substeps.cpu().numpy()
        cur = self.states.cpu().numpy()
        for i in range(self.n):
            r = self.rec[str(i)]
            new = bool(np.any(status[i] == 0))
            has = new or t_before[i] >= 0.0
            if has:
                t0 = 0.0 if new else t_before[i]
                ts, t = [], 0.0
                while t <= horizon:  # the example's accumulation (:172-181)
                    ts.append(min(t0 + t, horizon))
                    t += 0.05
                r["pred_curve"].append([bezier_positions(cfg, x[i], ts).tolist()])
            else:
                r["pred_curve"].append([[cur[i, :3].tolist()]])
            r["states"].extend(sub[i].tolist())

    def run(self, sim_runtime: float):
        while self.sim_t < sim_runtime - 1e-12:
            self.step()
        return self

    def states_json(self) -> dict:
        return {"dt": self.cfg["h"], "Ts": self.cfg["Ts"], "robots": self.rec}

    def write_json(self, path: str):
        with open(path, "w") as f:
            json.dump(self.states_json(), f, indent=4)
