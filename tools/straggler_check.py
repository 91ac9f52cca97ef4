"""Why do a launch's slowest agents take many solver steps? Reads a `bench.py --dump` file written
with the state trace (no --no-trace) and, for every agent of the timed steps whose IMPC iteration
0 took at least MIN_STEPS solver steps, re-solves that QP with the oracle (CPU) and counts the
sides active at its optimum (inequality rows within 1e-7 scaled of a bound): the dual active-set
solve keeps at most POL_K = 6 active sides and hands a QP with more to the PDIP.

    python tools/straggler_check.py gpurun_out/<tag>/dump.npz [MIN_STEPS]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
import oracle_lib as O  # noqa: E402
from mpccbf import swarm  # noqa: E402


def active_sides(qp, x, tol=1e-7):
    ax = qp["A"] @ x
    lo, hi = qp["lo"], qp["hi"]
    ineq = lo < hi
    al = ineq & (np.abs(ax - lo) <= tol * (1 + np.abs(lo)))
    au = ineq & (np.abs(ax - hi) <= tol * (1 + np.abs(hi)))
    return int(al.sum() + au.sum()), np.where(al | au)[0]


def main():
    d = np.load(sys.argv[1])
    min_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    traj, warm = d["traj"], int(d["warmup"])
    iters, status = d["iters"], d["status"]
    n = traj.shape[0]
    cfg = swarm.config(15)
    p = O.make_params(cfg)
    _, targets = swarm.lattice_swarm(n)
    refs = swarm.refs_from_targets(targets, cfg["k_hor"])
    for s in range(iters.shape[0]):
        ags = np.where(iters[s, :, 0] >= min_steps)[0]
        if len(ags) == 0:
            continue
        states = traj[:, warm + s, :]
        rp, col = swarm.knn_csr(states, 8, 3.0 * cfg["d_min"])
        for a in ags:
            nb = col[rp[a]:rp[a + 1]]
            r = O.impc_optimize(p, states, a, nb, refs[a])
            qp = O.assemble_qp(p, states[a], refs[a], states[nb], it=0)
            na, rows = (active_sides(qp, r["x"][0][:qp["n"]]) if r["status"][0] == O.OPTIMAL
                        else (-1, []))
            print(f"step {s} agent {a}: gpu iters {tuple(iters[s, a])} status {tuple(status[s, a])}; "
                  f"oracle {tuple(r['status'])}, active sides at iteration 0: {na} rows {list(rows)}")


if __name__ == "__main__":
    main()
