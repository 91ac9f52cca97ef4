"""Offline oracle check of a tools/status_dump.py snapshot: every agent's IMPC statuses (and the
objectives of OPTIMAL iterations) at the saved steps against the CPU oracle on the same states.

    python tools/status_check.py gpurun_out/sd1000.npz [--threads 8]
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
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--k-hor", type=int, default=15)
    a = ap.parse_args()
    import oracle_lib as O
    from mpccbf import swarm
    d = np.load(a.npz)
    cfg = swarm.config(a.k_hor)
    p = O.make_params(cfg)
    refs = swarm.refs_from_targets(d["targets"], a.k_hor)
    radius = 3.0 * cfg["d_min"]
    for k in d["snaps"]:
        states = d[f"states_{k}"]
        gs, go = d[f"status_{k}"], d[f"obj_{k}"]
        rp, col = swarm.knn_csr(states, 8, radius)
        r = O.impc_batch(p, states, refs, rp, col, 0, len(states), a.threads)
        os_, oo = r["status"], r["obj"]
        mism = np.nonzero(np.any(gs != os_, axis=1))[0]
        opt = (gs == 0) & (os_ == 0)
        rel = np.abs(go[opt] - oo[opt]) / np.maximum(1, np.abs(oo[opt]))
        # closest pair distance of every agent (is it inside d_min?)
        pos = states[:, :2]
        dmin_each = np.array([np.sqrt(np.min(np.sum((pos[col[rp[i]:rp[i + 1]]] - pos[i]) ** 2, 1)))
                              if rp[i + 1] > rp[i] else np.inf for i in range(len(states))])
        inf_gpu = gs[:, 0] == 3
        print(f"step {k}: status mismatches {len(mism)}; OPT both {int(opt.sum())}, max rel obj "
              f"{rel.max() if rel.size else 0:.2e}; GPU it0 INFEASIBLE {int(inf_gpu.sum())}, oracle "
              f"{int(np.sum(os_[:, 0] == 3))}; nearest-neighbour distance of infeasible agents: "
              f"min {dmin_each[inf_gpu].min() if inf_gpu.any() else np.nan:.3f} max "
              f"{dmin_each[inf_gpu].max() if inf_gpu.any() else np.nan:.3f} (d_min {cfg['d_min']})")
        for i in mism[:10]:
            print("   agent", i, "gpu", gs[i], "oracle", os_[i], "gpu obj", go[i], "oracle obj", oo[i])


if __name__ == "__main__":
    main()
