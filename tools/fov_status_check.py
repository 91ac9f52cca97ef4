"""FoV (config 5) status parity of the dual active-set first attempt: the bench's closed loop with
the default solver, and at every step the same states solved by a PDIP-only context
(mpccbf_options.dual_as_steps < 0); the states of steps whose statuses differ are saved
for an offline oracle check (--check).

    python tools/fov_status_check.py [steps] [out.npz]          (GPU)
    python tools/fov_status_check.py --check out.npz            (CPU: oracle on the mismatches)

MPCCBF_CHECK_SLACK=1 runs the FoV slack setting (slack_cost 1000, decay 0.9, covariances 0.1 I)
instead; the objectives of agents solved by both are compared too.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


SLACK = os.environ.get("MPCCBF_CHECK_SLACK") == "1"


def fov_cfg(swarm):
    over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if SLACK else {}
    return swarm.fov_config(20, **over)


def run(steps, out):
    import torch
    from mpccbf import Context, swarm
    cfg = fov_cfg(swarm)
    states, targets = swarm.heading_swarm(512)
    dev = torch.device("cuda", 0)
    ctx_p = Context(cfg, dual_as_steps=-1)  # the PDIP alone
    ctx = Context(cfg)
    tg = torch.tensor(targets, device=dev)
    cur = torch.tensor(states, device=dev)
    o = ctx.alloc_outputs(512)
    op = ctx_p.alloc_outputs(512)
    traj_t = torch.full((512,), -1.0, dtype=torch.float64, device=dev)
    o["x"].fill_(float("nan"))
    common = dict(targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"])
    if SLACK:
        common["cov"] = torch.tensor(np.tile([0.1, 0.0, 0.1], (512, 1)), dtype=torch.float64, device=dev)
    objdiff = 0.0
    saved = {}
    nmis = 0
    for s in range(steps):
        ctx_p.impc_solve(cur, x=op["x"], status=op["status"], obj=op["obj"], iters=op["iters"], **common)
        ctx.impc_solve(cur, x=o["x"], status=o["status"], obj=o["obj"], iters=o["iters"],
                       next_states=o["next_states"], traj_t=traj_t, step_index=s, pos_std=0.001,
                       vel_std=0.01, noise_seed=20251015, **common)
        torch.cuda.synchronize()
        a, b = o["status"].cpu().numpy(), op["status"].cpu().numpy()
        both = (a == 0) & (b == 0)
        if both.any():
            oa, ob = o["obj"].cpu().numpy(), op["obj"].cpu().numpy()
            rel = np.where(both, np.abs(oa - ob) / (1.0 + np.abs(ob)), 0.0)
            w = np.unravel_index(np.argmax(rel), rel.shape)
            if rel[w] > objdiff:  # keep the worst agent's inputs for the oracle (--check)
                objdiff = float(rel[w])
                saved["worst_states"] = cur.cpu().numpy()
                saved["worst_agent"] = np.array([w[0], w[1]])
                saved["worst_obj"] = np.array([oa[w], ob[w]])
        # (failed solves of the default context count too: UNKNOWN where an attempt was made)
        failed = (a[:, 0] == 5) | ((a[:, 0] == 0) & (a[:, 1] == 5))
        mis = np.nonzero(np.any(a != b, axis=1) | failed)[0]
        if len(mis):
            nmis += len(mis)
            saved[f"states_{s}"] = cur.cpu().numpy()
            saved[f"das_{s}"] = a
            saved[f"pdip_{s}"] = b
            saved[f"agents_{s}"] = mis
            print(f"step {s}: {len(mis)} mismatches: " + ", ".join(
                f"{i}: das {a[i].tolist()} pdip {b[i].tolist()}" for i in mis[:6]), flush=True)
        cur = o["next_states"].clone()
        if s % 100 == 0:
            print(f"step {s}: das hist {np.bincount(a.ravel(), minlength=6).tolist()} "
                  f"max rel objective difference {objdiff:.3g}", flush=True)
    np.savez_compressed(out, targets=targets, **saved)
    print("mismatching agent-steps", nmis, "max rel objective difference", objdiff, "saved", out)


def check(path):
    import oracle_lib as O
    from mpccbf import swarm
    d = np.load(path)
    cfg = fov_cfg(swarm)
    p = O.make_params(cfg)
    covs = np.tile([0.1, 0.0, 0.1], (512, 1)) if SLACK else None
    refs = swarm.refs_from_targets(d["targets"], cfg["k_hor"])
    tally = {}
    for key in d.files:
        if not key.startswith("agents_"):
            continue
        s = key.split("_")[1]
        states = d[f"states_{s}"]
        rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
        for a in d[key]:
            r = O.impc_optimize(p, states, int(a), col[rp[a]:rp[a + 1]], refs[a], covs)
            k = (tuple(d[f"das_{s}"][a]), tuple(d[f"pdip_{s}"][a]), tuple(r["status"]))
            tally[k] = tally.get(k, 0) + 1
    for k, v in sorted(tally.items(), key=lambda kv: -kv[1]):
        print(f"das {k[0]} pdip {k[1]} oracle {k[2]}: {v}")
    if "worst_agent" in d.files:  # the largest objective difference: which solve is the oracle's
        states = d["worst_states"]
        a, it = (int(v) for v in d["worst_agent"])
        rp, col = swarm.fov_csr(states, 8, cfg["fov_Rs"], cfg["fov_beta"])
        r = O.impc_optimize(p, states, a, col[rp[a]:rp[a + 1]], refs[a], covs)
        print(f"largest objective difference: agent {a} iteration {it}: das-first {d['worst_obj'][0]!r} "
              f"pdip {d['worst_obj'][1]!r} oracle {r['obj'][it]!r} (status {r['status'].tolist()})")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--check"]:
        check(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 300,
            sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/fov_status.npz")
