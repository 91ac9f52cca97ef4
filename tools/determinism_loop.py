"""Run-to-run determinism stress (diagnostics, GPU): the FoV closed loop of
tests/test_gpu_fov_slack.py::test_fov_closed_loop_is_deterministic repeated R times in one
process (each repetition: fresh context, output buffers pre-filled with different garbage, a
different allocation history); every repetition is compared bit for bit with the first and the
first differing (step, agent, iteration) entries are printed with both values.

    python tools/determinism_loop.py [repetitions] [slack 0|1] [steps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-cbf_amd"))
import mpccbf  # noqa: E402
from mpccbf import swarm  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
# PERTURB=1: before each repetition, a few steps of other IMPC kernels (collision, FoV without
# slack) run, so each repetition starts from different register / LDS contents left on the CUs
PERTURB = os.environ.get("PERTURB", "0") == "1"
# REGFILL=1: before every step, tools/regfill.hip writes a per-repetition pattern into every VGPR and
# AGPR of the chip, so a kernel reading a register it never wrote sees different values per
# repetition (build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/regfill.hip -o
# tools/build/libregfill.so)
REGFILL = os.environ.get("REGFILL", "0") == "1"
PATTERNS = (0x00000000, 0x7ff80000, 0x3ff00000, 0x40590000, 0xFFFFFFFF, 0x00000001)
_rf = None
if REGFILL:
    import ctypes
    _rf = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libregfill.so"))
    _rf.regfill_launch.argtypes = [ctypes.c_uint, ctypes.c_int]
SLACK = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
STEPS = int(sys.argv[3]) if len(sys.argv) > 3 else 30
n = 512
over = dict(slack_mode=1, slack_cost=1000.0, slack_decay_rate=0.9) if SLACK else {}
cfg = swarm.fov_config(20, **over)
states, targets = swarm.heading_swarm(n)
dev = torch.device("cuda", 0)
cov = torch.tensor(np.tile([0.1, 0.0, 0.1], (n, 1)), device=dev) if SLACK else None
ref = None
bad = 0
# REUSE=1: one Context for every repetition (no new operator upload / device allocations per run)
REUSE = os.environ.get("REUSE", "0") == "1"
ctx0 = mpccbf.Context(cfg) if REUSE else None
def perturb(kind):
    pc = swarm.config(15) if kind == 0 else swarm.fov_config(20)
    pn = 4096 if kind == 0 else 512
    st, tg2 = swarm.lattice_swarm(pn) if kind == 0 else swarm.heading_swarm(pn)
    pctx = mpccbf.Context(pc)
    pout = pctx.alloc_outputs(pn)
    cur2 = torch.tensor(st, device=dev)
    for _ in range(3):
        pctx.impc_solve(cur2, targets=torch.tensor(tg2, device=dev), knn_k=8,
                        knn_radius=pc.get("fov_Rs", 6.0), **pout)
        cur2 = pout["next_states"].clone()
    torch.cuda.synchronize()


for rep in range(R):
    if PERTURB:
        perturb(rep % 2)
    fill = (float("nan"), 1.0e30, -3.5, 0.0)[rep % 4]
    junk = torch.full((1 << (20 + rep % 4),), fill, dtype=torch.float64, device=dev)
    ctx = ctx0 if REUSE else mpccbf.Context(cfg)
    out = ctx.alloc_outputs(n)
    for k, v in out.items():
        v.fill_(fill if v.dtype == torch.float64 else -7 - rep)
    traj_t = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    out["x"].fill_(float("nan"))
    cur = torch.tensor(states, device=dev)
    tg = torch.tensor(targets, device=dev)
    log = {k: [] for k in ("status", "iters", "obj", "next_states")}
    for s in range(STEPS):
        if _rf is not None:
            torch.cuda.synchronize()
            assert _rf.regfill_launch(PATTERNS[rep % len(PATTERNS)], 8192) == 0
        ctx.impc_solve(cur, targets=tg, knn_k=8, knn_radius=cfg["fov_Rs"], cov=cov, traj_t=traj_t, step_index=s,
                       pos_std=0.001, vel_std=0.01, noise_seed=20251015, **out)
        for k in log:
            log[k].append(out[k].cpu().numpy().copy())
        cur = out["next_states"].clone()
    torch.cuda.synchronize()
    log = {k: np.stack(v) for k, v in log.items()}
    del junk
    WATCH = [int(v) for v in os.environ.get("WATCH", "").split(",") if v]
    if WATCH:
        print(f"rep {rep}: step-0 iters of {WATCH}: {log['iters'][0][WATCH].tolist()}", flush=True)
    if ref is None:
        ref = log
        print(f"rep 0: reference", flush=True)
        continue
    diffs = []
    for k in log:
        a, b = ref[k], log[k]
        same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else a == b
        if not same.all():
            idx = np.argwhere(~same)
            diffs.append((k, len(idx), [(tuple(i), a[tuple(i)], b[tuple(i)]) for i in idx[:4]]))
    if diffs:
        bad += 1
        print(f"rep {rep}: DIFFERS", flush=True)
        for d in diffs:
            print("   ", d[0], d[1], "entries; first:", d[2], flush=True)
    else:
        print(f"rep {rep}: identical", flush=True)
print("RESULT", "deterministic" if bad == 0 else f"{bad} of {R - 1} repetitions differ")
