"""Run the captured regression cases (tests/golden/regress_cases.json) through impc_solve and print
statuses / iteration counts (with MPCCBF_LIB pointing at a diagnostics build: exit reasons or the
per-attempt split) next to the oracle.

    MPCCBF_LIB=mpc-cbf_amd/build/dbg/libmpccbf.so python tools/run_case.py [name]
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(REPO, "mpc-cbf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mpccbf import Context, swarm  # noqa: E402

cases = json.load(open(os.path.join(REPO, "tests", "golden", "regress_cases.json")))["cases"]
want = sys.argv[1] if len(sys.argv) > 1 else None
dev = torch.device("cuda", 0)
for case in cases:
    if want and case["name"] != want:
        continue
    cfg = swarm.config(case["k_hor"])
    states = np.array(case["states"])
    n = len(states)
    rp = np.array([0, n - 1], np.int32)
    col = np.arange(1, n, dtype=np.int32)
    ctx = Context(cfg)
    out = ctx.alloc_outputs(1)
    stamps = torch.zeros(8 + 2 * 256, dtype=torch.int64, device=dev)
    ctx.impc_solve(torch.tensor(states, device=dev), torch.tensor(rp, device=dev),
                   torch.tensor(col, device=dev), targets=torch.tensor([case["target"]], dtype=torch.float64, device=dev),
                   num_agents=1, stamps=stamps, **out)
    torch.cuda.synchronize()
    print(case["name"], "status", out["status"].cpu().numpy()[0], "iters", out["iters"].cpu().numpy()[0],
          "obj", out["obj"].cpu().numpy()[0])
    if "trace" in os.environ.get("MPCCBF_LIB", ""):
        tr = stamps.cpu().numpy()[8:].view(np.float64).reshape(2, 64, 4)
        for k in range(32):
            if tr[0, k, 1] == 0:
                break
            print("   %2d rp %9.2e mu %9.2e alpha %7.4f rd %9.2e" % ((k,) + tuple(tr[0, k])))
