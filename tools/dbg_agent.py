"""Debug helper: GPU vs oracle for one agent of the all-neighbour test swarm."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'mpc-cbf_amd'))
import numpy as np, torch
import oracle_lib as O
from mpccbf import swarm, Context
cfg = swarm.config(15)
states, targets = swarm.lattice_swarm(36, seed=7)
states[:, :2] *= 0.5
rp, col = swarm.all_csr(36)
dev = torch.device("cuda", 0)
for variant in (0, 1, 2):
    ctx = Context(cfg)
    ctx.set_variant(variant)
    out = ctx.alloc_outputs(36)
    ctx.impc_solve(torch.tensor(states, device=dev), torch.tensor(rp, device=dev),
                   torch.tensor(col, device=dev), targets=torch.tensor(targets, device=dev), **out)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in out.items()}
    print("variant", variant, "status", g["status"][19], "obj", g["obj"][19], "iters", g["iters"][19])
    bad = [a for a in range(36) if g["status"][a][1] != 3 and a == 19]
p = O.make_params(cfg)
refs = swarm.refs_from_targets(targets, 15)
r = O.impc_optimize(p, states, 19, col[rp[19]:rp[20]], refs[19])
print("oracle", r["status"], r["obj"], r["qp_iters"])
print("gpu x", g["x"][19][:12])
print("orc x0", r["x"][0][:12])
