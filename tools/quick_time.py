"""Quick timing of the fused IMPC kernel + device KNN on a synthetic lattice swarm."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'mpc-cbf_amd'))
import numpy as np, torch
from mpccbf import swarm, Context
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 15
cfg = swarm.config(K)
states, targets = swarm.lattice_swarm(N)
dev = torch.device("cuda", 0)
st = torch.tensor(states, device=dev); tg = torch.tensor(targets, device=dev)
rp = torch.empty(N + 1, dtype=torch.int32, device=dev); col = torch.empty(N * 8, dtype=torch.int32, device=dev)
for variant in (0, 1, 2):
    ctx = Context(cfg); ctx.set_variant(variant)
    out = ctx.alloc_outputs(N)
    ctx.build_neighbors(st, 0, N, 8, 6.0, rp, col)
    for _ in range(3):
        ctx.impc_solve(st, rp, col, targets=tg, **out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        ctx.impc_solve(st, rp, col, targets=tg, **out)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    s = out["status"].cpu().numpy(); it = out["iters"].cpu().numpy()
    print(f"variant {variant}: N={N} K={K} impc {ms*1e3:.1f} us/step -> {2*N/ms*1e3:.3e} QP/s; "
          f"optimal {np.mean(s==0):.4f} iters mean {it.mean():.2f} max {it.max()}")
e0.record()
for _ in range(20):
    ctx.build_neighbors(st, 0, N, 8, 6.0, rp, col)
e1.record(); torch.cuda.synchronize()
print(f"knn build {e0.elapsed_time(e1)/20*1e3:.1f} us")
