"""Where the bench's potential time goes: runs bench.py's protocol (adapt, untimed sampling,
timed sampling) on covtype and records, for every timed potential launch, the number of listed
chains and its duration (HIP events on the launch stream).  Prints a table by active-count
bucket.  usage: python scripts/bench_launch_profile.py [chains] [steps] [adapt] [warmup]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS

C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
A = int(sys.argv[3]) if len(sys.argv) > 3 else 200
W = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = torch.device("cuda:0")
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
mcmc = MCMC(NUTS(P.logistic_regression), num_warmup=A, num_samples=W, num_chains=C, progress_bar=False)
mcmc.warmup(0, Xd, yd)
if W:
    mcmc.run(1, Xd, yd)
    mcmc.post_warmup_state = mcmc.last_state
mcmc.num_samples = K
eng = mcmc._engine
cnt = eng.view("counters")
log = torch.zeros(200000, dtype=torch.int32, device=dev)
evs = []
orig = eng.potential.evaluate
stream = torch.cuda.current_stream()


def logged(ev, s):
    p = 0 if ev is eng.eval_lists[0] else 1
    log[len(evs)] = cnt[2 + p]
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(stream)
    orig(ev, s)
    b.record(stream)
    evs.append((a, b))


eng.potential.evaluate = logged
torch.cuda.synchronize()
a0 = torch.cuda.Event(enable_timing=True)
b0 = torch.cuda.Event(enable_timing=True)
a0.record(stream)
mcmc.run(2, Xd, yd, extra_fields=("num_steps",))
b0.record(stream)
torch.cuda.synchronize()
wall = a0.elapsed_time(b0)
n = np.asarray(log[:len(evs)].cpu().numpy(), np.int64)
ms = np.array([x.elapsed_time(y) for x, y in evs])
ns = mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()
print(json.dumps({"chains": C, "steps": K, "launches": len(evs), "wall_ms": wall, "potential_ms": float(ms.sum()),
                  "useful": int(ns.sum()), "evaluated": int(n.sum()),
                  "per_chain_total_mean": float(ns.sum(1).mean()), "per_chain_total_max": int(ns.sum(1).max())}))
edges = [0, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 1 << 30]
print(f"{'active':>12} {'launches':>8} {'ms':>9} {'ms/launch':>9} {'TF/s':>7} {'share':>6}")
for lo, hi in zip(edges[:-1], edges[1:]):
    m = (n > lo) & (n <= hi)
    if not m.any():
        continue
    tf = 4.0 * N * D * n[m].sum() / (ms[m].sum() * 1e-3) / 1e12
    print(f"{lo + 1:>5}-{hi:<6} {int(m.sum()):>8} {ms[m].sum():>9.2f} {ms[m].mean():>9.4f} {tf:>7.1f} "
          f"{ms[m].sum() / ms.sum():>6.1%}")
