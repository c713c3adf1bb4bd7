"""Diagnostics: per-launch potential time vs active-chain count inside a real NUTS run."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import datasets, native
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS

W, K = int(sys.argv[1]), int(sys.argv[2])
X, y = datasets.covtype_synthetic(seed=0)
dev = torch.device("cuda:0")
Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
mcmc = MCMC(NUTS(P.logistic_regression), num_warmup=W, num_samples=K, num_chains=4096)
mcmc.warmup(0, Xd, yd)
eng = mcmc._engine
pot = eng.potential
cnt = eng.view("counters")
log_counts = torch.zeros(200000, dtype=torch.int32, device=dev)
evs = []
orig = pot.evaluate
stream = torch.cuda.current_stream()
def timed(ev, s):
    i = len(evs)
    p = 0 if ev is eng.eval_lists[0] else 1
    log_counts[i] = cnt[2 + p]
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(stream); orig(ev, s); b.record(stream)
    evs.append((a, b))
pot.evaluate = timed
torch.cuda.synchronize(); t0 = time.perf_counter()
mcmc.run(1, Xd, yd, extra_fields=("num_steps",))
torch.cuda.synchronize(); t1 = time.perf_counter()
n = len(evs)
ms = np.array([a.elapsed_time(b) for a, b in evs])
c = log_counts[:n].cpu().numpy()
ns = mcmc.get_extra_fields()["num_steps"].sum().item()
print(f"launches {n}  sum(active) {c.sum()}  sum(num_steps) {ns}  wall {t1-t0:.2f}s  pot {ms.sum()/1e3:.2f}s")
for lo, hi in [(0, 1), (1, 512), (512, 1024), (1024, 2048), (2048, 3072), (3072, 4097)]:
    m = (c >= lo) & (c < hi)
    if m.any():
        print(f"  active [{lo},{hi}): {m.sum()} launches, mean {ms[m].mean():.3f} ms, mean active {c[m].mean():.0f}, "
              f"TF(alg) {4*581012*55*c[m].sum()/(ms[m].sum()*1e-3)/1e12:.1f}")
