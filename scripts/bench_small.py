"""BASELINE config 0 (README.md eight schools, NUTS, 4 chains, vectorized; the reference's
CPU-runnable case): wall time of warmup + sampling with the persistent schedule vs the
launched step/potential loop.  usage: python scripts/bench_small.py [warmup] [samples] [chains]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS

W, S, C = (int(a) for a in (sys.argv[1:4] + ["1000", "1000", "4"][len(sys.argv[1:4]):]))
args = (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y)
from numpyro_amd.engine import Engine

for mode in ("1", "0", "1"):
    Engine.persistent = mode == "1"
    mcmc = MCMC(NUTS(P.eight_schools), num_warmup=W, num_samples=S, num_chains=C, progress_bar=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mcmc.run(0, *args, extra_fields=("num_steps",))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ns = int(mcmc.get_extra_fields()["num_steps"].sum())
    mu = mcmc.get_samples()["mu"].cpu().numpy()
    print(f"{'persistent' if mode == '1' else 'launched  '} W={W} S={S} C={C}: {dt:.3f} s "
          f"(warmup + sampling), {ns} sampling leapfrogs, mu mean {mu.mean():.2f} sd {mu.std():.2f}", flush=True)
