"""Cost of one leaf round of the fused wide step (SV, D = 2519) against the number of chains:
wall / rounds and the chain-slot occupancy (useful chain-leapfrogs / (rounds x chains)) of a
short adapted run, so the latency floor of a round (few live chains) and its throughput slope
(many) can be read apart.  usage: python scripts/wide_round_cost.py [C1,C2,...] [--lib path]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
args = [a for a in sys.argv[1:] if not a.startswith("--lib")]
if "--lib" in sys.argv:
    from numpyro_amd import native
    native.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    args = [a for a in args if a != native.LIB_PATH and not a.endswith(".so")]
import torch  # noqa: E402

from numpyro_amd import datasets  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402

r = datasets.sp500_synthetic()
for C in [int(c) for c in (args[0].split(",") if args else "64,256,1024,4096,8192".split(","))]:
    mcmc = MCMC(NUTS(P.stochastic_volatility), num_warmup=30, num_samples=5, num_chains=C, progress_bar=False)
    mcmc.warmup(0, r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mcmc.run(1, r, extra_fields=("num_steps",))
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ns = mcmc.get_extra_fields(group_by_chain=True)["num_steps"].to(torch.float64)
    rounds = mcmc.last_run_stats["launches"]
    print(json.dumps({"chains": C, "wall_s": round(wall, 4), "rounds": rounds, "us_per_round": round(wall / rounds * 1e6, 1),
                      "leapfrogs": int(ns.sum()), "leapfrog_per_s": round(float(ns.sum()) / wall),
                      "slot_occupancy": round(float(ns.sum()) / (rounds * C), 3),
                      "max_chain_leapfrogs": int(ns.sum(1).max()), "mean_chain_leapfrogs": round(float(ns.sum(1).mean()), 1)}),
          flush=True)
    del mcmc
    torch.cuda.empty_cache()
