"""Lockstep (sync_chains) chain groups vs the one-stream loop, repeated.

Covtype-shaped logistic regression (D = 55: k_nuts_step<8,16>, a chain's 32 lanes over eight
waves), 1024 chains in 4 groups on 4 streams, W = 30 / S = 12; each repetition's draws, tree
sizes and potential energies must equal the one-stream run's bitwise.  Run once with the
product library and once with NUMPYRO_AMD_LIB pointing at the round-5 WAIT resolution
(scripts/ab_wait_race_src.py) to see the race and its fix side by side.
usage: python scripts/diag_wait_race.py [--reps K] [--groups G] [--chains C] [--tag NAME]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import datasets  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.engine import Engine  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402


def run(X, y, C, G, sync):
    Engine.chain_groups = G
    mcmc = MCMC(NUTS(P.logistic_regression), num_warmup=30, num_samples=12, num_chains=C,
                chain_method="vectorized", progress_bar=False, sync_chains=sync)
    mcmc.warmup(3, X, y, collect_warmup=True, extra_fields=("num_steps", "potential_energy"))
    mcmc.run(3, X, y, extra_fields=("num_steps", "potential_energy"))
    assert mcmc._engine._groups() == G
    ef = mcmc.get_extra_fields(True)
    return (mcmc.get_samples(True)["coefs"].cpu().numpy(), ef["num_steps"].cpu().numpy(),
            ef["potential_energy"].cpu().numpy())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--groups", type=int, default=4)
    ap.add_argument("--chains", type=int, default=1024)
    ap.add_argument("--tag", default="product")
    a = ap.parse_args()
    X, y = datasets.covtype_synthetic(n_rows=4000, seed=1)
    X, y = torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda()
    ref = run(X, y, a.chains, 1, True)
    bad = []
    for r in range(a.reps):
        got = run(X, y, a.chains, a.groups, True)
        diff = np.nonzero(np.any(got[0] != ref[0], axis=(1, 2)) | np.any(got[1] != ref[1], axis=1))[0]
        if diff.size:
            bad.append({"rep": r, "chains": diff.tolist()[:64], "n": int(diff.size),
                        "blocks_of_16": sorted(set(int(c) // 16 for c in diff))})
        print(f"[{a.tag}] rep {r}: {diff.size} chains differ", flush=True)
    print(json.dumps({"tag": a.tag, "lib": os.environ.get("NUMPYRO_AMD_LIB", "product"), "reps": a.reps,
                      "groups": a.groups, "chains": a.chains, "reps_differing": len(bad), "detail": bad}))


if __name__ == "__main__":
    main()
