"""Locate the round-5 in-process pooled multi-device divergence.

MCMC(devices=[cuda:0, cuda:0], dense_mass="pooled"): two engines, one host thread each, meet at
every middle adaptation window end (shard.DeviceGroup.all_reduce_sum), then each rank finalizes
the pooled moments and factorizes them itself (dense.Whitening.set: torch.linalg.cholesky, then
T^-1 by triangular solves) and re-expresses its chains (Engine._reexpress).  Both ranks start the
factorization from bitwise-identical moments, so their T, mu and T^-1 must be bitwise equal; any
difference is produced by the factorization stage itself.

Per repetition this records, per rank and window end: the reduced moments (n, s1, s2), the
finalized (cov, mean), T, T^-1 and the re-expressed positions, and the run's draws, and compares
(i) rank 1 with rank 0 inside the repetition (the stages after the all_reduce) and (ii) every
repetition with the first.  --unlocked runs the factorizations concurrently (DeviceGroup's
linalg_lock replaced by a no-op), the configuration of the failing round-5 run.

usage: python scripts/diag_pooled_race.py [--reps K] [--dim D] [--unlocked] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--dim", type=int, default=600)
    ap.add_argument("--chains", type=int, default=48)
    ap.add_argument("--unlocked", action="store_true")
    ap.add_argument("--out", default="gpurun_out/diag_pooled_race.json")
    a = ap.parse_args()

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    import pooled_stages as PS

    reps = []
    for r in range(a.reps):
        t0 = time.time()
        with PS.recording(unlocked=a.unlocked) as rec:
            mcmc = MCMC(NUTS(P.funnel, dense_mass="pooled", max_tree_depth=6), num_warmup=30, num_samples=4,
                        num_chains=a.chains, devices=["cuda:0", "cuda:0"], progress_bar=False)
            mcmc.run(5, a.dim, extra_fields=("num_steps",))
        x = mcmc.get_samples(True)["x"]
        ns = mcmc.get_extra_fields(True)["num_steps"]
        reps.append({"records": list(rec), "x": PS.h(x), "ns": PS.h(ns), "x_t": x.cpu(), "s": time.time() - t0})
        print(f"rep {r}: {reps[-1]['s']:.1f} s, draws {reps[-1]['x']}", flush=True)

    def stages(rp, rank):
        return [{k: v for k, v in e.items() if k != "rank"} for e in rp["records"] if e["rank"] == rank]

    findings = []
    for i, rp in enumerate(reps):
        r0, r1 = stages(rp, 0), stages(rp, 1)
        for j, (e0, e1) in enumerate(zip(r0, r1)):
            diff = [k for k in e0 if k not in ("w",) and e0[k] != e1[k]]  # w: each rank's own chains
            if diff:
                findings.append({"rep": i, "record": j, "stage": e0["stage"], "rank1_vs_rank0_differs": diff})
        if i > 0:
            for rank in (0, 1):
                for j, (e0, e1) in enumerate(zip(stages(reps[0], rank), stages(rp, rank))):
                    diff = [k for k in e0 if e0[k] != e1[k]]
                    if diff:
                        findings.append({"rep": i, "rank": rank, "record": j, "stage": e0["stage"],
                                         "vs_rep0_differs": diff})
            if rp["x"] != reps[0]["x"]:
                d = (rp["x_t"] - reps[0]["x_t"]).abs()
                half = d.shape[0] // 2
                findings.append({"rep": i, "draws_differ": True, "max_abs": float(d.max()),
                                 "rank0_max": float(d[:half].max()), "rank1_max": float(d[half:].max())})
    out = {"unlocked": a.unlocked, "reps": a.reps, "dim": a.dim, "chains": a.chains,
           "draw_hashes": [rp["x"] for rp in reps], "tree_hashes": [rp["ns"] for rp in reps],
           "window_ends": [stages(reps[0], 0)], "findings": findings, "equal": not findings}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"unlocked": a.unlocked, "equal": not findings, "n_findings": len(findings),
                      "first": findings[:4]}))


if __name__ == "__main__":
    main()
