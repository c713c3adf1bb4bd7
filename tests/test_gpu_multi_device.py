"""MCMC(chain_method="parallel") in ONE process over several devices (the reference pmaps the
chains over local devices, numpyro/infer/mcmc.py:700-715; a callable chain_method is its
pmap-of-vectorized form, :296-320): one engine and one host thread per device, chains sharded
contiguously by global id.  Rehearsed on one GPU with two engines on cuda:0 (the driver's 8-GPU
node is not ours to launch): the draws must be bitwise those of the one-engine run (diagonal
mass: a chain's trajectory depends only on its global id) and of the torchrun path (pooled dense
mass: moments summed over the two shards)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TWO = ["cuda:0", "cuda:0"]


def _run(model, args, C, devices, chain_method="parallel", W=30, S=6, seed=3, **kw):
    mcmc = MCMC(NUTS(model, **kw), num_warmup=W, num_samples=S, num_chains=C, chain_method=chain_method,
                devices=devices, progress_bar=False)
    mcmc.warmup(seed, *args, extra_fields=("num_steps",), collect_warmup=True)
    warm = mcmc.get_samples(group_by_chain=True), mcmc.get_extra_fields(group_by_chain=True)
    mcmc.run(seed + 1, *args, extra_fields=("num_steps", "accept_prob", "adapt_state.step_size"))
    return mcmc, warm


@pytest.mark.parametrize("model", ["logreg", "sv", "eight_schools"])
def test_parallel_devices_equal_one_engine_bitwise(device, model):
    """Fused step (covtype-shaped logistic regression), persistent wide kernel (SV) and the
    one-launch small-model schedule (eight schools): two engines on two devices (here both
    cuda:0) draw bitwise what one engine draws, warmup and resumed sampling both; the state
    round-trips; a callable chain_method takes the same path."""
    if model == "logreg":
        X, y = datasets.covtype_synthetic(n_rows=4000, seed=1)
        fm, args, C = P.logistic_regression, (X, y), 100
    elif model == "sv":
        fm, args, C = P.stochastic_volatility, (datasets.sp500_synthetic(T=400),), 40
    else:
        fm, args, C = P.eight_schools, (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y), 37
    one, w1 = _run(fm, args, C, None, chain_method="vectorized")
    two, w2 = _run(fm, args, C, TWO)
    assert two._engines is not None and len(two._engines) == 2 and one._engines is None
    assert [e.C for e in two._engines] == [(C + 1) // 2, C // 2]
    for a, b in ((w1[0], w2[0]), (one.get_samples(True), two.get_samples(True))):
        for k in a:
            assert torch.equal(a[k].cpu(), b[k].cpu()), k
    for a, b in ((w1[1], w2[1]), (one.get_extra_fields(True), two.get_extra_fields(True))):
        for k in a:
            assert torch.equal(a[k].cpu(), b[k].cpu()), k
    st1, st2 = one.last_state, two.last_state
    assert torch.equal(st1.adapt_state.step_size.cpu(), st2.adapt_state.step_size.cpu())
    assert torch.equal(st1.potential_energy.cpu(), st2.potential_energy.cpu())
    # callable chain_method (pmap-of-vectorized in the reference): the same sharded path
    three, _ = _run(fm, args, C, TWO, chain_method=lambda f: f, W=30, S=6)
    for k, v in one.get_samples(True).items():
        assert torch.equal(v.cpu(), three.get_samples(True)[k].cpu())
    two.print_summary()


def pooled_run(devices):
    """dense_mass='pooled' funnel D=600 (BASELINE config 2's schedule): 48 chains, one middle
    adaptation window (W = 30) whose pooled moments are summed over the shards."""
    mcmc = MCMC(NUTS(P.funnel, dense_mass="pooled", max_tree_depth=6), num_warmup=30, num_samples=4, num_chains=48,
                devices=devices, progress_bar=False)
    mcmc.run(5, 600, extra_fields=("num_steps",))
    return mcmc.get_samples(True)["x"], mcmc.get_extra_fields(True)["num_steps"]


def test_parallel_pooled_dense_equals_torchrun(device, tmp_path):
    """The in-process two-device pooled run equals the 2-rank torchrun bitwise.  Both record the
    window ends' stage hashes (tests/pooled_stages.py: reduced moments, finalized covariance,
    T, T^-1, re-expressed positions per rank), so a divergence names the first stage where the
    two paths part (round 5 saw one unexplained rank-1 rounding divergence; 56 later repetitions
    with every stage hashed found none)."""
    import pooled_stages as PS

    with PS.recording() as rec:
        x2, n2 = pooled_run(TWO)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = tmp_path / "dist.pt"
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port),
                    os.path.join(ROOT, "tests", "dist_pooled_worker.py"), str(out)], check=True, timeout=600, env=env)
    ref = torch.load(out, weights_only=True)
    where = {r: PS.first_difference(PS.by_rank(rec, r), PS.by_rank(ref["stages"], r)) for r in (0, 1)}
    print(f"[pooled] stages per rank: {len(PS.by_rank(rec, 0))} / {len(PS.by_rank(rec, 1))} records; "
          f"first difference vs torchrun: {where}")
    assert torch.equal(ref["ns"], n2.cpu()), where
    assert torch.equal(ref["x"], x2.cpu()), where
    assert where == {0: None, 1: None}
    one_x, one_n = pooled_run(None)  # one engine pools in one GEMM: equal to rounding, not bitwise
    print(f"[pooled] one engine vs two: {float((one_x.cpu() - x2.cpu()).abs().max()):.2e} max |dx|, "
          f"{int((one_n.cpu() == n2.cpu()).sum())}/{n2.numel()} equal tree sizes")


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two distinct GPUs (the one-GPU box rehearses with two engines on cuda:0)")
@pytest.mark.parametrize("model", ["logreg", "bnn_dense"])
def test_parallel_two_distinct_devices(device, model):
    """MCMC(devices=["cuda:0", "cuda:1"]) on two distinct GPUs: per-thread device contexts, the
    per-device dynamic-LDS attribute of the big whitening tile (nmx_lds_limit: k_gemm_x3's 144 KB
    and k_bnn's 79 KB must be raised on each device) and the peer copies of the pooled moments.
    Diagonal mass draws bitwise what one engine draws; pooled dense equals the two-engines-on-one-
    GPU rehearsal bitwise (same shards, same rank-order sums)."""
    if model == "logreg":
        X, y = datasets.covtype_synthetic(n_rows=4000, seed=1)
        one, _ = _run(P.logistic_regression, (X, y), 100, None, chain_method="vectorized")
        two, _ = _run(P.logistic_regression, (X, y), 100, ["cuda:0", "cuda:1"])
        assert {str(e.device) for e in two._engines} == {"cuda:0", "cuda:1"}
        for k, v in one.get_samples(True).items():
            assert torch.equal(v.cpu(), two.get_samples(True)[k].cpu()), k
        return
    Xb, Yb = datasets.bnn_data(N=100, D_X=3)
    runs = []
    for devs in (["cuda:0", "cuda:0"], ["cuda:0", "cuda:1"]):
        mcmc = MCMC(NUTS(P.bnn, dense_mass="pooled", max_tree_depth=5), num_warmup=30, num_samples=3,
                    num_chains=64, devices=devs, progress_bar=False, postprocess_fn=lambda z: z)
        mcmc.run(4, Xb, Yb, 69, extra_fields=("num_steps",))
        runs.append((mcmc.get_samples(True)["w2"].cpu(), mcmc.get_extra_fields(True)["num_steps"].cpu()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
