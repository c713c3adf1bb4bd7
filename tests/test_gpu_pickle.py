"""Checkpoint / resume across pickling and processes (test/test_pickle.py:86-96,
215-220; mcmc.py:797-800, hmc.py:818-822) and MCMC(postprocess_fn=...) (mcmc.py:331-442).

A resumed run must be bitwise the run continued in the original process: the chain state
(arena), the adapted mass matrix and the Philox stream (keyed by seed, global chain id and
transition index) are all part of the pickled state."""
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest
import torch

from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import HMC, MCMC, NUTS

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ES = (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y)


@pytest.mark.parametrize("kernel", [HMC, NUTS])
def test_pickle_hmc(device, kernel):
    """test_pickle.py:86-96 (normal_model, :59-60): samples survive a pickle round trip of the
    MCMC object."""
    args = (np.zeros(1, np.float32), np.ones(1, np.float32))
    mcmc = MCMC(kernel(P.diag_normal), num_warmup=10, num_samples=10, num_chains=8)
    mcmc.run(0, *args)
    m2 = pickle.loads(pickle.dumps(mcmc))
    for k, v in mcmc.get_samples().items():
        torch.testing.assert_close(m2.get_samples()[k], v, rtol=0, atol=0)


@pytest.mark.parametrize("model,args,dense", [
    ("eight_schools", ES, False),             # persistent one-launch schedule
    ("sv", (datasets.sp500_synthetic(T=300),), False),   # wide (D-split) fused step
    ("mvn", None, "pooled"),                  # pooled dense mass (whitening state)
    ("mvn", None, True),                      # per-chain dense mass
])
def test_mcmc_pickle_post_warmup_resumes_bitwise(device, model, args, dense):
    """test_pickle.py:215-220: pickled_mcmc.post_warmup_state = pickled_mcmc.last_state, then
    run again -- here checked bitwise against the same continuation in-process."""
    if model == "mvn":
        rs = np.random.RandomState(0)
        a = rs.randn(5, 5)
        args = (np.zeros(5), a @ a.T + 0.5 * np.eye(5))
    fm = {"eight_schools": P.eight_schools, "sv": P.stochastic_volatility, "mvn": P.multivariate_normal}[model]
    mk = lambda: MCMC(NUTS(fm, dense_mass=dense), num_warmup=40, num_samples=10, num_chains=24)  # noqa: E731
    mcmc = mk()
    mcmc.run(0, *args)
    blob = pickle.dumps(mcmc)
    mcmc.post_warmup_state = mcmc.last_state
    mcmc.run(1, *args, extra_fields=("num_steps",))
    ref = mcmc.get_samples(), mcmc.get_extra_fields()["num_steps"]
    m2 = pickle.loads(blob)
    m2.post_warmup_state = m2.last_state
    m2.run(1, *args, extra_fields=("num_steps",))
    for k, v in ref[0].items():
        torch.testing.assert_close(m2.get_samples()[k], v, rtol=0, atol=0, msg=k)
    torch.testing.assert_close(m2.get_extra_fields()["num_steps"], ref[1], rtol=0, atol=0)
    assert int(m2.last_state.i[0]) == 60


_CHILD = r"""
import pickle, sys, torch
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
with open({blob!r}, "rb") as f:
    mcmc = pickle.load(f)
mcmc.post_warmup_state = mcmc.last_state
mcmc.run(5, *mcmc._args, extra_fields=("num_steps",))
torch.save({{"samples": {{k: v.cpu() for k, v in mcmc.get_samples().items()}},
            "num_steps": mcmc.get_extra_fields()["num_steps"].cpu()}}, {out!r})
"""


def test_resume_in_another_process(device, tmp_path):
    """Cross-process checkpoint: warm up here, pickle to a file, resume in a fresh Python
    process; its draws and tree sizes equal the in-process continuation bitwise."""
    X, y = datasets.covtype_synthetic(n_rows=3000, seed=0)
    mcmc = MCMC(NUTS(P.logistic_regression), num_warmup=60, num_samples=8, num_chains=32)
    mcmc.warmup(4, X, y)
    blob, out = tmp_path / "mcmc.pkl", tmp_path / "out.pt"
    with open(blob, "wb") as f:
        pickle.dump(mcmc, f)
    mcmc.post_warmup_state = mcmc.last_state
    mcmc.run(5, X, y, extra_fields=("num_steps",))
    code = _CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"), blob=str(blob), out=str(out))
    subprocess.run([sys.executable, "-c", code], check=True, timeout=300)
    got = torch.load(out, weights_only=True)
    torch.testing.assert_close(got["samples"]["coefs"], mcmc.get_samples()["coefs"].cpu(), rtol=0, atol=0)
    torch.testing.assert_close(got["num_steps"], mcmc.get_extra_fields()["num_steps"].cpu(), rtol=0, atol=0)


def test_kernel_state_pickles_and_resumes(device):
    """The functional surface: a state returned by kernel.sample() pickles (its engine's
    current arena goes with it) and a fresh kernel resumes it with the model args."""
    k = NUTS(P.eight_schools)
    st = k.init(3, 30, model_args=ES, num_chains=16)
    for _ in range(35):
        st = k.sample(st, ES, {})
    blob = pickle.dumps(st)
    ref = [st := k.sample(st, ES, {}) for _ in range(3)]
    k2 = pickle.loads(pickle.dumps(NUTS(P.eight_schools)))
    st2 = pickle.loads(blob)
    for r in ref:
        st2 = k2.sample(st2, ES, {})
        torch.testing.assert_close(st2.z["theta"], r.z["theta"], rtol=0, atol=0)
        torch.testing.assert_close(st2.num_steps, r.num_steps, rtol=0, atol=0)


def test_postprocess_fn(device):
    """MCMC(postprocess_fn=fn): fn receives the unconstrained site values (tau on the log
    scale, as the reference's z) and its output is what get_samples returns; print_summary
    keeps the sample sites unless exclude_deterministic=False."""
    def fn(z):
        return {"mu": z["mu"], "tau": torch.exp(z["tau"]), "theta": z["theta"], "log_tau": z["tau"],
                "theta2": 2.0 * z["theta"]}

    ref = MCMC(NUTS(P.eight_schools), num_warmup=50, num_samples=20, num_chains=16)
    ref.run(2, *ES)
    m = MCMC(NUTS(P.eight_schools), num_warmup=50, num_samples=20, num_chains=16, postprocess_fn=fn)
    m.run(2, *ES)
    a, b = ref.get_samples(), m.get_samples()
    assert set(b) == {"mu", "tau", "theta", "log_tau", "theta2"}
    torch.testing.assert_close(b["mu"], a["mu"], rtol=0, atol=0)
    torch.testing.assert_close(b["theta2"], 2.0 * a["theta"], rtol=0, atol=0)
    torch.testing.assert_close(b["tau"], a["tau"], rtol=2e-6, atol=0)  # host exp vs device exp
    assert m.get_samples(group_by_chain=True)["log_tau"].shape == (16, 20)
    assert set(m._site_arrays(True, include_deterministic=False)) == {"mu", "tau", "theta"}


def test_bound_potentials_pickle_unbound(device):
    """A bound potential pickles without its device data: the packed split-bf16 covtype image
    (`packed`, set to None in __init__) and a whitened potential's whitening go back to their
    unbound values, workspaces are dropped; the copy binds again and evaluates identically."""
    from numpyro_amd import native
    from numpyro_amd.dense import WhitenedPotential

    X, y = datasets.covtype_synthetic(n_rows=2000, seed=2)
    pot = P.LogisticRegression(X, y)
    pot.bind(64, 64, "cuda:0")
    assert pot.packed is not None and pot.packed.is_cuda
    blob = pickle.dumps(pot)
    cp = pickle.loads(blob)
    assert cp.packed is None and not hasattr(cp, "workspace")

    def cuda_tensors(obj):
        return [k for k, v in obj.__dict__.items() if isinstance(v, torch.Tensor) and v.is_cuda]

    assert not cuda_tensors(cp)
    cp.bind(64, 64, "cuda:0")
    z = (0.1 * torch.randn(55, 64, generator=torch.Generator().manual_seed(0))).cuda()
    outs = []
    for p_ in (pot, cp):
        g, pe = torch.empty_like(z), torch.empty(64, device="cuda")
        ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=64, ldc=64)
        p_.evaluate(ev, native.stream_ptr())
        outs.append((g, pe))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    wp = WhitenedPotential(P.funnel.potential(20))
    wp.bind(64, 64, "cuda:0")
    assert wp.whitening is not None
    wc = pickle.loads(pickle.dumps(wp))
    assert wc.whitening is None and not cuda_tensors(wc) and not cuda_tensors(wc.base)
