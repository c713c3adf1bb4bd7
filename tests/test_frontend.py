"""Model front end (numpyro_amd/frontend.py): the reference's example
models, written with numpyro's primitives, trace to the fused potentials of their structure
with the model's site names; other structures (or changed priors) are refused."""
import numpy as np
import pytest

import numpyro_amd as numpyro
from numpyro_amd import datasets
from numpyro_amd import distributions as dist
from numpyro_amd import potentials as P
from numpyro_amd.frontend import potential_from_model, trace_model
import model_zoo as Z


def test_examples_map_to_their_kernels():
    X, y = datasets.covtype_synthetic(n_rows=500, seed=0)
    cases = [
        (Z.covtype_model, (X, y), P.LogisticRegression, {"coefs": (55,)}),
        (Z.eight_schools, (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y), P.EightSchools,
         {"mu": (), "tau": (), "theta": (8,)}),
        (Z.funnel, (10,), P.Funnel, {"x": (9,), "y": ()}),
        (Z.funnel_reparam, (10,), P.FunnelNonCentered, {"x_decentered": (9,), "y": ()}),
        (Z.stochastic_volatility, (datasets.sp500_synthetic(T=50),), P.StochasticVolatility,
         {"nu": (), "s": (50,), "sigma": ()}),
        (Z.bnn, datasets.bnn_data(N=40, D_X=3) + (6,), P.BNN,
         {"prec_obs": (), "w1": (3, 6), "w2": (6, 6), "w3": (6, 1)}),
    ]
    for model, args, cls, sites in cases:
        pot = potential_from_model(model, args)
        assert type(pot) is cls, model
        assert {n: tuple(s) for n, s, _ in pot.sites} == sites, model


def test_data_and_site_names_carry_over():
    X, y = datasets.covtype_synthetic(n_rows=300, seed=1)

    def model(features, labels):
        beta = numpyro.sample("beta", dist.Normal(np.zeros(features.shape[1]), np.ones(features.shape[1])))
        numpyro.sample("y", dist.Bernoulli(logits=features @ beta), obs=labels)

    pot = potential_from_model(model, (X, y))
    assert isinstance(pot, P.LogisticRegression) and pot.sites[0][0] == "beta"
    assert pot.N == 300 and pot.dim == 55


def test_trace_records_plates_and_shapes():
    t = trace_model(Z.eight_schools, (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y))
    assert t.sites["theta"].shape == (8,) and t.sites["theta"].plates == ("J",)
    assert t.sites["obs"].obs is not None


@pytest.mark.parametrize("change", ["prior", "likelihood", "structure"])
def test_unsupported_structures_are_refused(change):
    def m(J, sigma, y):
        mu = numpyro.sample("mu", dist.Normal(0, 5 if change != "prior" else 10))
        tau = numpyro.sample("tau", dist.HalfCauchy(5))
        with numpyro.plate("J", J):
            theta = numpyro.sample("theta", dist.Normal(mu, tau))
            if change == "likelihood":
                numpyro.sample("obs", dist.StudentT(4.0, theta, sigma), obs=y)
            else:
                numpyro.sample("obs", dist.Normal(theta, sigma), obs=y)
        if change == "structure":
            numpyro.sample("extra", dist.Exponential(1.0))

    with pytest.raises(NotImplementedError, match="no fused kernel"):
        potential_from_model(m, (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y))


def test_model_cannot_run_eagerly():
    with pytest.raises(RuntimeError, match="traces them"):
        Z.funnel(10)


def test_masked_likelihood_and_infer_options_are_refused():
    """A masked likelihood (obs_mask, primitives.py:177-191) or infer options change the
    potential: refused, not silently mapped onto the full-data kernel."""
    X, y = datasets.covtype_synthetic(n_rows=200, seed=2)

    def masked(features, labels):
        beta = numpyro.sample("beta", dist.Normal(np.zeros(55), np.ones(55)))
        numpyro.sample("y", dist.Bernoulli(logits=features @ beta), obs=labels, obs_mask=labels > 0)

    def enum(features, labels):
        beta = numpyro.sample("beta", dist.Normal(np.zeros(55), np.ones(55)), infer={"enumerate": "parallel"})
        numpyro.sample("y", dist.Bernoulli(logits=features @ beta), obs=labels)

    for m in (masked, enum):
        with pytest.raises(NotImplementedError, match="not supported"):
            potential_from_model(m, (X, y))


def test_model_deterministic_sites_are_evaluated():
    """numpyro.deterministic sites of the model (primitives.py:293-314) come back with the
    draws: the traced expressions evaluated over a batch of constrained site values."""
    import torch

    X, Y = datasets.bnn_data(N=20, D_X=3)

    def bnn_det(X, Y, D_H):
        w1 = numpyro.sample("w1", dist.Normal(np.zeros((3, D_H)), np.ones((3, D_H))))
        z1 = numpyro.deterministic("z1", Z.jnp.tanh(Z.jnp.matmul(X, w1)))
        w2 = numpyro.sample("w2", dist.Normal(np.zeros((D_H, D_H)), np.ones((D_H, D_H))))
        z2 = Z.jnp.tanh(Z.jnp.matmul(z1, w2))
        w3 = numpyro.sample("w3", dist.Normal(np.zeros((D_H, 1)), np.ones((D_H, 1))))
        z3 = numpyro.deterministic("z3", Z.jnp.matmul(z2, w3))
        prec = numpyro.sample("prec_obs", dist.Gamma(3.0, 1.0))
        numpyro.deterministic("sigma_obs", 1.0 / Z.jnp.sqrt(prec))
        with numpyro.plate("data", X.shape[0]):
            numpyro.sample("Y", dist.Normal(z3, 1.0 / Z.jnp.sqrt(prec)).to_event(1), obs=Y)

    pot = potential_from_model(bnn_det, (X, Y, 4))
    assert isinstance(pot, P.BNN)
    rs = np.random.RandomState(0)
    B = (5, 2)  # [chains, draws]
    vals = {"w1": rs.randn(*B, 3, 4), "w2": rs.randn(*B, 4, 4), "w3": rs.randn(*B, 4, 1),
            "prec_obs": rs.rand(*B) + 0.5}
    out = pot.deterministic({k: torch.tensor(v, dtype=torch.float32) for k, v in vals.items()})
    z1 = np.tanh(np.einsum("nd,cidh->cinh", X, vals["w1"]))
    z3 = np.einsum("cinh,cihk->cink", np.tanh(np.einsum("cinh,cihk->cink", z1, vals["w2"])), vals["w3"])
    np.testing.assert_allclose(out["z1"].numpy(), z1, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out["z3"].numpy(), z3, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(out["sigma_obs"].numpy(), 1 / np.sqrt(vals["prec_obs"]), rtol=1e-6)
    # vector operands: covtype logits as a deterministic site
    Xc, yc = datasets.covtype_synthetic(n_rows=50, seed=3)

    def cov_det(data, labels):
        coefs = numpyro.sample("coefs", dist.Normal(np.zeros(55), np.ones(55)))
        logits = numpyro.deterministic("logits", Z.jnp.dot(data, coefs))
        numpyro.sample("obs", dist.Bernoulli(logits=logits), obs=labels)

    pot = potential_from_model(cov_det, (Xc, yc))
    c = rs.randn(7, 55).astype(np.float32)
    out = pot.deterministic({"coefs": torch.from_numpy(c)})
    np.testing.assert_allclose(out["logits"].numpy(), c @ Xc.T, rtol=1e-4, atol=1e-4)


def test_constant_deterministic_broadcasts_and_bad_ops_fail_at_mapping():
    """A constant deterministic site (numpyro.deterministic('c', 3.0)) has one value per draw;
    an expression the evaluator does not support raises when the model is mapped, not after
    sampling."""
    import torch

    Xc, yc = datasets.covtype_synthetic(n_rows=50, seed=3)

    def cov_const(data, labels):
        coefs = numpyro.sample("coefs", dist.Normal(np.zeros(55), np.ones(55)))
        numpyro.deterministic("c", 3.0)
        numpyro.deterministic("v", np.arange(3.0))
        numpyro.sample("obs", dist.Bernoulli(logits=Z.jnp.dot(data, coefs)), obs=labels)

    pot = potential_from_model(cov_const, (Xc, yc))
    out = pot.deterministic({"coefs": torch.zeros(4, 2, 55)})
    assert out["c"].shape == (4, 2) and float(out["c"][3, 1]) == 3.0
    assert out["v"].shape == (4, 2, 3) and torch.equal(out["v"][1, 0], torch.arange(3.0))

    from numpyro_amd.jnp import Sym

    def cov_bad(data, labels):
        coefs = numpyro.sample("coefs", dist.Normal(np.zeros(55), np.ones(55)))
        numpyro.deterministic("odd", Sym("erf", (coefs,), (55,)))
        numpyro.sample("obs", dist.Bernoulli(logits=Z.jnp.dot(data, coefs)), obs=labels)

    with pytest.raises(NotImplementedError, match="'erf' is not supported"):
        potential_from_model(cov_bad, (Xc, yc))
