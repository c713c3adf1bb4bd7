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
