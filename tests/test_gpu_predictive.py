"""Posterior predictive on the GPU (numpyro_amd.infer.Predictive, csrc/predictive.hip) vs the
NumPy oracle on the same Philox stream (oracle/predictive.py), plus distribution checks.
Tolerances: Bernoulli draws may differ only where U and p agree to f32 rounding (<= 0.1% of
draws); Normal draws within 1e-4 of the float64 oracle (f32 logf / sincosf in Box-Muller)."""
import numpy as np
import pytest
import torch

from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS, Predictive
from oracle import predictive as OPred

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def device():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda:0")


def test_logreg_predictive_matches_oracle(device):
    rs = np.random.RandomState(0)
    N, D, S = 3000, 55, 40
    X = rs.randn(N, D).astype(np.float32) * 0.3
    coefs = rs.randn(S, D).astype(np.float32)
    pred = Predictive(P.logistic_regression, {"coefs": torch.from_numpy(coefs)})
    out = pred(7, torch.from_numpy(X).to(device), None)["obs"]
    assert out.shape == (S, N) and out.dtype == torch.int32
    got = out.cpu().numpy()
    ref, p, u = OPred.predict_logreg(X, coefs, 7)
    mismatch = got != ref
    assert mismatch.mean() <= 1e-3
    assert np.all(np.abs(u[mismatch] - p[mismatch]) < 1e-5)
    # frequency of ones follows p
    np.testing.assert_allclose(got.mean(), p.mean(), atol=0.01)


def test_predictive_batch_ndims_and_observed_passthrough(device):
    rs = np.random.RandomState(1)
    X = rs.randn(500, 5).astype(np.float32)
    labels = (rs.rand(500) < 0.5).astype(np.float32)
    coefs = rs.randn(4, 6, 5).astype(np.float32)  # [chains, draws, D]
    pred = Predictive(P.logistic_regression, {"coefs": torch.from_numpy(coefs)}, batch_ndims=2)
    out = pred(3, X, None)
    assert out["obs"].shape == (4, 6, 500)
    flat = Predictive(P.logistic_regression, {"coefs": torch.from_numpy(coefs.reshape(24, 5))})(3, X, None)
    assert torch.equal(flat["obs"].reshape(4, 6, 500), out["obs"])
    # observed data passed: the site keeps it (numpyro.sample with obs=...)
    kept = Predictive(P.logistic_regression, {"coefs": torch.from_numpy(coefs.reshape(24, 5))})(3, X, labels)
    assert torch.equal(kept["obs"].cpu(), torch.from_numpy(labels.astype(np.int32)).expand(24, 500))
    # return_sites may name substituted latent sites
    both = Predictive(P.logistic_regression, {"coefs": torch.from_numpy(coefs.reshape(24, 5))},
                      return_sites=["coefs", "obs"])(3, X, None)
    assert set(both) == {"coefs", "obs"} and both["coefs"].shape == (24, 5)


def test_eight_schools_predictive_after_mcmc(device):
    J = 8
    sigma, y = datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y
    mcmc = MCMC(NUTS(P.eight_schools), num_warmup=200, num_samples=200, num_chains=8, progress_bar=False)
    mcmc.run(0, J, sigma, y)
    samples = mcmc.get_samples()
    out = Predictive(P.eight_schools, samples)(11, J, sigma)["obs"]
    assert out.shape == (1600, J)
    theta = samples["theta"].cpu().numpy().astype(np.float64)
    ref = OPred.predict_normal(theta, sigma, 11)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-4, atol=1e-4 * np.max(sigma))
    # predictive spread = posterior spread of theta + observation noise
    var = out.cpu().numpy().var(0)
    np.testing.assert_allclose(var, theta.var(0) + np.asarray(sigma) ** 2, rtol=0.15)


def test_bnn_predictive_matches_oracle(device):
    rs = np.random.RandomState(2)
    N, Dx, H, Dy, S = 40, 3, 7, 1, 16
    X = rs.randn(N, Dx).astype(np.float32)
    samples = {"prec_obs": rs.gamma(3.0, 1.0, S).astype(np.float32),
               "w1": rs.randn(S, Dx, H).astype(np.float32), "w2": rs.randn(S, H, H).astype(np.float32),
               "w3": rs.randn(S, H, Dy).astype(np.float32)}
    out = Predictive(P.bnn, {k: torch.from_numpy(v) for k, v in samples.items()})(5, X, None, H)["Y"]
    assert out.shape == (S, N, Dy)
    ref = OPred.predict_bnn(X, samples["prec_obs"], samples["w1"], samples["w2"], samples["w3"], 5)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-4, atol=1e-4)
