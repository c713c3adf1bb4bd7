"""Pin oracle/potentials.py: log-densities against scipy.stats (the reference's
test_log_prob strategy, test/test_distributions.py:1505-1560) and gradients against
central finite differences (test_log_prob_gradient, :1851-1905)."""
import numpy as np
import pytest
from scipy import stats

from numpyro_amd import datasets
from oracle import potentials as P


def _fd_grad(f, z, eps=1e-5):
    g = np.zeros_like(z)
    for i in range(len(z)):
        zp, zm = z.copy(), z.copy()
        zp[i] += eps
        zm[i] -= eps
        g[i] = (f(zp) - f(zm)) / (2 * eps)
    return g


def _models():
    rs = np.random.RandomState(0)
    X = rs.randn(200, 5)
    y = (rs.rand(200) < 0.4).astype(float)
    Xb, Yb = datasets.bnn_data(N=20, D_X=3)
    return {
        "logreg": (P.LogisticRegression(X, y), 5),
        "eight_schools": (P.EightSchools(datasets.EIGHT_SCHOOLS_Y, datasets.EIGHT_SCHOOLS_SIGMA), 10),
        "funnel": (P.Funnel(12), 12),
        "funnel_noncentered": (P.FunnelNonCentered(12), 12),
        "sv": (P.StochasticVolatility(datasets.sp500_synthetic(T=40)), 42),
        "bnn": (P.BNN(Xb, Yb, H=4), 1 + 12 + 16 + 4),
    }


@pytest.mark.parametrize("name", ["logreg", "eight_schools", "funnel", "sv", "bnn"])
def test_gradient_matches_finite_differences(name):
    model, dim = _models()[name]
    assert model.dim == dim
    rs = np.random.RandomState(1)
    z = rs.uniform(-1, 1, dim)
    pe, g = model.pe_grad(z)
    g_fd = _fd_grad(lambda v: model.pe_grad(v)[0], z)
    np.testing.assert_allclose(g, g_fd, rtol=1e-4, atol=1e-4)


def test_logreg_matches_scipy():
    rs = np.random.RandomState(2)
    X = rs.randn(50, 4)
    y = (rs.rand(50) < 0.5).astype(float)
    z = rs.randn(4)
    m = P.LogisticRegression(X, y)
    p = 1 / (1 + np.exp(-(X @ z)))
    ref = stats.norm.logpdf(z).sum() + stats.bernoulli.logpmf(y, p).sum()
    np.testing.assert_allclose(-m.pe_grad(z)[0], ref, rtol=1e-10)


def test_eight_schools_matches_scipy():
    m = P.EightSchools(datasets.EIGHT_SCHOOLS_Y, datasets.EIGHT_SCHOOLS_SIGMA)
    z = np.linspace(-1, 1, 10)
    mu, tau, theta = z[0], np.exp(z[1]), z[2:]
    ref = (stats.norm.logpdf(mu, 0, 5) + stats.halfcauchy.logpdf(tau, scale=5) + z[1]
           + stats.norm.logpdf(theta, mu, tau).sum()
           + stats.norm.logpdf(datasets.EIGHT_SCHOOLS_Y, theta, datasets.EIGHT_SCHOOLS_SIGMA).sum())
    np.testing.assert_allclose(m.log_joint(z), ref, rtol=1e-7)


def test_sv_matches_scipy():
    r = datasets.sp500_synthetic(T=30).astype(np.float64)
    m = P.StochasticVolatility(r)
    rs = np.random.RandomState(3)
    z = rs.uniform(-1, 1, 32)
    a, s, b = z[0], z[1:-1], z[-1]
    nu, sigma = np.exp(a), np.exp(b)
    grw = stats.norm.logpdf(s[0], 0, sigma) + stats.norm.logpdf(s[1:], s[:-1], sigma).sum()
    ref = (stats.expon.logpdf(sigma, scale=1 / 50.0) + b + grw
           + stats.expon.logpdf(nu, scale=10.0) + a
           + stats.t.logpdf(r, nu, 0, np.exp(s)).sum())
    np.testing.assert_allclose(m.log_joint(z), ref, rtol=1e-9)


def test_bnn_matches_scipy():
    X, Y = datasets.bnn_data(N=15, D_X=3)
    m = P.BNN(X, Y, H=3)
    rs = np.random.RandomState(4)
    z = rs.uniform(-1, 1, m.dim)
    u, w1, w2, w3 = m.unpack(z)
    p = np.exp(u)
    yhat = (np.tanh(np.tanh(X.astype(float) @ w1) @ w2) @ w3).ravel()
    ref = (stats.norm.logpdf(z[1:]).sum() + stats.gamma.logpdf(p, 3.0, scale=1.0) + u
           + stats.norm.logpdf(Y.ravel(), yhat, 1 / np.sqrt(p)).sum())
    np.testing.assert_allclose(m.log_joint(z), ref, rtol=1e-9)


def test_covtype_synthetic_statistics():
    X, y = datasets.covtype_synthetic(n_rows=20000, seed=0)
    assert X.shape == (20000, 55) and X.dtype == np.float32
    assert np.all(X[:, -1] == 1.0)
    np.testing.assert_allclose(X[:, :-1].mean(0), 0, atol=1e-5)
    np.testing.assert_allclose(X[:, :-1].std(0), 1, atol=1e-4)
    assert 0.30 < y.mean() < 0.38  # 33.8% positives at full size


def test_funnel_noncentered_matches_scipy_and_reparam():
    """Non-centred funnel: log density = N(0,3).logpdf(y) + sum N(0,1).logpdf(x_dec), and the
    deterministic x = exp(y/2) x_dec has the centred model's conditional N(0, exp(y/2))."""
    rs = np.random.RandomState(3)
    m = P.FunnelNonCentered(6)
    for _ in range(5):
        z = rs.randn(6) * 1.5
        want = stats.norm(0, 3).logpdf(z[-1]) + stats.norm(0, 1).logpdf(z[:-1]).sum()
        np.testing.assert_allclose(m.log_joint(z), want, rtol=1e-12)
        x = m.deterministic(z)["x"]
        np.testing.assert_allclose(x, np.exp(z[-1] / 2) * z[:-1])
        # change of variables: the centred log density at (x, y) = non-centred - log|dx/dx_dec|
        np.testing.assert_allclose(P.Funnel(6).log_joint(np.append(x, z[-1])),
                                   m.log_joint(z) - 5 * z[-1] / 2, rtol=1e-10)
