"""ORACLE (test infrastructure only) — potential energies and hand-derived gradients of
the benchmark models, in NumPy.

U(z) = -log p(z) in unconstrained space (numpyro/infer/util.py:302-327): log-densities
follow numpyro/distributions (cited per term) and positive sites carry the ExpTransform
log-Jacobian +u (numpyro/distributions/transforms.py:561-569).  The flattened z follows
ravel_pytree of the site dict in sorted key order.  Pinned in
tests/test_oracle_potentials.py against scipy.stats log-densities and finite differences
(the reference's own oracle strategy, test/test_distributions.py:1505-1560,1851-1905).
"""
from __future__ import annotations

import numpy as np
from scipy.special import gammaln, digamma

LOG_2PI = float(np.log(2 * np.pi))


def _lpN(x, loc, scale):
    """Normal.log_prob, continuous.py:2200-2204."""
    return -0.5 * ((x - loc) / scale) ** 2 - np.log(np.sqrt(2 * np.pi) * scale)


class LogisticRegression:
    """examples/covtype.py:66-71: coefs ~ Normal(0,1)^D, obs ~ Bernoulli(logits=X@coefs).

    BernoulliLogits.log_prob = -binary_cross_entropy_with_logits (discrete.py:137-139,
    distributions/util.py:295-298).
    """

    sites = (("coefs", None, "real"),)

    def __init__(self, X, y, dtype=np.float64):
        self.X = np.asarray(X, dtype)
        self.y = np.asarray(y, dtype)
        self.dtype = dtype
        self.dim = self.X.shape[1]

    def pe_grad(self, z):
        f = self.dtype
        z = np.asarray(z, f)
        l = self.X @ z
        bce = np.maximum(l, f(0)) + np.log1p(np.exp(-np.abs(l))) - l * self.y
        pe = bce.sum(dtype=f) + (f(0.5) * z * z).sum(dtype=f) + f(self.dim * 0.5 * LOG_2PI)
        sig = f(1) / (f(1) + np.exp(-l))
        g = self.X.T @ (sig - self.y) + z
        return f(pe), g.astype(f)

    def pe_grad_batch(self, Z):
        """Z [C, D] -> (pe [C], grad [C, D]) in float64."""
        Z = np.asarray(Z, np.float64)
        X = np.asarray(self.X, np.float64)  # no copy when the potential holds float64 data
        y = np.asarray(self.y, np.float64)
        L = X @ Z.T  # [N, C]
        bce = np.maximum(L, 0) + np.log1p(np.exp(-np.abs(L))) - L * y[:, None]
        pe = bce.sum(0) + 0.5 * (Z * Z).sum(1) + self.dim * 0.5 * LOG_2PI
        sig = 1.0 / (1.0 + np.exp(-L))
        G = (X.T @ (sig - y[:, None])).T + Z
        return pe, G


class EightSchools:
    """README.md:47-55 (centred): mu ~ N(0,5), tau ~ HalfCauchy(5), theta_j ~ N(mu,tau),
    y_j ~ N(theta_j, sigma_j).  z = (mu, log tau, theta[8])."""

    sites = (("mu", None, "real"), ("tau", None, "positive"), ("theta", 8, "real"))

    def __init__(self, y, sigma, dtype=np.float64):
        self.y = np.asarray(y, np.float64)
        self.sigma = np.asarray(sigma, np.float64)
        self.dtype = dtype
        self.dim = 2 + len(self.y)

    def log_joint(self, z):
        mu, u, theta = z[0], z[1], z[2:]
        tau = np.exp(u)
        lp = _lpN(mu, 0.0, 5.0)
        # HalfCauchy(5).log_prob = Cauchy.log_prob + log 2 (continuous.py:720-722, :238-244)
        lp += -np.log(np.pi) - np.log(5.0) - np.log1p((tau / 5.0) ** 2) + np.log(2.0)
        lp += u  # ExpTransform log|J|
        lp += _lpN(theta, mu, tau).sum()
        lp += _lpN(self.y, theta, self.sigma).sum()
        return lp

    def pe_grad(self, z):
        z = np.asarray(z, np.float64)
        mu, u, theta = z[0], z[1], z[2:]
        tau2 = np.exp(2 * u)
        g = np.empty_like(z)
        g[0] = mu / 25.0 - ((theta - mu) / tau2).sum()
        g[1] = (2 * tau2 / 25.0) / (1 + tau2 / 25.0) - (((theta - mu) ** 2) / tau2 - 1).sum() - 1
        g[2:] = (theta - mu) / tau2 + (theta - self.y) / self.sigma ** 2
        return self.dtype(-self.log_joint(z)), g.astype(self.dtype)


class Funnel:
    """examples/funnel.py:44-46 (centred): y ~ N(0,3), x ~ N(0, exp(y/2))^(dim-1).
    z = (x[dim-1], y) (sorted site names)."""

    def __init__(self, dim=10, dtype=np.float64):
        self.dim = dim
        self.K = dim - 1
        self.dtype = dtype
        self.sites = (("x", self.K, "real"), ("y", None, "real"))

    def log_joint(self, z):
        x, y = z[:-1], z[-1]
        return _lpN(y, 0.0, 3.0) + _lpN(x, 0.0, np.exp(y / 2)).sum()

    def pe_grad(self, z):
        z = np.asarray(z, np.float64)
        x, y = z[:-1], z[-1]
        e = np.exp(-y)
        g = np.empty_like(z)
        g[:-1] = x * e
        g[-1] = y / 9.0 + self.K / 2.0 - 0.5 * e * (x * x).sum()
        return self.dtype(-self.log_joint(z)), g.astype(self.dtype)


class FunnelNonCentered:
    """examples/funnel.py:49, reparam(model, config={"x": LocScaleReparam(0)}) with
    numpyro/infer/reparam.py:104-145 at centered = 0: x_decentered ~ N(0, 1)^(dim-1),
    y ~ N(0, 3); deterministic x = exp(y/2) * x_decentered.  z = (x_decentered[dim-1], y)."""

    def __init__(self, dim=10, dtype=np.float64):
        self.dim = dim
        self.K = dim - 1
        self.dtype = dtype
        self.sites = (("x_decentered", self.K, "real"), ("y", None, "real"))

    def log_joint(self, z):
        xd, y = z[:-1], z[-1]
        return _lpN(y, 0.0, 3.0) + _lpN(xd, 0.0, 1.0).sum()

    def pe_grad(self, z):
        z = np.asarray(z, np.float64)
        g = z.copy()
        g[-1] = z[-1] / 9.0
        return self.dtype(-self.log_joint(z)), g.astype(self.dtype)

    def deterministic(self, z):
        z = np.asarray(z, np.float64)
        return {"x": np.exp(z[..., -1:] / 2) * z[..., :-1]}


class StochasticVolatility:
    """examples/stochastic_volatility.py:57-65: sigma ~ Exp(50), s ~ GRW(sigma, T),
    nu ~ Exp(0.1), r ~ StudentT(nu, 0, exp(s)).  z = (log nu, s[T], log sigma)."""

    def __init__(self, returns, dtype=np.float64):
        self.r = np.asarray(returns, np.float64)
        self.T = len(self.r)
        self.dim = self.T + 2
        self.dtype = dtype
        self.sites = (("nu", None, "positive"), ("s", self.T, "real"), ("sigma", None, "positive"))

    def log_joint(self, z):
        a, s, b = z[0], z[1:-1], z[-1]
        nu, sigma = np.exp(a), np.exp(b)
        lp = np.log(50.0) - 50.0 * sigma + b  # Exponential.log_prob (continuous.py:473-475) + J
        d = np.diff(s, prepend=0.0)  # GRW: N(0,sigma).lp(s0) + sum N(s_{t-1},sigma).lp(s_t)
        lp += _lpN(d, 0.0, sigma).sum()
        lp += np.log(0.1) - 0.1 * nu + a
        # StudentT.log_prob (continuous.py:2373-2384), loc 0, scale exp(s)
        y = self.r / np.exp(s)
        zt = s + 0.5 * np.log(nu) + 0.5 * np.log(np.pi) + gammaln(0.5 * nu) - gammaln(0.5 * (nu + 1))
        lp += (-0.5 * (nu + 1.0) * np.log1p(y ** 2 / nu) - zt).sum()
        return lp

    def pe_grad(self, z):
        z = np.asarray(z, np.float64)
        a, s, b = z[0], z[1:-1], z[-1]
        nu, sigma = np.exp(a), np.exp(b)
        T = self.T
        d = np.diff(s, prepend=0.0)
        q = self.r ** 2 * np.exp(-2 * s) / nu
        g = np.empty_like(z)
        d_next = np.append(d[1:], 0.0)
        gs = -(d - d_next) / sigma ** 2 + (nu + 1) * q / (1 + q) - 1
        gb = -50.0 * sigma + 1 + (d ** 2).sum() / sigma ** 2 - T
        ga = nu * (-0.1 + (-0.5 * np.log1p(q) + 0.5 * (nu + 1) * q / (nu * (1 + q)) - 0.5 / nu
                          - 0.5 * digamma(nu / 2) + 0.5 * digamma((nu + 1) / 2)).sum()) + 1
        g[0], g[1:-1], g[-1] = ga, gs, gb
        return self.dtype(-self.log_joint(z)), (-g).astype(self.dtype)


class BNN:
    """examples/bnn.py:43-74: w1 [Dx,H], w2 [H,H], w3 [H,1] ~ N(0,1), prec_obs ~ Gamma(3,1),
    Y ~ N(tanh(tanh(X w1) w2) w3, 1/sqrt(prec)).  z = (log prec, w1, w2, w3) row-major."""

    def __init__(self, X, Y, H, dtype=np.float64):
        self.X = np.asarray(X, np.float64)
        self.Y = np.asarray(Y, np.float64).reshape(-1)
        self.N, self.Dx = self.X.shape
        self.H = H
        self.dim = 1 + self.Dx * H + H * H + H
        self.dtype = dtype
        self.sites = (("prec_obs", None, "positive"), ("w1", (self.Dx, H), "real"),
                      ("w2", (H, H), "real"), ("w3", (H, 1), "real"))

    def unpack(self, z):
        H, Dx = self.H, self.Dx
        u = z[0]
        o = 1
        w1 = z[o:o + Dx * H].reshape(Dx, H); o += Dx * H
        w2 = z[o:o + H * H].reshape(H, H); o += H * H
        w3 = z[o:o + H].reshape(H, 1)
        return u, w1, w2, w3

    def log_joint(self, z):
        u, w1, w2, w3 = self.unpack(z)
        p = np.exp(u)
        h1 = np.tanh(self.X @ w1)
        h2 = np.tanh(h1 @ w2)
        yhat = (h2 @ w3).reshape(-1)
        lp = _lpN(w1, 0, 1).sum() + _lpN(w2, 0, 1).sum() + _lpN(w3, 0, 1).sum()
        lp += (3.0 - 1) * np.log(p) - p - gammaln(3.0) + u  # Gamma(3,1) (continuous.py:515-524) + J
        lp += _lpN(self.Y, yhat, 1.0 / np.sqrt(p)).sum()
        return lp

    def pe_grad(self, z):
        z = np.asarray(z, np.float64)
        u, w1, w2, w3 = self.unpack(z)
        p = np.exp(u)
        h1 = np.tanh(self.X @ w1)
        h2 = np.tanh(h1 @ w2)
        yhat = (h2 @ w3).reshape(-1)
        e = self.Y - yhat
        g_yhat = (-p * e)[:, None]  # dU/dyhat
        gw3 = w3 + h2.T @ g_yhat
        ga2 = (g_yhat @ w3.T) * (1 - h2 ** 2)
        gw2 = w2 + h1.T @ ga2
        ga1 = (ga2 @ w2.T) * (1 - h1 ** 2)
        gw1 = w1 + self.X.T @ ga1
        gu = -(3.0 - p + self.N / 2.0 - 0.5 * p * (e ** 2).sum())
        g = np.concatenate([[gu], gw1.ravel(), gw2.ravel(), gw3.ravel()])
        return self.dtype(-self.log_joint(z)), g.astype(self.dtype)


class IsoNormal:
    """Unnormalized N(mu, diag(sd^2)) test target (test/infer/test_mcmc.py:28-72)."""

    def __init__(self, mu, sd, dtype=np.float64):
        self.mu = np.asarray(mu, np.float64)
        self.sd = np.asarray(sd, np.float64)
        self.dim = len(self.mu)
        self.dtype = dtype

    def pe_grad(self, z):
        z = np.asarray(z, np.float64)
        d = (z - self.mu) / self.sd
        return self.dtype(0.5 * (d * d).sum()), (d / self.sd).astype(self.dtype)


class MVN:
    """Unnormalized N(mu, P^-1): U = 0.5 (z-mu)^T P (z-mu) (test/infer/test_mcmc.py:73-100,
    :313-343 targets)."""

    def __init__(self, prec, mu=None, dtype=np.float64):
        self.prec = np.asarray(prec, np.float64)
        self.dim = self.prec.shape[0]
        self.mu = np.zeros(self.dim) if mu is None else np.asarray(mu, np.float64)
        self.dtype = dtype

    def pe_grad(self, z):
        d = np.asarray(z, np.float64) - self.mu
        g = self.prec @ d
        return self.dtype(0.5 * d @ g), g.astype(self.dtype)
