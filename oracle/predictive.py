"""ORACLE (test infrastructure only) — posterior predictive draws of the fused models'
observed sites, in NumPy, on the device's Philox stream (csrc/predictive.hip).

Follows numpyro/infer/util.py:803-885 (_predictive: the model re-run with each posterior
sample substituted, observed sites drawn from their likelihood) for
examples/covtype.py:66-71 (obs ~ Bernoulli(logits = X @ coefs); BernoulliLogits.sample =
random.bernoulli(key, expit(logits)): U < p, numpyro/distributions/discrete.py:130-135),
README.md:47-55 (obs ~ Normal(theta, sigma)) and examples/bnn.py:43-74 (Y ~ Normal(
tanh(tanh(X w1) w2) w3, 1/sqrt(prec_obs))).  The uniforms / normals are the Philox words of
event EV_PREDICT keyed (seed, sample, site 0, element) — the device's stream; parity with
the reference's jax.random stream is unpinned, parity of the distributions
is what the statistical tests check.
"""
from __future__ import annotations

import numpy as np

from . import philox


def _words(seed, S, n):
    s = np.arange(S)[:, None]
    i = np.arange(n)[None, :]
    return philox.rng(seed, s, 0, philox.EV_PREDICT, i, 0)  # [S, n, 4]


def predict_logreg(X, coefs, seed):
    """X [N, D], coefs [S, D] -> (draws [S, N] int32, probabilities [S, N], uniforms [S, N])."""
    logits = np.asarray(coefs, np.float64) @ np.asarray(X, np.float64).T
    p = 1.0 / (1.0 + np.exp(-logits))
    u = philox.u01(_words(seed, p.shape[0], p.shape[1])[..., 0]).astype(np.float64)
    return (u < p).astype(np.int32), p, u


def predict_normal(loc, scale, seed):
    """loc [S, J], scale [J] -> loc + scale * z, z the first Box-Muller normal of each block."""
    loc = np.asarray(loc, np.float64)
    w = _words(seed, loc.shape[0], loc.shape[1])
    z, _ = philox.box_muller(w[..., 0], w[..., 1])
    return loc + np.asarray(scale, np.float64)[None, :] * z.astype(np.float64)


def bnn_mean(X, w1, w2, w3):
    """examples/bnn.py:43-74 network output for one sample (float64)."""
    z1 = np.tanh(np.asarray(X, np.float64) @ w1)
    z2 = np.tanh(z1 @ w2)
    return z2 @ w3


def predict_bnn(X, prec_obs, w1, w2, w3, seed):
    """X [N, Dx]; per-sample prec_obs [S], w1 [S, Dx, H], w2 [S, H, H], w3 [S, H, Dy] -> [S, N, Dy]."""
    S = len(prec_obs)
    N, Dy = np.shape(X)[0], np.shape(w3)[-1]
    w = _words(seed, S, N * Dy)
    z, _ = philox.box_muller(w[..., 0], w[..., 1])
    z = z.astype(np.float64).reshape(S, N, Dy)
    out = np.empty((S, N, Dy))
    for s in range(S):
        out[s] = bnn_mean(X, w1[s], w2[s], w3[s]) + z[s] / np.sqrt(float(prec_obs[s]))
    return out
