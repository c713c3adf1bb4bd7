"""Synthetic stand-ins for the benchmark datasets (no network: SURVEY.md §0.3, §8d).

Shapes follow the reference loaders (numpyro/examples/datasets.py): covtype features
(581012, 54) plus an intercept column (examples/covtype.py:44-62), SP500 returns (2517,),
and the bnn toy regression of examples/bnn.py:103-121.  Everything is seeded NumPy.
"""
from __future__ import annotations

import numpy as np

COVTYPE_N = 581012
COVTYPE_FEATURES = 54
SP500_T = 2517

# MAP estimate quoted in examples/covtype.py:79-139 (used as the generating truth).
COVTYPE_REF_COEFS = np.array([
    +2.03420663e00, -3.53567265e-02, -1.49223924e-01, -3.07049364e-01, -1.00028366e-01,
    -1.46827862e-01, -1.64167881e-01, -4.20344204e-01, +9.47479829e-02, -1.12681836e-02,
    +2.64442056e-01, -1.22087866e-01, -6.00568838e-02, -3.79419506e-01, -1.06668741e-01,
    -2.97053963e-01, -2.05253899e-01, -4.69537191e-02, -2.78072730e-02, -1.43250525e-01,
    -6.77954629e-02, -4.34899796e-03, +5.90927452e-02, +7.23133609e-02, +1.38526391e-02,
    -1.24497898e-01, -1.50733739e-02, -2.68872194e-02, -1.80925727e-02, +3.47936489e-02,
    +4.03552800e-02, -9.98773426e-03, +6.20188080e-02, +1.15002751e-01, +1.32145107e-01,
    +2.69109547e-01, +2.45785132e-01, +1.19035013e-01, -2.59744357e-02, +9.94279515e-04,
    +3.39266285e-02, -1.44057125e-02, -6.95222765e-02, -7.52013028e-02, +1.21171586e-01,
    +2.29205526e-02, +1.47308692e-01, -8.34354162e-02, -9.34122875e-02, -2.97472421e-02,
    -3.03937674e-01, -1.70958012e-01, -1.59496680e-01, -1.88516974e-01, -1.20889175e00,
], dtype=np.float64)


def covtype_synthetic(n_rows: int = COVTYPE_N, seed: int = 0):
    """Synthetic covtype: X ~ N(0,1) standardized per column + intercept column,
    y ~ Bernoulli(sigmoid(X @ ref_coefs)).  Returns (X float32 [n, 55], y float32 [n])."""
    rs = np.random.Generator(np.random.PCG64(seed))
    feats = rs.standard_normal((n_rows, COVTYPE_FEATURES), dtype=np.float32)
    mu = feats.mean(0, dtype=np.float64)
    sd = feats.std(0, dtype=np.float64)
    feats = ((feats - mu) / sd).astype(np.float32)
    X = np.empty((n_rows, COVTYPE_FEATURES + 1), np.float32)
    X[:, :COVTYPE_FEATURES] = feats
    X[:, COVTYPE_FEATURES] = 1.0
    logits = X.astype(np.float64) @ COVTYPE_REF_COEFS
    p = 1.0 / (1.0 + np.exp(-logits))
    y = (rs.random(n_rows) < p).astype(np.float32)
    return X, y


def covtype_structured(n_rows: int = COVTYPE_N, seed: int = 0):
    """Synthetic covtype with the real data's column structure (numpyro/examples/datasets.py
    COVTYPE: 10 quantitative columns, then one-hot wilderness area (4) and soil type (40)), all
    54 columns standardized as examples/covtype.py:48 does, + intercept.  Each one-hot group
    sums to one, so after standardization both groups are collinear with the intercept: the
    likelihood leaves two directions to the N(0, 1) prior while the others have posterior sd
    ~1/sqrt(N), which is why NUTS on the real covtype saturates its trees (~948 leapfrogs per
    transition, notebooks/source/logistic_regression.ipynb:237).  Soil types follow a skewed
    (Zipf-like) frequency as in the real data; quantitative columns are correlated Gaussians.
    y ~ Bernoulli(sigmoid(X @ ref_coefs)).  Returns (X float32 [n, 55], y float32 [n])."""
    rs = np.random.Generator(np.random.PCG64(seed))
    q = 10
    A = rs.standard_normal((q, q)) * 0.4 + np.eye(q)
    quant = (rs.standard_normal((n_rows, q)) @ A.T).astype(np.float32)
    wild_p = np.array([0.45, 0.05, 0.44, 0.06])
    soil_p = 1.0 / np.arange(1, 41) ** 1.3
    soil_p = soil_p[rs.permutation(40)]
    soil_p /= soil_p.sum()
    wild = rs.choice(4, size=n_rows, p=wild_p)
    soil = rs.choice(40, size=n_rows, p=soil_p)
    feats = np.zeros((n_rows, COVTYPE_FEATURES), np.float32)
    feats[:, :q] = quant
    feats[np.arange(n_rows), q + wild] = 1.0
    feats[np.arange(n_rows), q + 4 + soil] = 1.0
    mu = feats.mean(0, dtype=np.float64)
    sd = feats.std(0, dtype=np.float64)
    sd[sd == 0] = 1.0
    feats = ((feats - mu) / sd).astype(np.float32)
    X = np.empty((n_rows, COVTYPE_FEATURES + 1), np.float32)
    X[:, :COVTYPE_FEATURES] = feats
    X[:, COVTYPE_FEATURES] = 1.0
    logits = X.astype(np.float64) @ COVTYPE_REF_COEFS
    p = 1.0 / (1.0 + np.exp(-logits))
    y = (rs.random(n_rows) < p).astype(np.float32)
    return X, y


def sp500_synthetic(T: int = SP500_T, seed: int = 0):
    """Synthetic daily returns: log-vol random walk (sigma 0.02) + StudentT(10) noise."""
    rs = np.random.Generator(np.random.PCG64(seed))
    s = np.cumsum(rs.normal(0.0, 0.02, T)) - 4.5
    r = rs.standard_t(10.0, T) * np.exp(s)
    return r.astype(np.float32)


def bnn_data(N: int = 100, D_X: int = 3, sigma_obs: float = 0.05, seed: int = 0):
    """examples/bnn.py:103-121 restated with NumPy (X = powers of a linspace)."""
    rs = np.random.RandomState(seed)
    X = np.linspace(-1, 1, N)
    X = np.power(X[:, np.newaxis], np.arange(D_X))
    W = 0.5 * rs.randn(D_X)
    Y = X @ W + 0.5 * np.power(0.5 + X[:, 1], 2.0) * np.sin(4.0 * X[:, 1])
    Y += sigma_obs * rs.randn(N)
    Y = Y[:, np.newaxis]
    Y -= Y.mean()
    Y /= Y.std()
    return X.astype(np.float32), Y.astype(np.float32)


EIGHT_SCHOOLS_Y = np.array([28.0, 8.0, -3.0, 7.0, -1.0, 1.0, 18.0, 12.0], np.float32)
EIGHT_SCHOOLS_SIGMA = np.array([15.0, 10.0, 16.0, 11.0, 9.0, 11.0, 10.0, 18.0], np.float32)
