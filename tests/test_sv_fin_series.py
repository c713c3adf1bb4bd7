"""The stochastic-volatility potential's StudentT normaliser differences (csrc/nmx_wide_models.h,
nmx_lgamma_digamma_half_diff): L = lgamma(x) - lgamma(x + 1/2) and Psi = digamma(x) -
digamma(x + 1/2) by recurrence to x >= 8 and differenced Stirling series.  This restates the
device formula step by step in Python double and checks it against scipy over the range nu / 2
takes (nu = e^a, a in [-4, 5], and [0.02, 60]); the device function itself is checked against the
float64 oracle potential on the GPU (tests/test_gpu_potentials.py, SV at T = 2517)."""
import math

import numpy as np
from scipy.special import digamma, gammaln


def half_diff(x):
    X, pn, pd, num, den = x, 1.0, 1.0, 0.0, 1.0
    while X < 8.0:
        h = X + 0.5
        q = X * h
        pn *= X
        pd *= h
        num = num * q + 0.5 * den
        den *= q
        X += 1.0
    H = X + 0.5
    rxh = 1.0 / (X * H)
    inv, invh = H * rxh, X * rxh
    u = 0.5 * inv
    t = u / (2.0 + u)
    t2 = t * t
    l1p = 2.0 * t * (1.0 + t2 * (1 / 3 + t2 * (1 / 5 + t2 * (1 / 7 + t2 * (1 / 9 + t2 * (1 / 11))))))

    def lser(iz):
        iz2 = iz * iz
        return iz * (1 / 12 - iz2 * (1 / 360 - iz2 * (1 / 1260 - iz2 * (1 / 1680 - iz2 / 1188))))

    def pser(iz):
        iz2 = iz * iz
        return iz2 * (1 / 12 - iz2 * (1 / 120 - iz2 * (1 / 252 - iz2 * (1 / 240 - iz2 / 132))))

    rpd = 1.0 / (pd * den)
    r = pn * den * rpd
    L = -0.5 * math.log(X * r * r) - X * l1p + 0.5 + lser(inv) - lser(invh)
    Psi = -l1p - 0.5 * inv + 0.5 * invh - pser(inv) + pser(invh) - num * pd * rpd
    return L, Psi


def test_half_diffs_match_scipy():
    xs = np.concatenate([np.linspace(0.02, 1.0, 200), np.linspace(1.0, 60.0, 500),
                         0.5 * np.exp(np.linspace(-4.0, 5.0, 300))])
    for x in xs:
        L, P = half_diff(float(x))
        assert abs(L - (gammaln(x) - gammaln(x + 0.5))) <= 2e-13, x
        assert abs(P - (digamma(x) - digamma(x + 0.5))) <= 2e-13, x
