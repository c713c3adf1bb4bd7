"""The stochastic-volatility potential's StudentT normaliser differences (csrc/nmx_wide_models.h,
nmx_lgamma_digamma_half_diff): L = lgamma(x) - lgamma(x + 1/2) and Psi = digamma(x) -
digamma(x + 1/2) by recurrence to x >= 8 and differenced Stirling series.  This restates the
device formula step by step in Python double and checks it against scipy over the range nu / 2
takes (nu = e^a, a in [-4, 5], and [0.02, 60]); the device function itself is checked against the
float64 oracle potential on the GPU (tests/test_gpu_potentials.py, SV at T = 2517)."""
import math

import numpy as np
from scipy.special import digamma, gammaln


def log_f64(y):
    """nmx_log_f64: y = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s) by ten series terms."""
    m, e = math.frexp(y)
    if m < 0.70710678118654752440:
        m *= 2.0
        e -= 1
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    p = 1.0 / 21
    for k in (19, 17, 15, 13, 11, 9, 7, 5, 3):
        p = 1.0 / k + s2 * p
    return e * 6.93147180369123816490e-01 + (2.0 * s + (2.0 * s * s2 * p + e * 1.90821492927058770002e-10))


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
    L = -0.5 * log_f64(X * r * r) - X * l1p + 0.5 + lser(inv) - lser(invh)
    Psi = -l1p - 0.5 * inv + 0.5 * invh - pser(inv) + pser(invh) - num * pd * rpd
    return L, Psi


def test_half_diffs_match_scipy():
    xs = np.concatenate([np.linspace(0.02, 1.0, 200), np.linspace(1.0, 60.0, 500),
                         0.5 * np.exp(np.linspace(-4.0, 5.0, 300))])
    for x in xs:
        L, P = half_diff(float(x))
        assert abs(L - (gammaln(x) - gammaln(x + 0.5))) <= 2e-13, x
        assert abs(P - (digamma(x) - digamma(x + 0.5))) <= 2e-13, x


def test_log_f64_within_two_ulp():
    for y in np.concatenate([np.logspace(-30, 30, 4001), np.linspace(0.5, 2.0, 2001)]):
        ref = math.log(float(y))
        assert abs(log_f64(float(y)) - ref) <= 2.0 * np.spacing(abs(ref)) + 1e-300, y
