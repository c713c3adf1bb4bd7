"""Posterior diagnostics over [chains, draws, ...] arrays (host NumPy, float64), with the
semantics of numpyro/diagnostics.py: split Gelman-Rubin (:64-80), Geyer initial
monotone sequence ESS from FFT autocovariance (:101-203), HPDI (:206-231), summary and
print_summary tables (:234-342).  Accepts torch tensors as well as arrays."""
from __future__ import annotations

from collections import OrderedDict
from itertools import product

import numpy as np

__all__ = ["autocorrelation", "autocovariance", "effective_sample_size", "gelman_rubin", "hpdi",
           "split_gelman_rubin", "summary", "print_summary", "print_summary_table"]


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _chain_variances(x):
    """(within-chain variance W, pooled estimator var+) for x [C, N, ...]."""
    C, N = x.shape[:2]
    w = x.var(axis=1, ddof=1).mean(axis=0)
    est = w * (N - 1) / N
    if C > 1:
        est = est + x.mean(axis=1).var(axis=0, ddof=1)
    else:
        w = est
    return w, est


def gelman_rubin(x):
    x = _np(x)
    assert x.ndim >= 2 and x.shape[0] >= 2 and x.shape[1] >= 2
    w, est = _chain_variances(x)
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.sqrt(est / w)


def split_gelman_rubin(x):
    x = _np(x)
    assert x.ndim >= 2 and x.shape[1] >= 4
    half = x.shape[1] // 2
    return gelman_rubin(np.concatenate([x[:, :half], x[:, -half:]], axis=0))


def _next_fast_len(n):
    if n <= 2:
        return n
    while True:
        m = n
        for p in (2, 3, 5):
            while m % p == 0:
                m //= p
        if m == 1:
            return n
        n += 1


def autocorrelation(x, axis=0, bias=True):
    x = _np(x)
    n = x.shape[axis]
    m2 = 2 * _next_fast_len(n)
    y = np.swapaxes(x, axis, -1)
    y = y - y.mean(axis=-1, keepdims=True)
    f = np.fft.rfft(y, n=m2, axis=-1)
    ac = np.fft.irfft(f * np.conjugate(f), n=m2, axis=-1)[..., :n]
    if not bias:
        ac = ac / np.arange(n, 0.0, -1)
    with np.errstate(invalid="ignore", divide="ignore"):
        ac = (ac / ac[..., :1]).astype(np.float64)
    return np.swapaxes(ac, axis, -1)


def autocovariance(x, axis=0, bias=True):
    x = _np(x)
    return autocorrelation(x, axis, bias) * x.var(axis=axis, keepdims=True)


def effective_sample_size(x, bias=True):
    x = _np(x).astype(np.float64)
    assert x.ndim >= 2 and x.shape[1] >= 2
    gamma = autocovariance(x, axis=1, bias=bias)
    w, est = _chain_variances(x)
    rho = 1.0 - (w - gamma.mean(axis=0)) / est
    rho[0] = 1.0
    pairs = rho[:-1:2, ...] + rho[1::2, ...]  # Geyer initial positive sequence
    mono = np.concatenate([pairs[:1], np.minimum.accumulate(np.clip(pairs[1:, ...], 0, None), axis=0)],
                          axis=0)
    tau = -1.0 + 2.0 * mono.sum(axis=0)
    return np.prod(x.shape[:2]) / tau


def hpdi(x, prob=0.90, axis=0):
    x = np.swapaxes(_np(x), axis, 0)
    xs = np.sort(x, axis=0)
    mass = x.shape[0]
    k = int(prob * mass)
    width = xs[k:] - xs[:mass - k]
    start = width.argmin(axis=0)
    lo = np.take_along_axis(xs, start[None, ...], axis=0)
    hi = np.take_along_axis(xs, (start + k)[None, ...], axis=0)
    return np.concatenate([np.swapaxes(lo, axis, 0), np.swapaxes(hi, axis, 0)], axis=axis)


def summary(samples, prob=0.90, group_by_chain=True):
    if not isinstance(samples, dict):
        samples = {"Param:0": samples}
    out = {}
    for name, value in samples.items():
        value = _np(value)
        if not group_by_chain:
            value = value[None, ...]
        if value.size == 0:
            continue
        value = value.astype(np.float64)
        flat = value.reshape((-1,) + value.shape[2:])
        h = hpdi(flat, prob=prob)
        out[name] = OrderedDict([
            ("mean", flat.mean(axis=0)),
            ("std", flat.std(axis=0, ddof=1)),
            ("median", np.median(flat, axis=0)),
            ("{:.1f}%".format(50 * (1 - prob)), h[0]),
            ("{:.1f}%".format(50 * (1 + prob)), h[1]),
            ("n_eff", effective_sample_size(value)),
            ("r_hat", split_gelman_rubin(value)),
        ])
    return out


def print_summary(samples, prob=0.90, group_by_chain=True):
    if not isinstance(samples, dict):
        samples = {"Param:0": samples}
    if not group_by_chain:
        samples = {k: _np(v)[None, ...] for k, v in samples.items()}
    print_summary_table(summary(samples, prob, group_by_chain=True), prob)


def print_summary_table(table, prob=0.90):
    """Print a {site: OrderedDict(stat -> array)} table as numpyro's print_summary does."""
    if not table:
        return
    table = {k: OrderedDict((s, _np(v)) for s, v in st.items()) for k, st in table.items()}
    width = max(max(len(k) + 2 + 3 * st["mean"].ndim for k, st in table.items()), 10)
    name_fmt = "{:>" + str(width) + "}"
    cols = [""] + list(next(iter(table.values())).keys())
    print()
    print((name_fmt + " {:>9}" * 7).format(*cols))
    row_fmt = name_fmt + " {:>9.2f}" * 7
    for name, stats in table.items():
        shape = stats["mean"].shape
        if len(shape) == 0:
            print(row_fmt.format(name, *[float(v) for v in stats.values()]))
        else:
            for idx in product(*map(range, shape)):
                label = name + "[{}]".format(",".join(map(str, idx)))
                print(row_fmt.format(label, *[float(v[idx]) for v in stats.values()]))
    print()
