"""``Predictive``: posterior predictive draws for the fused models.

Mirrors ``numpyro.infer.Predictive`` (numpyro/infer/util.py:888-1090): constructed from a
model and a dict of posterior samples (``MCMC.get_samples()``, leading batch dims per
``batch_ndims``), called with ``(rng_key, *model_args, **model_kwargs)`` where the observed
argument is ``None``, it returns ``{site: [*batch_shape, *site_shape]}`` for every sample site
not in ``posterior_samples`` (the observed sites) plus any ``return_sites`` asked for.  The
reference re-runs the traced model once per sample under ``substitute`` (:803-885); here each
model's observed-site sampler is one HIP kernel over all samples (csrc/predictive.hip).

An observed site whose data is passed (not ``None``) keeps that data, as ``numpyro.sample``
with ``obs=`` does under the reference's Predictive.  Deterministic sites (the model's
``numpyro.deterministic`` and reparameterised sites such as the non-centred funnel's ``x``,
reparam.py:140-142) are returned by default, as the reference's ``_predictive`` does
(util.py:870-877), computed from the posterior samples.  Models: covtype logistic regression
(``obs``), eight schools (``obs``), BNN (``Y``), stochastic volatility (``r``: its returns are
both the observation and the series length, examples/stochastic_volatility.py:57-65, so -- as in
the reference -- the observed data come back), funnel and its LocScaleReparam form (no observed
site: deterministic ``x`` and any ``return_sites``, as examples/funnel.py:84-87 uses it).  Out of
scope (raise): guides / params (SVI), ``infer_discrete``, prior predictive (no posterior samples).
"""
from __future__ import annotations

import math
import warnings

import numpy as np
import torch

from .. import native
from .. import potentials as P
from ..native import check, lib, ptr
from ..random import key_to_seed


def _as_device(x, device):
    return torch.as_tensor(x if torch.is_tensor(x) else np.asarray(x), dtype=torch.float32).to(device).contiguous()


def _observed(value, S, device, dtype=torch.float32):
    """An observed site keeps its data (numpyro.sample with obs=...): [S, *shape]."""
    v = torch.as_tensor(value if torch.is_tensor(value) else np.asarray(value)).to(device, dtype)
    return v.unsqueeze(0).expand(S, *v.shape)


def _predict_logreg(samples, seed, device, data, labels=None, subsample_size=None):
    if subsample_size is not None:
        raise NotImplementedError("subsample_size is out of scope here")
    X = _as_device(data, device)
    N, D = X.shape
    coefs = samples["coefs"].reshape(-1, D).to(device, torch.float32).contiguous()
    S = coefs.shape[0]
    if labels is not None:
        return {"obs": _observed(labels, S, device, torch.int32)}
    out = torch.empty(S, N, dtype=torch.int32, device=device)
    check(lib().nmx_predict_logreg(ptr(X), N, D, ptr(coefs), S, seed, ptr(out), native.stream_ptr()),
          "nmx_predict_logreg")
    return {"obs": out}


def _predict_eight_schools(samples, seed, device, J, sigma, y=None):
    theta = samples["theta"].reshape(-1, J).to(device, torch.float32).contiguous()
    if y is not None:
        return {"obs": _observed(y, theta.shape[0], device)}
    sig = _as_device(sigma, device).reshape(J)
    out = torch.empty_like(theta)
    check(lib().nmx_predict_normal(ptr(theta), ptr(sig), J, theta.shape[0], seed, ptr(out), native.stream_ptr()),
          "nmx_predict_normal")
    return {"obs": out}


def _predict_bnn(samples, seed, device, X, Y, D_H, D_Y=1):
    Xd = _as_device(X, device)
    N, Dx = Xd.shape
    S = samples["prec_obs"].reshape(-1).shape[0]
    if Y is not None:
        return {"Y": _observed(Y, S, device)}
    flat = torch.cat([samples["prec_obs"].reshape(S, 1), samples["w1"].reshape(S, -1), samples["w2"].reshape(S, -1),
                      samples["w3"].reshape(S, -1)], dim=1).to(device, torch.float32).contiguous()
    out = torch.empty(S, N, D_Y, dtype=torch.float32, device=device)
    check(lib().nmx_predict_bnn(ptr(Xd), N, Dx, D_H, D_Y, ptr(flat), S, seed, ptr(out), native.stream_ptr()),
          "nmx_predict_bnn")
    return {"Y": out}


def _predict_sv(samples, seed, device, returns):
    if returns is None:
        raise ValueError("stochastic volatility: `returns` set the series length (examples/stochastic_volatility.py:"
                         "57-65); the observed site r keeps them")
    S = samples["s"].reshape(samples["s"].shape[0], -1).shape[0]
    return {"r": _observed(returns, S, device)}


def _predict_none(samples, seed, device, *args, **kwargs):
    return {}


# FusedModel -> (observed sites, sampler(samples, seed, device, *args, **kwargs))
_PREDICTORS = {
    "logistic_regression": (("obs",), _predict_logreg),
    "eight_schools": (("obs",), _predict_eight_schools),
    "bnn": (("Y",), _predict_bnn),
    "stochastic_volatility": (("r",), _predict_sv),
    "funnel": ((), _predict_none),
    "funnel_reparam": ((), _predict_none),
}


# models whose Predictive draws nothing on the device (no free observed site)
_HOST_ONLY = {"stochastic_volatility", "funnel", "funnel_reparam"}


class Predictive:
    """numpyro.infer.Predictive (numpyro/infer/util.py:888-1090) for the fused models."""

    def __init__(self, model, posterior_samples=None, *, guide=None, params=None, num_samples=None,
                 return_sites=None, infer_discrete=False, parallel=False, batch_ndims=None,
                 exclude_deterministic=True):
        if posterior_samples is None and num_samples is None:
            raise ValueError("Either posterior_samples or num_samples must be specified.")
        if posterior_samples is not None and guide is not None:
            raise ValueError("Only one of guide or posterior_samples can be provided, not both.")
        if guide is not None or params:
            raise NotImplementedError("Predictive with a guide / params (SVI) is out of scope here")
        if infer_discrete:
            raise NotImplementedError("infer_discrete is out of scope here")
        if posterior_samples is None:
            raise NotImplementedError("prior predictive (no posterior_samples) is out of scope here")
        if not isinstance(model, P.FusedModel) or model.__name__ not in _PREDICTORS:
            raise NotImplementedError(f"no predictive sampler for {model!r} "
                                      f"(available: {sorted(_PREDICTORS)})")
        batch_ndims = 1 if batch_ndims is None else batch_ndims
        batch_shape = None
        proto = None
        for name, v in posterior_samples.items():
            shp = tuple(v.shape[:batch_ndims])
            if batch_shape is not None and shp != batch_shape:
                raise ValueError(f"Batch shapes at site {name} and {proto} should be the same, "
                                 f"but got {shp} and {batch_shape}")
            if batch_shape is None:
                batch_shape, proto = shp, name
        if batch_shape is None:
            raise ValueError("No sample sites in posterior samples to infer `num_samples`.")
        batch_size = int(math.prod(batch_shape))
        if num_samples is not None and num_samples != batch_size:
            warnings.warn(f"Sample's batch dimension size {batch_size} is different from the provided "
                          f"{num_samples} num_samples argument. Defaulting to {batch_size}.", UserWarning)
        if return_sites is not None:
            assert isinstance(return_sites, (list, tuple, set))
        self.model = model
        self.posterior_samples = posterior_samples
        self.num_samples = batch_size
        self.return_sites = return_sites
        self.batch_ndims = batch_ndims
        self._batch_shape = batch_shape
        self.exclude_deterministic = exclude_deterministic
        self.parallel = parallel

    def __call__(self, rng_key, *args, **kwargs):
        observed, sampler = _PREDICTORS[self.model.__name__]
        nb = self.batch_ndims
        S = self.num_samples
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        if device is None:
            if self.model.__name__ not in _HOST_ONLY:
                raise RuntimeError("Predictive needs a GPU (the samplers are HIP kernels)")
            device = torch.device("cpu")  # nothing is drawn: observed data / deterministic sites
        flat = {k: torch.as_tensor(v).reshape(S, *v.shape[nb:]) for k, v in self.posterior_samples.items()}
        draws = sampler(flat, key_to_seed(rng_key), device, *args, **kwargs)
        # deterministic sites from the (constrained) latent values: recomputed from the samples
        # (exclude_deterministic=True, the default) or taken as given
        pot = self.model.potential(*args, **kwargs)
        latent = {n: flat[n] for n, _, _ in pot.sites if n in flat}
        dets = pot.deterministic(latent) if len(latent) == len(pot.sites) else {}
        if not self.exclude_deterministic:
            dets.update({k: v for k, v in flat.items() if k in dets})
        if self.return_sites is None:
            names = [n for n in observed if n not in self.posterior_samples] + list(dets)
        else:
            names = list(self.return_sites)
        out = {}
        for n in names:
            if n in draws and n not in self.posterior_samples:
                v = draws[n]
            elif n in dets:
                v = dets[n]
            elif n in flat:  # a substituted latent site, returned as given
                v = flat[n]
            else:
                continue
            out[n] = v.reshape(*self._batch_shape, *v.shape[1:])
        return out
