"""numpyro's modelling primitives (numpyro/primitives.py: sample :154-239, plate :497-601,
deterministic :293-314) for models run through the model front end.

Outside a trace a model cannot be evaluated here (there is no JAX): ``sample`` of a latent
site raises.  Inside ``frontend.trace_model`` every latent site becomes a symbolic value
(numpyro_amd.jnp.Sym), observed sites and plates are recorded, and the front end maps the
recorded structure onto a fused potential kernel."""
from __future__ import annotations

import contextlib

_TRACE = []  # stack of active tracers (frontend.ModelTrace)


def _tracer():
    if not _TRACE:
        raise RuntimeError("numpyro_amd models run only under NUTS/HMC (the model front end traces them; "
                           "there is no eager evaluation without JAX)")
    return _TRACE[-1]


def sample(name, fn, obs=None, rng_key=None, sample_shape=(), infer=None, obs_mask=None):
    """numpyro.sample (primitives.py:154-239).  `obs_mask` (a masked likelihood with imputed
    latent entries, :177-191) and `infer` options (enumeration, auxiliary sites) change the
    potential; the fused kernels implement the full-data likelihood only, so both are refused
    here instead of being dropped."""
    if obs_mask is not None:
        raise NotImplementedError(f"sample site {name!r}: obs_mask (masked likelihood) is not supported by the "
                                  "fused potentials")
    if infer:
        raise NotImplementedError(f"sample site {name!r}: infer={dict(infer)!r} is not supported by the fused "
                                  "potentials")
    return _tracer().sample(name, fn, obs, tuple(sample_shape))


def deterministic(name, value):
    return _tracer().deterministic(name, value)


def param(name, init_value=None, **kwargs):
    raise NotImplementedError("numpyro.param belongs to SVI, outside this engine")


@contextlib.contextmanager
def plate(name, size, subsample_size=None, dim=None):
    if subsample_size is not None and subsample_size != size:
        raise NotImplementedError("subsampling plates are not supported (full-data potentials only)")
    t = _tracer()
    t.plates.append((name, int(size), dim))
    try:
        yield None
    finally:
        t.plates.pop()
