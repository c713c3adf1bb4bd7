"""Model front end: a model written against numpyro's API -- sample /
plate / deterministic with numpyro_amd.distributions and numpyro_amd.jnp -- is traced once per
data binding and mapped onto the fused potential kernel of its structure.

The reference turns a model into potential_fn by tracing its effect handlers
(numpyro/infer/util.py:632-800 initialize_model, :546-611 potential_fn_gen) and
differentiates it with JAX.  Here the trace records each site's distribution, parameters
(constants, or symbolic expressions of latent sites: numpyro_amd.jnp.Sym), plates and
observed data; a matcher per supported structure checks the priors' constants and the
likelihood's expression and returns the bound fused potential, with the model's own site
names.  Supported structures: the reference's examples on the hot path (covtype logistic
regression, eight schools, funnel and its LocScaleReparam(0) form, stochastic volatility,
the BNN) and the test targets (diagonal normal, multivariate normal).  Anything else raises
NotImplementedError naming the traced sites: there is no generic (autodiff) path.
"""
from __future__ import annotations

import numbers

import numpy as np

from . import distributions as dist
from . import potentials as P
from .jnp import Sym, shape_of
from .primitives import _TRACE


class Site:
    def __init__(self, name, fn, obs, shape, plates):
        self.name, self.fn, self.obs, self.shape, self.plates = name, fn, obs, tuple(shape), tuple(plates)

    def __repr__(self):
        kind = "obs" if self.obs is not None else "latent"
        return f"{self.name}: {kind} {type(_base(self.fn)).__name__}{list(self.shape)}"


class ModelTrace:
    def __init__(self, reparam_config=None):
        self.sites = {}
        self.plates = []
        self.deterministics = {}
        self.reparam = dict(reparam_config or {})

    def sample(self, name, fn, obs, sample_shape):
        if name in self.sites:
            raise ValueError(f"sample site {name!r} already exists")
        plate_shape = tuple(size for _, size, _ in self.plates)
        batch = np.broadcast_shapes(fn.batch_shape, plate_shape) if plate_shape else fn.batch_shape
        shape = tuple(sample_shape) + tuple(batch) + fn.event_shape
        self.sites[name] = Site(name, fn, obs, shape, [p[0] for p in self.plates])
        if obs is not None:
            return obs
        return Sym("latent", (name,), shape)

    def deterministic(self, name, value):
        self.deterministics[name] = value
        return value


def trace_model(model, args=(), kwargs=None, reparam_config=None):
    t = ModelTrace(reparam_config)
    _TRACE.append(t)
    try:
        model(*args, **(kwargs or {}))
    finally:
        _TRACE.pop()
    return t


# ----------------------------------------------------------------------------- helpers
def _base(fn):
    while isinstance(fn, (dist.Independent, dist.ExpandedDistribution)):
        fn = fn.base_dist
    return fn


def _host(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _const(x, value=None):
    """x is a constant (not symbolic); with value: every element equals it."""
    if isinstance(x, Sym):
        return False
    if value is None:
        return True
    a = _host(x)
    return a.size > 0 and bool(np.all(a == value))


def _latent(x, name=None):
    ok = isinstance(x, Sym) and x.op == "latent"
    return ok and (name is None or x.args[0] == name)


def _is(fn, cls):
    return isinstance(_base(fn), cls)


def _std_normal(site):
    b = _base(site.fn)
    return isinstance(b, dist.Normal) and _const(b.loc, 0.0) and _const(b.scale, 1.0)


def _split(trace):
    lat = [s for s in trace.sites.values() if s.obs is None]
    obs = [s for s in trace.sites.values() if s.obs is not None]
    return lat, obs


def _renamed(pot, names):
    """The fused potential with the model's site names (same layout and transforms);
    `names` maps the kernel's site names to the model's."""
    pot.sites = [(names.get(n, n), s, t) for n, s, t in pot.sites]
    inv = {v: k for k, v in names.items()}
    base_det = pot.deterministic

    def deterministic(sites):
        out = base_det({inv.get(k, k): v for k, v in sites.items()})
        return {names.get(k, k): v for k, v in out.items()}

    pot.deterministic = deterministic
    return pot


def _half(x):
    """x / 2 or x * 0.5 -> the symbolic x, else None."""
    if isinstance(x, Sym) and x.op == "div" and _const(x.args[1], 2.0):
        return x.args[0]
    if isinstance(x, Sym) and x.op == "mul":
        a, b = x.args
        if _const(b, 0.5):
            return a
        if _const(a, 0.5):
            return b
    return None


# ----------------------------------------------------------------------------- matchers
def _match_logistic(trace):
    """examples/covtype.py:66-71: coefs ~ Normal(0, 1)^D, obs ~ Bernoulli(logits=X @ coefs)."""
    lat, obs = _split(trace)
    if len(lat) != 1 or len(obs) != 1 or not _std_normal(lat[0]) or len(lat[0].shape) != 1:
        return None
    o = obs[0]
    if not _is(o.fn, dist.BernoulliLogits):
        return None
    lg = _base(o.fn).logits
    if not (isinstance(lg, Sym) and lg.op == "matmul" and _const(lg.args[0]) and _latent(lg.args[1], lat[0].name)):
        return None
    return _renamed(P.LogisticRegression(lg.args[0], o.obs), {"coefs": lat[0].name})


def _match_eight_schools(trace):
    """README.md:47-55: mu ~ N(0, 5), tau ~ HalfCauchy(5), theta ~ N(mu, tau) [J], y ~ N(theta, sigma)."""
    lat, obs = _split(trace)
    if len(lat) != 3 or len(obs) != 1:
        return None
    by = {type(_base(s.fn)).__name__: s for s in lat if s.shape == ()}
    mu, tau = by.get("Normal"), by.get("HalfCauchy")
    theta = [s for s in lat if s.shape != ()]
    if mu is None or tau is None or len(theta) != 1:
        return None
    theta = theta[0]
    bm, bt, bth = _base(mu.fn), _base(tau.fn), _base(theta.fn)
    if not (_const(bm.loc, 0.0) and _const(bm.scale, 5.0) and _const(bt.scale, 5.0)):
        return None
    if not (isinstance(bth, dist.Normal) and _latent(bth.loc, mu.name) and _latent(bth.scale, tau.name)):
        return None
    o = obs[0]
    bo = _base(o.fn)
    if not (isinstance(bo, dist.Normal) and _latent(bo.loc, theta.name) and _const(bo.scale)):
        return None
    J = theta.shape[0]
    return _renamed(P.EightSchools(J, _host(bo.scale), _host(o.obs)),
                    {"mu": mu.name, "tau": tau.name, "theta": theta.name})


def _match_funnel(trace):
    """examples/funnel.py:44-49: y ~ N(0, 3), x ~ N(0, exp(y / 2)) [dim - 1]; with
    reparam(config={"x": LocScaleReparam(0)}) the non-centred form."""
    lat, obs = _split(trace)
    if len(lat) != 2 or obs:
        return None
    y = [s for s in lat if s.shape == ()]
    x = [s for s in lat if s.shape != ()]
    if len(y) != 1 or len(x) != 1:
        return None
    y, x = y[0], x[0]
    by, bx = _base(y.fn), _base(x.fn)
    if not (isinstance(by, dist.Normal) and _const(by.loc, 0.0) and _const(by.scale, 3.0)):
        return None
    if not (isinstance(bx, dist.Normal) and _const(bx.loc, 0.0) and isinstance(bx.scale, Sym)
            and bx.scale.op == "exp" and _latent(_half(bx.scale.args[0]), y.name)):
        return None
    dim = x.shape[0] + 1
    cfg = trace.reparam.get(x.name)
    if cfg is None:
        return _renamed(P.Funnel(dim), {"x": x.name, "y": y.name})
    if isinstance(cfg, LocScaleReparam) and cfg.centered == 0:
        return _renamed(P.FunnelNonCentered(dim), {"x_decentered": x.name + "_decentered", "y": y.name,
                                                   "x": x.name})
    return None


def _match_sv(trace):
    """examples/stochastic_volatility.py:57-65: sigma ~ Exp(50), s ~ GRW(sigma, T), nu ~ Exp(0.1),
    r ~ StudentT(nu, 0, exp(s))."""
    lat, obs = _split(trace)
    if len(lat) != 3 or len(obs) != 1:
        return None
    grw = [s for s in lat if _is(s.fn, dist.GaussianRandomWalk)]
    exps = [s for s in lat if _is(s.fn, dist.Exponential)]
    if len(grw) != 1 or len(exps) != 2:
        return None
    s = grw[0]
    sigma = [e for e in exps if _latent(_base(s.fn).scale, e.name)]
    if len(sigma) != 1 or not _const(_base(sigma[0].fn).rate, 50.0):
        return None
    sigma = sigma[0]
    nu = [e for e in exps if e is not sigma][0]
    if not _const(_base(nu.fn).rate, 0.1):
        return None
    o = obs[0]
    bo = _base(o.fn)
    if not (isinstance(bo, dist.StudentT) and _latent(bo.df, nu.name) and _const(bo.loc, 0.0)
            and isinstance(bo.scale, Sym) and bo.scale.op == "exp" and _latent(bo.scale.args[0], s.name)):
        return None
    return _renamed(P.StochasticVolatility(_host(o.obs)), {"sigma": sigma.name, "s": s.name, "nu": nu.name})


def _match_bnn(trace):
    """examples/bnn.py:43-74: w1, w2, w3 ~ N(0, 1), z1 = tanh(X w1), z2 = tanh(z1 w2), z3 = z2 w3,
    prec_obs ~ Gamma(3, 1), Y ~ N(z3, 1 / sqrt(prec_obs))."""
    lat, obs = _split(trace)
    if len(lat) != 4 or len(obs) != 1:
        return None
    o = obs[0]
    bo = _base(o.fn)
    if not isinstance(bo, dist.Normal):
        return None
    z3, sig = bo.loc, bo.scale
    if not (isinstance(z3, Sym) and z3.op == "matmul"):
        return None
    z2, w3 = z3.args
    if not (isinstance(z2, Sym) and z2.op == "tanh" and _latent(w3)):
        return None
    m2 = z2.args[0]
    if not (isinstance(m2, Sym) and m2.op == "matmul" and _latent(m2.args[1])):
        return None
    z1, w2 = m2.args
    if not (isinstance(z1, Sym) and z1.op == "tanh"):
        return None
    m1 = z1.args[0]
    if not (isinstance(m1, Sym) and m1.op == "matmul" and _const(m1.args[0]) and _latent(m1.args[1])):
        return None
    X, w1 = m1.args
    if not (isinstance(sig, Sym) and sig.op == "div" and _const(sig.args[0], 1.0) and isinstance(sig.args[1], Sym)
            and sig.args[1].op == "sqrt" and _latent(sig.args[1].args[0])):
        return None
    prec = sig.args[1].args[0].args[0]
    names = {"w1": w1.args[0], "w2": w2.args[0], "w3": w3.args[0], "prec_obs": prec}
    sites = trace.sites
    if not all(_std_normal(sites[names[k]]) for k in ("w1", "w2", "w3")):
        return None
    bp = _base(sites[prec].fn)
    if not (isinstance(bp, dist.Gamma) and _const(bp.concentration, 3.0) and _const(bp.rate, 1.0)):
        return None
    Y = _host(o.obs)
    H = sites[names["w2"]].shape[0]
    D_Y = Y.shape[-1] if Y.ndim > 1 else 1
    return _renamed(P.BNN(_host(X), Y.reshape(Y.shape[0], -1), H, D_Y), names)


def _match_normal(trace):
    """x ~ Normal(mu, sd) (test/infer/test_mcmc.py:28-72 target) or MultivariateNormal."""
    lat, obs = _split(trace)
    if len(lat) != 1 or obs:
        return None
    s = lat[0]
    b = _base(s.fn)
    if isinstance(b, dist.Normal) and _const(b.loc) and _const(b.scale):
        n = int(np.prod(s.shape)) if s.shape else 1
        mu = np.broadcast_to(_host(b.loc), s.shape).reshape(n)
        sd = np.broadcast_to(_host(b.scale), s.shape).reshape(n)
        pot = P.DiagNormal(mu, sd, name=s.name)
        pot.sites = [(s.name, s.shape if s.shape else (), P.REAL)]
        return pot
    if isinstance(b, dist.MultivariateNormal) and _const(b.loc):
        return P.MultivariateNormal(_host(b.loc), b.covariance_matrix, b.precision_matrix, name=s.name)
    return None


MATCHERS = (_match_logistic, _match_eight_schools, _match_funnel, _match_sv, _match_bnn, _match_normal)


def potential_from_model(model, args=(), kwargs=None):
    """Trace `model(*args, **kwargs)` and return the fused potential of its structure."""
    cfg = getattr(model, "_nmx_reparam", None)
    fn = getattr(model, "_nmx_model", model)
    trace = trace_model(fn, args, kwargs, cfg)
    for m in MATCHERS:
        pot = m(trace)
        if pot is not None:
            return _with_traced_deterministics(pot, trace)
    raise NotImplementedError(
        "no fused kernel for this model structure (sites: " + ", ".join(map(repr, trace.sites.values())) +
        "); supported: the reference's covtype logistic regression, eight schools, funnel (+ LocScaleReparam), "
        "stochastic volatility and BNN examples, and diagonal / multivariate normal targets")


# ----------------------------------------------------------------------------- deterministic sites
_SYM_UNARY = {"tanh": "tanh", "exp": "exp", "sqrt": "sqrt", "log": "log", "neg": "neg"}
_SYM_BINARY = {"add": "add", "sub": "sub", "mul": "mul", "div": "div", "pow": "pow"}


def eval_sym(x, values):
    """Value of a traced expression over a batch of draws: `values` maps latent site names to
    tensors [*batch, *site shape] (constrained values, as the model sees them).  Constants
    broadcast against the trailing (event) dimensions; a product with a vector operand (event
    rank 1, known from the trace) treats it as a column / row."""
    import torch

    if not isinstance(x, Sym):
        ref = next(iter(values.values()))
        return torch.as_tensor(_host(x), dtype=torch.float32, device=ref.device)
    if x.op == "latent":
        return values[x.args[0]]
    if x.op in _SYM_UNARY:
        return getattr(torch, _SYM_UNARY[x.op])(eval_sym(x.args[0], values))
    if x.op in _SYM_BINARY:
        a, b = (eval_sym(v, values) for v in x.args)
        return getattr(torch, _SYM_BINARY[x.op])(a, b)
    if x.op == "matmul":
        a_s, b_s = x.args
        a, b = eval_sym(a_s, values), eval_sym(b_s, values)
        va, vb = len(shape_of(a_s)) == 1, len(shape_of(b_s)) == 1
        if vb:
            b = b.unsqueeze(-1)
        if va:
            a = a.unsqueeze(-2)
        out = torch.matmul(a, b)
        if vb:
            out = out.squeeze(-1)
        if va:
            out = out.squeeze(-2)
        return out
    raise NotImplementedError(f"deterministic expression with operation {x.op!r}")


def _check_sym(x, name):
    """Raise NotImplementedError at model-mapping time for an expression eval_sym cannot evaluate."""
    if not isinstance(x, Sym) or x.op == "latent":
        return
    if x.op not in _SYM_UNARY and x.op not in _SYM_BINARY and x.op != "matmul":
        raise NotImplementedError(f"deterministic site {name!r}: operation {x.op!r} is not supported "
                                  f"(supported: {sorted(_SYM_UNARY) + sorted(_SYM_BINARY) + ['matmul']})")
    for a in x.args:
        _check_sym(a, name)


def _with_traced_deterministics(pot, trace):
    """The model's own numpyro.deterministic sites (primitives.py:293-314) come back with the
    samples (MCMC.get_samples, postprocess_fn), evaluated from the traced expressions after
    the fused potential's deterministic sites."""
    dets = dict(trace.deterministics)
    if not dets:
        return pot
    for name, expr in dets.items():  # unsupported operations fail here, not after sampling
        _check_sym(expr, name)
    base = pot.deterministic
    site_shape = {n: tuple(s) for n, s, _ in pot.sites}

    def deterministic(sites):
        import torch

        out = base(sites)
        vals = dict(sites)
        vals.update(out)
        n0 = next(n for n in sites if n in site_shape)
        v0 = sites[n0]
        batch = tuple(v0.shape[:v0.dim() - len(site_shape[n0])])
        for name, expr in dets.items():
            v = eval_sym(expr, vals)
            # a constant (or batch-free) expression still has one value per draw
            ev = tuple(shape_of(expr)) if isinstance(expr, Sym) else tuple(torch.as_tensor(v).shape)
            if tuple(v.shape) != batch + ev:
                v = v.expand(*batch, *ev).clone()
            out[name] = v
            vals[name] = v
        return out

    pot.deterministic = deterministic
    return pot


# ----------------------------------------------------------------------------- reparam
class LocScaleReparam:
    """numpyro.infer.reparam.LocScaleReparam (infer/reparam.py:93-170) marker for the front end."""

    def __init__(self, centered=None, shape_params=None):
        self.centered = centered


def reparam(fn=None, config=None):
    """numpyro.handlers.reparam (handlers.py:589-653) for front-end models."""
    if fn is None:
        return lambda f: reparam(f, config)

    def wrapped(*args, **kwargs):
        return fn(*args, **kwargs)

    wrapped._nmx_model = getattr(fn, "_nmx_model", fn)
    wrapped._nmx_reparam = dict(getattr(fn, "_nmx_reparam", None) or {}, **(config or {}))
    wrapped.__name__ = getattr(fn, "__name__", "model")
    return wrapped


def is_numeric(x):
    return isinstance(x, numbers.Number) or _const(x)
