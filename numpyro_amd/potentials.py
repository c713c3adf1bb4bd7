"""Fused potentials: the model side of the hot path.

The reference turns a model into ``potential_fn(z)`` by tracing its effect handlers
(numpyro/infer/util.py:546-611) and differentiates it with ``jax.value_and_grad``
(numpyro/infer/hmc_util.py:242-252).  Here each supported model is a hand-written HIP
kernel computing U and dU/dz for all chains at once; this module binds a model's data
to its kernel and describes its sample sites (names, shapes, support transforms) in the
order of ``ravel_pytree`` over the sorted site dict, so samples come back keyed by site
exactly like ``MCMC.get_samples()``.

``FusedModel`` objects play the role of the reference's model functions:
``NUTS(logistic_regression)`` then ``mcmc.run(key, features, labels)`` binds the data.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import native
from .native import check, lib, ptr

REAL, POSITIVE = 0, 1  # transform codes: identity, ExpTransform (transforms.py:537-577)


class Potential:
    """Base class.  Subclasses set ``sites`` = [(name, shape, transform)] and ``dim``."""

    sites: list = []
    dim: int = 0

    def bind(self, num_chains: int, ldc: int, device) -> None:
        before = dict(self.__dict__)
        self.num_chains, self.ldc, self.device = num_chains, ldc, torch.device(device)
        self._codes = None
        self._bind(num_chains, ldc, self.device)
        # what binding made or replaced (device copies of the data, workspaces, whitening) is not
        # pickled: attributes binding created are dropped, attributes it replaced (e.g. a
        # `packed = None` set in __init__) go back to their unbound value, so an unpickled
        # potential is unbound and binds again on its engine
        made = set(self.__dict__) - set(before)
        replaced = {k: v for k, v in before.items() if k in self.__dict__ and self.__dict__[k] is not v
                    and k not in ("num_chains", "ldc", "device", "_codes")}
        self._bound_keys = getattr(self, "_bound_keys", set()) | made
        unbound = getattr(self, "_unbound_values", {})
        for k, v in replaced.items():
            unbound.setdefault(k, v)
        self._unbound_values = unbound

    def __getstate__(self):
        drop = getattr(self, "_bound_keys", set()) | {"_bound_keys", "_unbound_values"}
        unbound = getattr(self, "_unbound_values", {})
        return {k: unbound.get(k, v) for k, v in self.__dict__.items() if k not in drop}

    def _bind(self, num_chains, ldc, device):
        pass

    def evaluate(self, eval_batch: native.EvalBatch, stream: int) -> None:
        raise NotImplementedError

    def transform_codes(self):
        if self._codes is None:
            codes = []
            for _, shape, tr in self.sites:
                codes += [tr] * int(np.prod(shape, dtype=np.int64))
            assert len(codes) == self.dim
            self._codes = torch.tensor(codes, dtype=torch.int8, device=self.device)
        return self._codes

    def deterministic(self, sites):
        """Deterministic sites computed from the sampled ones ({} unless the model has any)."""
        return {}

    def unflatten(self, flat):
        """[..., D] -> {site: [..., *shape]} (ravel_pytree order)."""
        out, o = {}, 0
        for name, shape, _ in self.sites:
            n = int(np.prod(shape, dtype=np.int64))
            out[name] = flat[..., o:o + n].reshape(*flat.shape[:-1], *shape)
            o += n
        return out

    def flatten(self, params: dict):
        """{site: [C, *shape]} unconstrained -> [C, D]."""
        parts = []
        for name, shape, _ in self.sites:
            v = torch.as_tensor(params[name], dtype=torch.float32)
            parts.append(v.reshape(v.shape[0], -1))
        return torch.cat(parts, dim=1)


def _dev(x, device, dtype=torch.float32):
    return torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x, dtype=dtype).to(device).contiguous()


class DiagNormal(Potential):
    """U = 0.5 sum((z - mu)^2 / sd^2): test target of test/infer/test_mcmc.py:28-72."""

    def __init__(self, mu, sd, name="x"):
        self.mu_h = np.asarray(mu, np.float32).reshape(-1)
        self.sd_h = np.broadcast_to(np.asarray(sd, np.float32), self.mu_h.shape).copy()
        self.dim = self.mu_h.size
        self.sites = [(name, (self.dim,), REAL)]

    def _bind(self, C, ldc, device):
        self.mu = _dev(self.mu_h, device)
        self.prec = _dev(1.0 / self.sd_h.astype(np.float64) ** 2, device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_diag_normal(ptr(self.mu), ptr(self.prec), self.dim, ctypes.byref(ev), stream),
              "nmx_pe_diag_normal")

    def small_model(self):
        """Inline potential of the persistent schedule (nmx_nuts_run_small)."""
        return native.SMALL_DIAG_NORMAL, self.mu, self.prec, self.dim


class EightSchools(Potential):
    """README.md:47-55: mu ~ N(0,5), tau ~ HalfCauchy(5), theta ~ N(mu, tau), y ~ N(theta, sigma)."""

    def __init__(self, J, sigma, y):
        self.J = int(J)
        self.sigma_h = np.asarray(sigma, np.float32)
        self.y_h = np.asarray(y, np.float32)
        self.dim = 2 + self.J
        self.sites = [("mu", (), REAL), ("tau", (), POSITIVE), ("theta", (self.J,), REAL)]

    def _bind(self, C, ldc, device):
        self.y = _dev(self.y_h, device)
        self.sigma = _dev(self.sigma_h, device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_eight_schools(ptr(self.y), ptr(self.sigma), self.J, ctypes.byref(ev), stream),
              "nmx_pe_eight_schools")

    def small_model(self):
        """Inline potential of the persistent schedule (nmx_nuts_run_small)."""
        return native.SMALL_EIGHT_SCHOOLS, self.y, self.sigma, self.J


class LogisticRegression(Potential):
    """examples/covtype.py:66-71 (coefs ~ N(0, 1)^D, obs ~ Bernoulli(logits=X @ coefs))."""

    def __init__(self, data, labels):
        self.X_in, self.y_in = data, labels
        shape = tuple(data.shape)
        self.N, self.dim = int(shape[0]), int(shape[1])
        if self.dim > 64:
            raise ValueError("the fused logistic-regression kernel supports up to 64 features")
        self.sites = [("coefs", (self.dim,), REAL)]
        self.packed = None

    # workspaces: one per chain group evaluated concurrently (Engine chain groups, one stream each)
    slots = 4

    def _bind(self, C, ldc, device):
        if self.packed is None or self.packed.device != device:
            X = _dev(self.X_in, device)
            y = _dev(self.y_in, device)
            nb = lib().nmx_logreg_packed_bytes(self.N, self.dim)
            self.packed = torch.empty(nb // 4, dtype=torch.float32, device=device)
            with torch.cuda.device(device):
                check(lib().nmx_logreg_pack(ptr(X), ptr(y), self.N, self.dim, ptr(self.packed),
                                            native.stream_ptr()), "nmx_logreg_pack")
            del X, y
        wb = lib().nmx_logreg_workspace_bytes(self.N, self.dim, C)
        self.workspace = torch.empty(wb, dtype=torch.uint8, device=device)
        self._more_ws = []  # slots 1.. (allocated on first use)

    def evaluate(self, ev, stream, slot=0):
        ws = self.workspace
        if slot:
            while len(self._more_ws) < slot:
                self._more_ws.append(torch.empty_like(self.workspace))
            ws = self._more_ws[slot - 1]
        check(lib().nmx_logreg_pe_grad(ptr(self.packed), self.N, self.dim, ctypes.byref(ev),
                                       ptr(ws), stream), "nmx_logreg_pe_grad")

    def flops_per_eval(self, num_chains):
        """Algorithmic FLOPs of one evaluation (two GEMMs): 4 N D C."""
        return 4.0 * self.N * self.dim * num_chains


class StochasticVolatility(Potential):
    """examples/stochastic_volatility.py:57-65 (sigma ~ Exp(50), s ~ GRW(sigma), nu ~ Exp(0.1),
    r ~ StudentT(nu, 0, exp(s)))."""

    def __init__(self, returns):
        self.r_in = returns
        self.T = int(np.asarray(returns.cpu() if torch.is_tensor(returns) else returns).shape[0])
        self.dim = self.T + 2
        self.sites = [("nu", (), POSITIVE), ("s", (self.T,), REAL), ("sigma", (), POSITIVE)]

    def _bind(self, C, ldc, device):
        self.r = _dev(self.r_in, device)
        self.workspace = torch.empty(lib().nmx_pe_wide_workspace_bytes(self.dim, C), dtype=torch.uint8,
                                     device=device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_stochastic_volatility(ptr(self.r), self.T, ctypes.byref(ev), ptr(self.workspace),
                                                 stream), "nmx_pe_stochastic_volatility")

    def bytes_per_eval(self):
        """Algorithmic HBM bytes per chain evaluation: read z, write grad (f32)."""
        return 2 * 4 * self.dim

    def wide_model(self):
        """Model of the wide step fused with this potential (nmx_nuts_step_wide_model)."""
        return native.WIDE_SV, self.r, self.T


class Funnel(Potential):
    """examples/funnel.py:44-46, centred: y ~ N(0, 3), x ~ N(0, exp(y/2))^(dim-1)."""

    def __init__(self, dim=10):
        self.dim = int(dim)
        self.sites = [("x", (self.dim - 1,), REAL), ("y", (), REAL)]

    def _bind(self, C, ldc, device):
        self.workspace = torch.empty(lib().nmx_pe_wide_workspace_bytes(self.dim, C), dtype=torch.uint8,
                                     device=device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_funnel(self.dim, ctypes.byref(ev), ptr(self.workspace), stream), "nmx_pe_funnel")

    def wide_model(self):
        return native.WIDE_FUNNEL, None, self.dim

    def bytes_per_eval(self):
        return 2 * 4 * self.dim


class FunnelNonCentered(Potential):
    """examples/funnel.py:49, ``reparam(model, config={"x": LocScaleReparam(0)})``: the
    decentered site x_decentered ~ N(0, 1)^(dim-1) replaces x (numpyro/infer/reparam.py:
    104-145 with centered = 0), and x = 0 + exp(y/2) * x_decentered is a deterministic site."""

    def __init__(self, dim=10):
        self.dim = int(dim)
        self.sites = [("x_decentered", (self.dim - 1,), REAL), ("y", (), REAL)]

    def _bind(self, C, ldc, device):
        self.workspace = torch.empty(lib().nmx_pe_wide_workspace_bytes(self.dim, C), dtype=torch.uint8,
                                     device=device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_funnel_noncentered(self.dim, ctypes.byref(ev), ptr(self.workspace), stream),
              "nmx_pe_funnel_noncentered")

    def wide_model(self):
        return native.WIDE_FUNNEL_NC, None, self.dim

    def deterministic(self, sites):
        # reparam.py:140-142: value = loc + scale ** (1 - centered) * (decentered - centered * loc)
        return {"x": torch.exp(sites["y"] / 2)[..., None] * sites["x_decentered"]}

    def bytes_per_eval(self):
        return 2 * 4 * self.dim


class BNN(Potential):
    """examples/bnn.py:43-74: w1 [Dx,H], w2 [H,H], w3 [H,1] ~ N(0,1), prec_obs ~ Gamma(3,1),
    Y ~ N(tanh(tanh(X w1) w2) w3, 1/sqrt(prec_obs)); sites in ravel_pytree (sorted) order."""

    def __init__(self, X, Y, D_H, D_Y=1):
        if D_Y != 1:
            raise NotImplementedError("the fused BNN kernel supports D_Y = 1 (examples/bnn.py)")
        self.X_in, self.Y_in = X, Y
        shape = tuple(X.shape)
        self.N, self.Dx = int(shape[0]), int(shape[1])
        self.H = int(D_H)
        self.dim = 1 + self.Dx * self.H + self.H * self.H + self.H
        self.sites = [("prec_obs", (), POSITIVE), ("w1", (self.Dx, self.H), REAL), ("w2", (self.H, self.H), REAL),
                      ("w3", (self.H, 1), REAL)]

    def _bind(self, C, ldc, device):
        self.X = _dev(self.X_in, device)
        self.Y = _dev(self.Y_in, device).reshape(-1)
        self.workspace = torch.empty(lib().nmx_pe_bnn_workspace_bytes(self.Dx, self.H, C), dtype=torch.uint8,
                                     device=device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_bnn(ptr(self.X), ptr(self.Y), self.N, self.Dx, self.H, ctypes.byref(ev),
                               ptr(self.workspace), stream), "nmx_pe_bnn")

    def evaluate_rows(self, ev, z_rows, g_rows, stream):
        """The same on operands in rows (position p: z_rows[p], g_rows[p]; raw pointers):
        nmx_pe_bnn_rows, no transposes (WhitenedPotential on a chain-row arena)."""
        check(lib().nmx_pe_bnn_rows(ptr(self.X), ptr(self.Y), self.N, self.Dx, self.H, ctypes.byref(ev), z_rows,
                                    g_rows, stream), "nmx_pe_bnn_rows")

    def flops_per_eval(self, num_chains):
        """Forward + adjoint: ~6 N H^2 + 6 N Dx H FLOPs per chain."""
        return (6.0 * self.N * self.H * self.H + 6.0 * self.N * self.Dx * self.H) * num_chains


class MultivariateNormal(Potential):
    """U = 0.5 (z - mu)^T P (z - mu): the MultivariateNormal targets of
    test/infer/test_mcmc.py:73-100 (`test_correlated_mvn`) and :313-343 (`test_dense_mass`).
    grad = P z - P mu is one chain-batched MFMA product (nmx_gemm_chains)."""

    def __init__(self, loc=None, covariance_matrix=None, precision_matrix=None, name="x"):
        if (covariance_matrix is None) == (precision_matrix is None):
            raise ValueError("give exactly one of covariance_matrix / precision_matrix")
        if precision_matrix is None:
            prec = np.linalg.inv(np.asarray(covariance_matrix, np.float64))
        else:
            prec = np.asarray(precision_matrix, np.float64)
        self.prec_h = 0.5 * (prec + prec.T)
        self.dim = self.prec_h.shape[0]
        self.mu_h = (np.zeros(self.dim) if loc is None else np.asarray(loc, np.float64)).reshape(-1)
        self.sites = [(name, (self.dim,), REAL)]

    def _bind(self, C, ldc, device):
        lda = lib().nmx_dense_padded_dim(self.dim)
        pt = np.zeros((lda, lda), np.float32)
        pt[:self.dim, :self.dim] = self.prec_h.T
        self.lda = lda
        self.prec_t = _dev(pt, device)
        self.mu = _dev(self.mu_h, device)
        self.neg_prec_mu = _dev(-(self.prec_h @ self.mu_h), device)

    def evaluate(self, ev, stream):
        check(lib().nmx_pe_mvn(ptr(self.prec_t), self.lda, ptr(self.mu), ptr(self.neg_prec_mu), self.dim,
                               ctypes.byref(ev), stream), "nmx_pe_mvn")


# ------------------------------------------------------------------------------------------
# Model functions (the reference's examples) -> fused potentials.
# ------------------------------------------------------------------------------------------
class FusedModel:
    """A model callable whose potential is a fused kernel.  ``builder(*args, **kwargs)``
    returns a bound-data Potential (the analogue of initialize_model's potential_fn_gen)."""

    def __init__(self, name, builder, doc=""):
        self.__name__ = name
        self.builder = builder
        self.__doc__ = doc

    def potential(self, *args, **kwargs) -> Potential:
        return self.builder(*args, **kwargs)

    def __call__(self, *args, **kwargs):
        raise TypeError(f"{self.__name__} is a fused model: pass it to NUTS/HMC, do not call it")

    def __repr__(self):
        return f"FusedModel({self.__name__})"

    def __reduce__(self):
        # pickled by reference, like a model function (module-level name in this module)
        return (_fused_model, (self.__name__,))


def _fused_model(name):
    return globals()[name]


logistic_regression = FusedModel(
    "logistic_regression", lambda data, labels, subsample_size=None: LogisticRegression(data, labels),
    "examples/covtype.py:66-71 model(data, labels)")

eight_schools = FusedModel(
    "eight_schools", lambda J, sigma, y=None: EightSchools(J, sigma, y),
    "README.md:47-55 eight_schools(J, sigma, y)")

diag_normal = FusedModel("diag_normal", lambda mu, sd: DiagNormal(mu, sd))

stochastic_volatility = FusedModel(
    "stochastic_volatility", lambda returns: StochasticVolatility(returns),
    "examples/stochastic_volatility.py:57-65 model(returns)")

funnel = FusedModel("funnel", lambda dim=10: Funnel(dim), "examples/funnel.py:44-46 model(dim)")

funnel_reparam = FusedModel(
    "funnel_reparam", lambda dim=10: FunnelNonCentered(dim),
    'examples/funnel.py:49 reparam_model = reparam(model, config={"x": LocScaleReparam(0)})')

bnn = FusedModel("bnn", lambda X, Y, D_H, D_Y=1: BNN(X, Y, D_H, D_Y), "examples/bnn.py:43-74 model(X, Y, D_H)")

multivariate_normal = FusedModel(
    "multivariate_normal",
    lambda loc=None, covariance_matrix=None, precision_matrix=None: MultivariateNormal(
        loc, covariance_matrix, precision_matrix),
    "x ~ MultivariateNormal(loc, covariance_matrix | precision_matrix)")

LOG_2PI = math.log(2 * math.pi)


# ------------------------------------------------------------------ generic (torch) potential
class _DevicePtr:
    """A raw device buffer as a torch tensor (the __cuda_array_interface__ protocol, which torch
    imports without a copy): the engine hands potentials raw pointers (nmx_eval_batch)."""

    def __init__(self, p, shape, typestr, strides=None):
        self.__cuda_array_interface__ = {"data": (int(p), False), "shape": tuple(shape), "typestr": typestr,
                                         "strides": strides, "version": 2}


def _wrap(p, shape, dtype, device):
    typestr = {torch.float32: "<f4", torch.int32: "<i4"}[dtype]
    return torch.as_tensor(_DevicePtr(p, shape, typestr), device=device)


class TorchPotential(Potential):
    """A user ``potential_fn`` (numpyro/infer/hmc.py:127-130): ``U = fn(z)`` over ONE chain's
    unconstrained values -- a dict {site: tensor} like ``init_params`` (ravel_pytree order: sorted
    names) or a single tensor -- written with torch operations.  ``U`` and ``dU/dz`` of the
    evaluated chains come from ``torch.func.vmap(torch.func.grad_and_value(fn))``, the analogue of
    the reference's vmapped ``jax.value_and_grad(potential_fn)`` (hmc_util.py:242-252,
    hmc.py:797).  This is the generic path: torch kernels on the compacted list of chains that
    need a leaf, with no fused HIP potential -- a model with a registered fused kernel (the
    ``numpyro_amd.potentials`` FusedModels, or a traced model the front end maps onto one) is the
    fast path.  No host synchronisation: the listed chains are gathered and their results
    scattered back on the device, positions past the list's count leaving the arena untouched.
    A function that ``vmap`` cannot trace (data-dependent Python control flow) is evaluated one
    chain at a time instead (correct, slow)."""

    def __init__(self, fn, example):
        self.fn = fn
        if isinstance(example, dict):
            self.array_site = False
            names = sorted(example)
            self.sites = [(k, tuple(torch.as_tensor(example[k]).shape), REAL) for k in names]
        else:
            self.array_site = True
            self.sites = [("z", tuple(torch.as_tensor(example).shape), REAL)]
        self.dim = int(sum(int(np.prod(s, dtype=np.int64)) for _, s, _ in self.sites))
        if self.dim <= 0:
            raise ValueError("potential_fn: init_params hold no coordinates")
        self._vmap_ok = None

    def structure(self, flat):
        """[..., D] -> fn's argument structure (dict of sites, or the single tensor)."""
        if self.array_site:
            return flat.reshape(*flat.shape[:-1], *self.sites[0][1])
        return self.unflatten(flat)

    def _value_and_grad(self, zc):
        """(U [n], dU/dz [n, D]) of the rows of zc [n, D]."""
        def u(zf):
            return self.fn(self.structure(zf))

        if self._vmap_ok is not False:
            try:
                g, v = torch.func.vmap(torch.func.grad_and_value(u))(zc)
                self._vmap_ok = True
                return v.to(torch.float32), g.to(torch.float32)
            except Exception:  # noqa: BLE001  (a function vmap cannot trace: evaluated per chain)
                if self._vmap_ok:
                    raise
                self._vmap_ok = False
        vals, grads = [], []
        for row in zc:
            x = row.detach().clone().requires_grad_(True)
            val = torch.as_tensor(u(x), dtype=torch.float32)
            (gr,) = torch.autograd.grad(val, x)
            vals.append(val.detach())
            grads.append(gr)
        return torch.stack(vals), torch.stack(grads)

    def evaluate(self, ev, stream):
        dev, D, ldc = self.device, self.dim, int(ev.ldc)
        st = torch.cuda.ExternalStream(stream, device=dev) if stream else torch.cuda.default_stream(dev)
        with torch.cuda.stream(st), torch.no_grad():
            Z = _wrap(ev.z, (D, ldc), torch.float32, dev)
            G = _wrap(ev.grad, (D, ldc), torch.float32, dev)
            PE = _wrap(ev.pe, (ldc,), torch.float32, dev)
            n = min(int(ev.num_chains), ldc)
            pos = torch.arange(n, device=dev)
            if ev.active_idx:
                chains = _wrap(ev.active_idx, (ldc,), torch.int32, dev)[:n].long().clamp(0, ldc - 1)
                valid = pos < _wrap(ev.active_count, (1,), torch.int32, dev).long()
            else:
                chains = pos
                valid = (_wrap(ev.phase, (ldc,), torch.int32, dev)[:n] >= native.PH_LEAF) if ev.phase \
                    else torch.ones(n, dtype=torch.bool, device=dev)
            zc = Z.t()[chains]  # [n, D]
        with torch.cuda.stream(st):
            u, g = self._value_and_grad(zc)
        with torch.cuda.stream(st), torch.no_grad():
            # positions past the count (or not selected) write the first valid position's values to
            # its own chain -- identical duplicates -- or, with none valid, chain 0's old values
            first = torch.argmax(valid.to(torch.int32))
            anyv = valid.any()
            tgt = torch.where(valid, chains, chains[first])
            old_g, old_u = G.t()[chains[first]], PE[chains[first]]
            fill_g = torch.where(anyv, g[first], old_g)
            fill_u = torch.where(anyv, u[first], old_u)
            G.t()[tgt] = torch.where(valid[:, None], g, fill_g[None, :])
            PE[tgt] = torch.where(valid, u, fill_u)
