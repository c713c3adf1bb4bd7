"""``MCMC`` driver with numpyro's API (numpyro/infer/mcmc.py:224-800).

``run`` / ``warmup`` / ``get_samples`` / ``get_extra_fields`` / ``print_summary`` /
``post_warmup_state`` / ``last_state`` keep their reference meaning.  All chains of a
process live on one GPU and run as one vectorized batch on the device state machine; a
chain's trajectory is a function of (key, global chain id) only, so ``chain_method``
"parallel", "sequential" and "vectorized" give the same per-chain results (the reference
guarantees the same up to its stream, test/infer/test_mcmc.py:553-592).  Under
``torch.distributed`` each rank owns a contiguous shard of the chains
(``numpyro_amd.shard``): no collective while sampling; ``print_summary`` and
``gather_samples`` reduce / gather across ranks at the end (RCCL on the GPU box).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import diagnostics, native, shard
from ..random import key_to_seed
from .hmc import restore_state, snapshot_state

_FIELD_ALIASES = {"adapt_state.step_size": "step_size", "i": "i"}
# HMCState fields (hmc.py:31-48) the device does not collect per transition but that follow from
# what it does: the gradient at each collected draw (the model's potential evaluated again at the
# unconstrained draws after the run -- the same per-chain kernel, so the sampler's own gradient
# for real-valued sites), the configured trajectory length, the momentum carried between
# transitions (None: a fresh momentum is drawn every transition, as in the reference unless a
# state carries r), and the mass matrices of sampling draws (constant after warmup)
_DERIVED_FIELDS = ("z_grad", "trajectory_length", "r", "adapt_state.inverse_mass_matrix",
                   "adapt_state.mass_matrix_sqrt", "adapt_state.mass_matrix_sqrt_inv")


from ..shard import shard_chains  # noqa: E402  (re-exported: contiguous chain shard per rank)


_VMAP_CHUNK = 1 << 16  # draws per vmapped postprocess_fn call (bounds the batched intermediates)


def _vmap_unsupported(e):
    """An error torch.func.vmap raises for a function it cannot batch (data-dependent control
    flow, .item() / Python numbers, an op without a batching rule), not a bug of the function."""
    if not isinstance(e, (RuntimeError, TypeError, NotImplementedError, ValueError)):
        return False
    msg = str(e).lower()
    return any(k in msg for k in ("vmap", "batched", "batching", "functorch", "data-dependent"))


def _postprocess_per_draw(fn, sites):
    """postprocess_fn applied to each draw's site dict ({site: [*shape]}), as the reference's
    fori_collect does per iteration (util.py:277-407 _collect_and_postprocess, vmapped over
    chains when vectorized, mcmc.py:422-442): vectorized over the C x S draws by torch.func.vmap
    in chunks of _VMAP_CHUNK draws, or -- only when vmap cannot batch fn (e.g. it converts to
    Python numbers) -- one call per draw, with a warning (8192 chains x 1000 draws is 8M calls).
    Any other error of fn propagates.  sites: {site: [C, S, *shape]} -> {name: [C, S, *out_shape]}."""
    import warnings

    v0 = next(iter(sites.values()))
    C, S = int(v0.shape[0]), int(v0.shape[1])
    n = C * S
    flat = {k: v.reshape(n, *v.shape[2:]) for k, v in sites.items()}
    try:
        parts = [dict(torch.func.vmap(fn)({k: v[i:i + _VMAP_CHUNK] for k, v in flat.items()}))
                 for i in range(0, n, _VMAP_CHUNK)]
        res = {k: torch.cat([torch.as_tensor(p[k]) for p in parts]) for k in parts[0]} if parts else {}
    except Exception as e:  # noqa: BLE001  (re-raised unless vmap could not batch fn)
        if not _vmap_unsupported(e):
            raise
        warnings.warn(f"postprocess_fn cannot be vmapped ({type(e).__name__}: {str(e)[:120]}); applying it "
                      f"once per draw ({n} calls)", RuntimeWarning, stacklevel=3)
        rows = [dict(fn({k: v[i] for k, v in flat.items()})) for i in range(n)]
        res = {k: torch.stack([torch.as_tensor(r[k], device=v0.device) for r in rows]) for k in rows[0]} if rows else {}
    return {k: torch.as_tensor(v).reshape(C, S, *torch.as_tensor(v).shape[1:]) for k, v in res.items()}


class MCMC:
    def __init__(self, sampler, *, num_warmup, num_samples, num_chains=1, thinning=1,
                 postprocess_fn=None, chain_method="parallel", progress_bar=True,
                 jit_model_args=False, device=None, sync_chains=False, chain_offset=None,
                 poll_every=16, devices=None):
        self.sampler = sampler
        self._sample_field = sampler.sample_field
        self._default_fields = sampler.default_fields
        self.num_warmup = int(num_warmup)
        self.num_samples = int(num_samples)
        self.num_chains = int(num_chains)
        if not isinstance(thinning, int) or thinning < 1:
            raise ValueError("thinning must be a positive integer")
        self.thinning = thinning
        # postprocess_fn (mcmc.py:331,345,422-442): maps a dict of unconstrained site values to
        # the collected values; None = the sampler's (constrain + deterministic sites, done on
        # the device and by the potential).  Applied per draw on site-shaped values, as the
        # reference's fori_collect does (_postprocess_per_draw)
        self.postprocess_fn = postprocess_fn
        if not callable(chain_method) and chain_method not in ("parallel", "vectorized", "sequential"):
            raise ValueError('Only supporting the following methods to draw chains: "sequential", '
                             '"parallel", or "vectorized"')
        self.chain_method = chain_method
        self.progress_bar = progress_bar
        self.device = device
        # chain_method="parallel" (the reference's default: pmap over local devices,
        # mcmc.py:700-715) or a callable (pmap-of-vectorized, mcmc.py:296-320) shards the chains
        # of this process over `devices` -- a list, or "all" for every visible GPU -- one engine
        # and one host thread per device.  Opt-in: without `devices` a process runs one engine
        # on its current GPU (one process per GPU under torch.distributed is the scaling path)
        if devices == "all":
            n = torch.cuda.device_count() if torch.cuda.is_available() else 0
            devices = [torch.device("cuda", i) for i in range(n)]
        self.devices = None if devices is None else [torch.device(d) for d in devices]
        self.sync_chains = sync_chains
        self.poll_every = int(poll_every)
        # chain shard of this process
        if chain_offset is not None:
            self.chain_lo, self.chain_hi = int(chain_offset), int(chain_offset) + self.num_chains
            self.local_chains = self.num_chains
        elif torch.distributed.is_available() and torch.distributed.is_initialized():
            r, w = torch.distributed.get_rank(), torch.distributed.get_world_size()
            self.chain_lo, self.chain_hi = shard_chains(self.num_chains, r, w)
            self.local_chains = self.chain_hi - self.chain_lo
        else:
            self.chain_lo, self.chain_hi, self.local_chains = 0, self.num_chains, self.num_chains
        self._engine = None
        self._engine_key = None
        self._engines = None  # multi-device run: one engine per device (chain shards)
        self._warmup_state = None
        self._last_state = None
        self._samples = None
        self._fields = None
        self._collected = ()
        self._args, self._kwargs = (), {}
        self._host_potential = None  # (args key, potential) for results of an unpickled MCMC
        self.last_run_stats = {}

    # ------------------------------------------------------------------ engine
    def _get_engine(self, args, kwargs):
        key = (id(self.sampler), tuple(id(a) for a in args), tuple(sorted((k, id(v)) for k, v in kwargs.items())),
               id(getattr(self.sampler, "_potential", None)) if getattr(self.sampler, "_potential_fn", None) else 0)
        if self._engine is None or self._engine_key != key:
            dev = self.device if self.device is not None or not self.devices else self.devices[0]
            self._engine = self.sampler.make_engine(self.local_chains, args, kwargs, device=dev,
                                                    chain_offset=self.chain_lo, sync_chains=self.sync_chains)
            self._engine_key = key
        return self._engine

    def _run_devices(self):
        """Devices of a multi-device run of this process's chains, or None (one engine)."""
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            return None  # one process per GPU: this rank's shard lives on its device
        if self.devices is None:
            if self.chain_method == "parallel" and self.local_chains > 1 and not getattr(MCMC, "_warned_devices", False):
                n = torch.cuda.device_count() if torch.cuda.is_available() else 0
                if n > 1:
                    # the reference's "parallel" pmaps over every local device (mcmc.py:700-715);
                    # here that is opt-in, so a multi-GPU script would silently use one device
                    MCMC._warned_devices = True
                    warnings.warn(f"chain_method='parallel' runs on one GPU unless devices= is given; {n} GPUs "
                                  "are visible: pass devices='all' to shard the chains over them as the reference's "
                                  "pmap does (or launch one process per GPU with torch.distributed)",
                                  UserWarning, stacklevel=4)
            return None
        devs = self.devices
        devs = devs[:max(1, self.local_chains)]
        return devs if len(devs) > 1 else None

    def _get_engines(self, args, kwargs, devs):
        import pickle

        from .hmc import _args_key

        key = (id(self.sampler), _args_key(args, kwargs), tuple(str(d) for d in devs))
        if self._engines is None or self._engine_key != key:
            engines = []
            pot_fn = getattr(self.sampler, "_potential_fn", None)
            for g, dev in enumerate(devs):
                lo, hi = shard_chains(self.local_chains, g, len(devs))
                if pot_fn is not None and g > 0:
                    # a user potential object binds to one device: the other shards get copies
                    # (a pickled potential is unbound; a torch potential_fn wrapper is copied: its
                    # function need not pickle)
                    import copy

                    from ..engine import Engine
                    from ..potentials import TorchPotential

                    pot = self.sampler._potential
                    pot = copy.copy(pot) if isinstance(pot, TorchPotential) else pickle.loads(pickle.dumps(pot))
                    eng = Engine(pot, hi - lo, self.sampler.options(), device=dev,
                                 chain_offset=self.chain_lo + lo, sync_chains=self.sync_chains)
                else:
                    eng = self.sampler.make_engine(hi - lo, args, kwargs, device=dev, chain_offset=self.chain_lo + lo,
                                                   sync_chains=self.sync_chains)
                engines.append(eng)
            group = shard.DeviceGroup(len(engines))
            for g, eng in enumerate(engines):
                eng.device_group = (group, g)
            self._engines, self._engine_key = engines, key
            self._engine = engines[0]
        return self._engines

    # ------------------------------------------------------------------ state
    @property
    def post_warmup_state(self):
        return self._warmup_state

    @post_warmup_state.setter
    def post_warmup_state(self, state):
        self._warmup_state = state

    @property
    def last_state(self):
        return self._last_state

    def _snapshot(self, eng, seed):
        return snapshot_state(eng, seed, keep_arena=True)

    def _restore(self, eng, state):
        restore_state(eng, state)

    # ------------------------------------------------------------------ run
    def warmup(self, rng_key, *args, extra_fields=(), collect_warmup=False, init_params=None, **kwargs):
        self._warmup_state = None
        self._run(rng_key, args, kwargs, extra_fields, init_params, n_iter=self.num_warmup,
                  lower=0 if collect_warmup else self.num_warmup)
        self._warmup_state = self._last_state

    def run(self, rng_key, *args, extra_fields=(), init_params=None, **kwargs):
        if self._warmup_state is not None:
            self._run(rng_key, args, kwargs, extra_fields, None, n_iter=self.num_samples, lower=0,
                      resume=self._warmup_state)
        else:
            self._run(rng_key, args, kwargs, extra_fields, init_params,
                      n_iter=self.num_warmup + self.num_samples, lower=self.num_warmup)

    def _run(self, rng_key, args, kwargs, extra_fields, init_params, n_iter, lower, resume=None):
        assert isinstance(extra_fields, (tuple, list))
        collect, derived = [], []
        for f in (self._sample_field,) + tuple(self._default_fields) + tuple(extra_fields):
            f = _FIELD_ALIASES.get(f, f)
            if f == self._sample_field or f in native.COLLECT:
                if f not in collect:
                    collect.append(f)
            elif f in _DERIVED_FIELDS:
                if f.startswith("adapt_state.m") or f.startswith("adapt_state.i"):
                    if lower < self.num_warmup and n_iter > 0 and resume is None:
                        raise ValueError(f"extra field {f!r}: collected for sampling draws only (the matrices "
                                         "change at the adaptation window ends during warmup)")
                if f not in derived:
                    derived.append(f)
            elif f.startswith("~"):
                continue
            else:
                raise ValueError(f"extra field {f!r} is not collected by the device engine; "
                                 f"available: {native.COLLECT + list(_DERIVED_FIELDS)}")
        self._collected = tuple(collect)
        self._derived = tuple(derived)
        self._derived_cache = {}
        # z_grad is evaluated at the unconstrained draws: collect them unconstrained and apply
        # the support transforms on the host (_site_arrays)
        self._host_constrain = "z_grad" in derived and self.postprocess_fn is None
        seed = key_to_seed(rng_key)
        bind = getattr(self.sampler, "bind_potential_fn", None)
        if bind is not None and resume is None:
            bind(init_params, self.local_chains)
        devs = self._run_devices()
        if devs is not None:
            return self._run_multi(devs, seed, args, kwargs, init_params, n_iter, lower, resume)
        eng = self._get_engine(args, kwargs)
        self._args, self._kwargs = tuple(args), dict(kwargs)
        eng.constrain_samples = self.postprocess_fn is None and not self._host_constrain
        dev = eng.device
        with torch.cuda.device(dev):
            if resume is not None:
                self._restore(eng, resume)
            else:
                ip = None
                if init_params is not None:
                    from .hmc import _flatten_init

                    ip = torch.as_tensor(_flatten_init(eng.potential, init_params, self.local_chains),
                                         dtype=torch.float32)
                    if ip.dim() == 1:
                        ip = ip[None, :].expand(eng.C, -1)
                    if ip.shape[0] == self.num_chains and self.local_chains != self.num_chains:
                        ip = ip[self.chain_lo:self.chain_hi]
                    if ip.shape[0] != eng.C:
                        raise ValueError("`init_params` must have the same leading dimension as `num_chains`.")
                eng.initialize(seed, self.num_warmup, init_params=ip, radius=self.sampler.init_radius())
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record()
            samples, fields, launches = eng.run(n_iter, seed, collect_begin=lower, thinning=self.thinning,
                                                poll_every=self.poll_every,
                                                collect_samples=not getattr(self, "_fields_only", False))
            end.record()
            end.synchronize()
            self.last_run_stats = {"launches": launches, "device_ms": start.elapsed_time(end),
                                   "iterations": n_iter}
        self._samples, self._fields = samples, fields
        self._last_state = self._snapshot(eng, seed)

    def _run_multi(self, devs, seed, args, kwargs, init_params, n_iter, lower, resume):
        """The chains sharded over `devs` (contiguous global chain ids, like the torchrun ranks),
        each shard's engine driven by its own host thread (the library calls release the GIL),
        draws and fields gathered to the first device in global chain order."""
        import threading
        import time

        engines = self._get_engines(args, kwargs, devs)
        self._args, self._kwargs = tuple(args), dict(kwargs)
        G = len(engines)
        ip_all = None
        if resume is None and init_params is not None:
            from .hmc import _flatten_init

            ip_all = torch.as_tensor(_flatten_init(engines[0].potential, init_params, self.local_chains),
                                     dtype=torch.float32)
            if ip_all.dim() == 1:
                ip_all = ip_all[None, :].expand(self.local_chains, -1)
            if ip_all.shape[0] != self.local_chains:
                raise ValueError("`init_params` must have the same leading dimension as `num_chains`.")
        parts = None
        if resume is not None:
            parts = getattr(resume, "_parts", None)
            if parts is None or len(parts) != G:
                raise ValueError(f"the state to resume holds no per-device snapshots for these {G} devices "
                                 "(it comes from a run on another device layout)")
        out, errs = [None] * G, []
        group = engines[0].device_group[0]

        def work(g):
            eng = engines[g]
            try:
                eng.constrain_samples = self.postprocess_fn is None and not self._host_constrain
                with torch.cuda.device(eng.device):
                    if parts is not None:
                        self._restore(eng, parts[g])
                    else:
                        ip = None
                        if ip_all is not None:
                            lo, hi = shard_chains(self.local_chains, g, G)
                            ip = ip_all[lo:hi]
                        eng.initialize(seed, self.num_warmup, init_params=ip, radius=self.sampler.init_radius())
                    t0 = time.perf_counter()
                    samples, fields, launches = eng.run(n_iter, seed, collect_begin=lower, thinning=self.thinning,
                                                        poll_every=self.poll_every,
                                                        collect_samples=not getattr(self, "_fields_only", False))
                    torch.cuda.synchronize(eng.device)
                    out[g] = (samples[:, :, :eng.C], fields[:, :, :eng.C], launches,
                              (time.perf_counter() - t0) * 1e3, self._snapshot(eng, seed))
            except BaseException as e:  # noqa: BLE001  (re-raised below; the others must not wait)
                errs.append(e)
                group.abort()

        threads = [threading.Thread(target=work, args=(g,)) for g in range(G)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errs:
            for eng in engines:  # a broken barrier cannot be reused
                eng.device_group = None
            self._engines = None
            raise errs[0]
        d0 = engines[0].device
        self._samples = torch.cat([o[0].to(d0) for o in out], dim=2)
        self._fields = torch.cat([o[1].to(d0) for o in out], dim=2)
        self.last_run_stats = {"launches": max(o[2] for o in out), "device_ms": max(o[3] for o in out),
                               "iterations": n_iter, "devices": [str(e.device) for e in engines]}
        self._last_state = _combine_states([o[4] for o in out], engines, d0)

    # ------------------------------------------------------------------ results
    def _model_potential(self):
        """The model's potential (site layout, deterministic sites): the engine's, or -- for an
        unpickled MCMC, which has no engine -- rebuilt from the sampler and the run's args."""
        if self._engine is not None:
            return self._engine.model_potential
        if self._host_potential is None:
            self._host_potential = self.sampler.potential(self._args, self._kwargs)
        return self._host_potential

    def _site_arrays(self, group_by_chain, include_deterministic=True):
        pot = self._model_potential()
        C = self.local_chains
        S = self._samples.shape[0]
        flat = self._samples[:, :, :C].permute(2, 0, 1)  # [C, S, D]
        if getattr(self, "_host_constrain", False):
            from ..potentials import POSITIVE

            codes = pot.transform_codes().to(flat.device)
            if bool((codes == POSITIVE).any()):
                flat = torch.where(codes == POSITIVE, torch.exp(flat), flat)
        out = pot.unflatten(flat)
        if self.postprocess_fn is not None:
            # draws are unconstrained here (Engine.constrain_samples = False)
            names = set(out)
            out = _postprocess_per_draw(self.postprocess_fn, out)
            if not include_deterministic:  # print_summary keeps the sample sites (mcmc.py:748-758)
                out = {k: v for k, v in out.items() if k in names}
        elif include_deterministic:
            out.update(pot.deterministic(out))
        if not group_by_chain:
            out = {k: v.reshape(C * S, *v.shape[2:]) for k, v in out.items()}
        return out

    def get_samples(self, group_by_chain=False):
        out = self._site_arrays(group_by_chain)
        if getattr(self._model_potential(), "array_site", False) and self.postprocess_fn is None:
            return out["z"]  # potential_fn over one array: the samples are that array (mcmc.py:761-786)
        return out

    def get_extra_fields(self, group_by_chain=False):
        out = {}
        for f in self._collected:
            if f == self._sample_field:
                continue
            v = self._fields[:, native.COLLECT.index(f), :self.local_chains].t()  # [C, S]
            if f == "num_steps" or f == "i":
                v = v.round().to(torch.int32)
            elif f == "diverging":
                v = v > 0.5
            if not group_by_chain:
                v = v.reshape(-1)
            out["adapt_state.step_size" if f == "step_size" else f] = v
        for f in getattr(self, "_derived", ()):
            out[f] = self._derived_field(f, group_by_chain)
        return out

    def _derived_field(self, f, group_by_chain):
        """The _DERIVED_FIELDS values, [C, S, ...] (or flattened over chains and draws)."""
        C, S = self.local_chains, self._samples.shape[0]
        eng = self._engine
        if f == "r":
            return None
        if f == "trajectory_length":
            tl = self.sampler.options().trajectory_length if self.sampler.options().algo == native.ALGO_HMC else None
            if tl is None:
                return None
            v = torch.full((C, S), float(tl), dtype=torch.float32, device=self._samples.device)
            return v if group_by_chain else v.reshape(-1)
        if f == "z_grad":
            if "z_grad" not in self._derived_cache:
                if self._engines is not None:
                    raise NotImplementedError("extra field 'z_grad' with chains over several devices")
                g = torch.empty_like(self._samples)  # [S, D, ldc]
                for k in range(S):
                    g[k] = eng.model_gradient(self._samples[k].contiguous())
                self._derived_cache["z_grad"] = g
            pot = self._model_potential()
            gv = self._derived_cache["z_grad"][:, :, :C].permute(2, 0, 1)  # [C, S, D]
            out = pot.unflatten(gv)
            if getattr(pot, "array_site", False):
                out = out["z"]
                return out if group_by_chain else out.reshape(C * S, *out.shape[2:])
            return out if group_by_chain else {k: v.reshape(C * S, *v.shape[2:]) for k, v in out.items()}
        # adapt_state mass matrices: the post-warmup matrices of every sampling draw
        imm, msq, msq_inv = (self._last_state.adapt_state.inverse_mass_matrix,
                             self._last_state.adapt_state.mass_matrix_sqrt,
                             self._last_state.adapt_state.mass_matrix_sqrt_inv)
        m = {"adapt_state.inverse_mass_matrix": imm, "adapt_state.mass_matrix_sqrt": msq,
             "adapt_state.mass_matrix_sqrt_inv": msq_inv}[f]

        # one matrix shared by every chain (pooled, or a given dense matrix that is not adapted)
        # or one per chain (diagonal [C, D], per-chain dense [C, D, D])
        shared = eng is not None and eng.dense and not eng.chain_dense

        def per_draw(v):
            v = torch.as_tensor(v)
            v = v[None].expand(C, *v.shape) if shared else v
            v = v[:, None].expand(C, S, *v.shape[1:])
            return v if group_by_chain else v.reshape(C * S, *v.shape[2:])

        return {k: per_draw(v) for k, v in m.items()} if isinstance(m, dict) else per_draw(m)

    def gather_samples(self, group_by_chain=False):
        """get_samples over the chains of every rank (all_gather; identical to get_samples
        with one process)."""
        out = {k: shard.gather_chains(v) for k, v in self._site_arrays(True).items()}
        if not group_by_chain:
            out = {k: v.reshape(v.shape[0] * v.shape[1], *v.shape[2:]) for k, v in out.items()}
        return out

    def print_summary(self, prob=0.9, exclude_deterministic=True):
        """numpyro/infer/mcmc.py:710-738.  Under torch.distributed the table covers every
        rank's chains (moments and diagnostics by all_reduce, quantiles from the gathered
        draws) and rank 0 prints it."""
        rank, world = shard.dist_info()
        arrays = self._site_arrays(True, include_deterministic=not exclude_deterministic)
        if world == 1:
            sites = {k: v.detach().cpu().numpy() for k, v in arrays.items()}
            diagnostics.print_summary(sites, prob=prob)
        else:
            stats = shard.summary(arrays, prob=prob)
            if rank == 0:
                diagnostics.print_summary_table(stats, prob)
        ef = self.get_extra_fields()
        if "diverging" in ef:
            n = torch.tensor([float(ef["diverging"].sum())], dtype=torch.float64, device=ef["diverging"].device)
            n = shard._all_reduce(n) if world > 1 else n
            if rank == 0:
                print("Number of divergences: {}".format(int(n.item())))

    def transfer_states_to_host(self):
        self._samples = self._samples.cpu()
        self._fields = self._fields.cpu()

    def __getstate__(self):
        # mcmc.py:797-800: the engine (device arena, bound kernels) is rebuilt on the next run;
        # post_warmup_state / last_state keep host copies of the chain state (HMCState)
        state = self.__dict__.copy()
        state["_engine"] = None
        state["_engine_key"] = None
        state["_engines"] = None
        state["_host_potential"] = None
        return state


def _combine_states(parts, engines, device):
    """One HMCState over the chains of every device (global chain order: per-chain fields
    concatenated, a pooled / shared dense matrix taken once); the per-device snapshots ride
    along as `_parts` for resuming (MCMC.post_warmup_state = last_state)."""
    from .hmc import HMCAdaptState, HMCState

    shared_mass = engines[0].dense and not engines[0].chain_dense

    def cat(vals, shared=False):
        v0 = vals[0]
        if isinstance(v0, torch.Tensor):
            if shared or v0.dim() == 0:
                return v0.to(device)
            return torch.cat([v.to(device) for v in vals], dim=0)
        if isinstance(v0, dict):
            return {k: cat([v[k] for v in vals], shared) for k in v0}
        if isinstance(v0, tuple) and not hasattr(v0, "_fields"):
            return tuple(cat([v[i] for v in vals], shared) for i in range(len(v0)))
        return v0

    a = [p.adapt_state for p in parts]
    adapt = HMCAdaptState(
        cat([x.step_size for x in a]),
        cat([x.inverse_mass_matrix for x in a], shared_mass),
        cat([x.mass_matrix_sqrt for x in a], shared_mass),
        cat([x.mass_matrix_sqrt_inv for x in a], shared_mass),
        cat([x.ss_state for x in a]), cat([x.mm_state for x in a]), cat([x.window_idx for x in a]), a[0].rng_key)
    st = HMCState(*[cat([getattr(p, f) for p in parts]) if f not in ("adapt_state", "trajectory_length", "rng_key")
                    else (adapt if f == "adapt_state" else getattr(parts[0], f)) for f in HMCState._fields])
    st._parts = list(parts)
    st._engine = None
    st._layout = ("devices", tuple(p._layout for p in parts))
    return st
