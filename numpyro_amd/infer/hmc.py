"""HMC / NUTS kernels with numpyro's constructor signatures (numpyro/infer/hmc.py:541-948).

The kernel objects validate and hold the sampler options; the transitions themselves run
in the device state machine (csrc/nuts.hip) driven by ``numpyro_amd.engine.Engine``.
``MCMCKernel`` keeps the plug-in surface of numpyro/infer/mcmc.py:32-158 (``init``,
``sample``, ``sample_field``, ``default_fields``, ``postprocess_fn``).
"""
from __future__ import annotations

import math
import warnings
from collections import namedtuple

from .. import native
from ..engine import Engine, SamplerOptions
from ..potentials import FusedModel, Potential

_HMCStateBase = namedtuple(
    "HMCState",
    ["i", "z", "z_grad", "potential_energy", "energy", "r", "trajectory_length", "num_steps",
     "accept_prob", "mean_accept_prob", "diverging", "adapt_state", "rng_key"])


class HMCState(_HMCStateBase):
    """numpyro/infer/hmc.py:31-48 field names; values are per-chain torch tensors (chains
    first).  Carries a device snapshot so it can be used as ``post_warmup_state``.

    Pickling (test/test_pickle.py:215-220; MCMC.__getstate__ / HMC.__getstate__ at
    mcmc.py:797-800, hmc.py:818-822): the snapshot travels as host tensors without the engine
    reference; an engine of the same layout (model, chains, dimension, depth, mass-matrix
    mode) resumes it, in this or another process."""

    def __reduce__(self):
        extra = {k: v for k, v in self.__dict__.items() if k != "_engine"}
        eng = self.__dict__.get("_engine")
        if extra.get("_arena") is None and eng is not None and eng.generation == extra.get("_generation"):
            # the current state of its engine (kernel.sample's in-place snapshot): its arena is it
            extra["_arena"] = eng.arena
        if extra.get("_arena") is not None:
            extra["_arena"] = extra["_arena"].cpu()
        w = extra.get("_whitening")
        if w is not None:
            extra["_whitening"] = tuple(None if t is None else t.cpu() for t in w)
        return (_rebuild_state, (tuple(self), extra))


def _rebuild_state(fields, extra):
    st = HMCState(*fields)
    st.__dict__.update(extra)
    st._engine = None
    return st


HMCAdaptState = namedtuple(  # hmc_util.py:18-30
    "HMCAdaptState",
    ["step_size", "inverse_mass_matrix", "mass_matrix_sqrt", "mass_matrix_sqrt_inv", "ss_state",
     "mm_state", "window_idx", "rng_key"])


def snapshot_state(eng, seed, keep_arena=True):
    """HMCState of every chain of `eng` after its last transition (hmc.py:31-48 fields, chains
    first).  `keep_arena` copies the device state so the snapshot can be resumed later
    (MCMC.post_warmup_state / last_state); without it the state is resumable only while the
    engine has not moved on (MCMCKernel.sample's in-place stepping)."""
    C = eng.C
    z_flat, zgrad = eng.model_state()
    pot = eng.potential
    z = pot.unflatten(z_flat) if len(pot.sites) else z_flat
    imm, msq, msq_inv = eng.mass_state()
    adapt = HMCAdaptState(
        eng.chain_state("step_size").clone(), imm, msq, msq_inv,
        (eng.chain_state("da_xt").clone(), eng.chain_state("da_xavg").clone(),
         eng.chain_state("da_gavg").clone(), eng.chain_state("da_t").clone(),
         eng.chain_state("da_prox").clone()),
        (eng.chain_state("wf_mean").clone(), eng.chain_state("wf_m2").clone(),
         eng.chain_state("wf_n").clone()),
        eng.chain_state("window_idx").clone(), seed)
    st = HMCState(
        eng.chain_state("iter").clone(), z, zgrad,
        eng.chain_state("pe").clone(), eng.chain_state("energy").clone(), None,
        eng.opts.trajectory_length, eng.chain_state("last_nsteps").clone(),
        eng.chain_state("last_acc").clone(), eng.chain_state("mean_acc").clone(),
        eng.chain_state("last_div").clone().bool(), adapt, seed)
    st._arena = eng.arena.clone() if keep_arena else None
    st._whitening = eng.whitening_state()
    st._iteration = eng.iteration
    st._num_warmup = eng.num_warmup
    st._generation = eng.generation
    st._iter_capacity = eng.iter_capacity
    st._layout = eng.layout()
    st._engine = eng
    assert C == st.i.shape[0]
    return st


def _refuse_combined(state):
    """A state of a multi-device MCMC run (layout ('devices', ...)) holds one snapshot per device:
    only that MCMC (post_warmup_state / last_state with the same devices) can resume it."""
    lay = getattr(state, "_layout", None)
    if isinstance(lay, tuple) and lay and lay[0] == "devices":
        raise ValueError(f"this state comes from a run over {len(lay[1])} devices (MCMC(devices=...)) and holds "
                         "one snapshot per device; resume it with an MCMC over the same devices (post_warmup_state "
                         "= state), not with a single engine or kernel.sample()")


def restore_state(eng, state):
    """Make `state` the engine's current state (no copy when it already is).  A state of
    another engine -- e.g. unpickled from another process -- is copied in when its layout
    matches (same model, chains, dimension, depth, mass-matrix mode), and is then bound to
    this engine."""
    _refuse_combined(state)
    own = getattr(state, "_engine", None) is eng
    if not own:
        if getattr(state, "_engine", None) is not None or getattr(state, "_layout", None) != eng.layout():
            raise ValueError("the state belongs to a different model/data binding (layout "
                             f"{getattr(state, '_layout', None)} vs {eng.layout()})")
    elif eng.generation == state._generation:
        return
    if state._arena is None:
        raise ValueError("this state was advanced in place by a later sample() call and holds no device "
                         "copy; pass the state returned by the most recent sample()")
    if eng.arena is None or eng.iter_capacity != state._iter_capacity:
        eng._alloc(state._iter_capacity)
    eng.arena.copy_(state._arena)
    eng.set_whitening_state(state._whitening)
    eng.iteration = state._iteration
    eng.num_warmup = state._num_warmup
    eng._pool = None
    eng.generation = state._generation
    state._engine = eng


class PooledGroups(list):
    """dense_mass=pooled([("x", "y"), ...]): the structured mass of the listed site groups
    (hmc.py:239-252: dense blocks, one diagonal block over the other sites) adapted ONCE from the
    draws of all chains -- the labelled opt-in for groups whose per-chain blocks do not fit (the
    reference adapts one matrix per chain; dense_mass='pooled' is the same for one dense block over
    every site)."""


def pooled(groups):
    """Mark a structured dense_mass as pooled over chains (PooledGroups)."""
    return PooledGroups(tuple(g) for g in groups)


class MCMCKernel:
    """Interface of numpyro/infer/mcmc.py:32-158."""

    def postprocess_fn(self, model_args, model_kwargs):
        return lambda x: x

    def init(self, rng_key, num_warmup, init_params, model_args, model_kwargs):
        raise NotImplementedError

    def sample(self, state, model_args, model_kwargs):
        raise NotImplementedError

    @property
    def sample_field(self):
        raise NotImplementedError

    @property
    def default_fields(self):
        return (self.sample_field,)

    @property
    def is_ensemble_kernel(self):
        return False

    def get_diagnostics_str(self, state):
        return ""


def _args_key(model_args, model_kwargs):
    """Identity of the model arguments an engine's potential is bound to (MCMC._get_engine keys
    its engine the same way)."""
    return (tuple(id(a) for a in (model_args or ())),
            tuple(sorted((k, id(v)) for k, v in (model_kwargs or {}).items())))


def init_to_uniform(site=None, radius=2):
    """Marker for the default init strategy (numpyro/infer/initialization.py:95-129)."""
    return ("uniform", float(radius))


def _flatten_init(pot, init_params, num_chains):
    """init_params (a dict of sites with a leading chain dimension, or [C, D] / [D]) -> [C, D];
    for one chain of a potential_fn the reference's unbatched values are accepted too."""
    import torch

    from ..potentials import TorchPotential

    if isinstance(pot, TorchPotential) and num_chains == 1:
        if isinstance(init_params, dict):
            init_params = {k: torch.as_tensor(v)[None] for k, v in init_params.items()}
        else:
            init_params = torch.as_tensor(init_params).reshape(1, -1)
    elif isinstance(pot, TorchPotential) and not isinstance(init_params, dict):
        init_params = torch.as_tensor(init_params).reshape(num_chains, -1)
    return pot.flatten(init_params) if isinstance(init_params, dict) else init_params


class HMC(MCMCKernel):
    """Hamiltonian Monte Carlo with fixed trajectory length (numpyro/infer/hmc.py:541-822)."""

    _algo = native.ALGO_HMC

    def __init__(self, model=None, potential_fn=None, kinetic_fn=None, step_size=1.0,
                 inverse_mass_matrix=None, adapt_step_size=True, adapt_mass_matrix=True,
                 dense_mass=False, target_accept_prob=0.8, num_steps=None,
                 trajectory_length=2 * math.pi, init_strategy=init_to_uniform,
                 find_heuristic_step_size=False, forward_mode_differentiation=False,
                 regularize_mass_matrix=True):
        if not (model is None) ^ (potential_fn is None):
            raise ValueError("Only one of `model` or `potential_fn` must be specified.")
        if type(self) is HMC:
            if num_steps is None and trajectory_length is None:
                raise ValueError("At least one of `num_steps` or `trajectory_length` must be specified.")
            if adapt_step_size and num_steps is not None and trajectory_length is not None:
                warnings.warn("If both `num_steps` and `trajectory_length` are specified step size "
                              "can't be adapted", stacklevel=2)
        if kinetic_fn is not None:
            from .hmc_util import euclidean_kinetic_energy
            if kinetic_fn is not euclidean_kinetic_energy:
                raise NotImplementedError("custom kinetic_fn: the engine integrates the Euclidean kinetic energy "
                                          "(numpyro_amd.infer.hmc_util.euclidean_kinetic_energy) only")
        self._pooled = isinstance(dense_mass, PooledGroups)
        if isinstance(dense_mass, str):
            if dense_mass != "pooled":
                raise ValueError("dense_mass must be a bool, 'pooled' or a list of site groups")
            warnings.warn("dense_mass='pooled': one dense mass matrix is adapted from the draws of all chains "
                          "(not per chain as in numpyro); chains share it", stacklevel=2)
        if self._pooled:
            warnings.warn("dense_mass=pooled([...]): one structured mass matrix (dense blocks over the listed "
                          "site groups, diagonal elsewhere) is adapted from the draws of all chains (not per chain "
                          "as in numpyro); chains share it", stacklevel=2)
        if isinstance(dense_mass, (list, tuple)):
            # structured mass (hmc.py:239-252): dense blocks over the listed site groups, one
            # diagonal block over the remaining sites; adapted per chain (dense.MassBlocks)
            dense_mass = [tuple(g) for g in dense_mass]
            if not all(len(g) > 0 and all(isinstance(n, str) for n in g) for g in dense_mass):
                raise ValueError("dense_mass as a list holds tuples of site names, e.g. [('x', 'y')]")
        # an inverse_mass_matrix dict {site group: block} (hmc_util.py:439-487) is assembled in
        # ravel coordinates by the engine (dense.assemble_inverse_mass_matrix)
        if model is not None and not (isinstance(model, FusedModel) or callable(model)):
            raise TypeError("`model` must be a model function (numpyro_amd.sample / plate / distributions, "
                            "mapped onto a fused kernel by numpyro_amd.frontend) or a fused model")
        if potential_fn is not None and not (isinstance(potential_fn, Potential) or callable(potential_fn)):
            raise TypeError("`potential_fn` must be a callable of the unconstrained parameters (torch "
                            "operations) or a numpyro_amd.potentials.Potential")
        self._model = model
        self._potential_fn = potential_fn
        self._step_size = float(step_size)
        self._inverse_mass_matrix = inverse_mass_matrix
        self._adapt_step_size = adapt_step_size
        self._adapt_mass_matrix = adapt_mass_matrix
        self._dense_mass = dense_mass
        self._target_accept_prob = target_accept_prob
        self._num_steps = num_steps
        self._trajectory_length = (float(trajectory_length) if trajectory_length is not None else None)
        self._max_tree_depth = 10
        self._init_strategy = init_strategy
        self._regularize_mass_matrix = regularize_mass_matrix
        self._find_heuristic_step_size = bool(find_heuristic_step_size)
        # a plain callable becomes a TorchPotential once init_params show its argument structure
        # (bind_potential_fn); a Potential is used as given
        self._potential = potential_fn if isinstance(potential_fn, Potential) else None
        self._sample_fn = None

    @property
    def model(self):
        return self._model

    @property
    def sample_field(self):
        return "z"

    @property
    def default_fields(self):
        return ("z", "diverging")

    def get_diagnostics_str(self, state):
        return "{} steps of size {:.2e}. acc. prob={:.2f}".format(
            state.num_steps, state.adapt_state.step_size, state.mean_accept_prob)

    def options(self) -> SamplerOptions:
        md = self._max_tree_depth
        md = tuple(md) if isinstance(md, (tuple, list)) else (int(md), int(md))
        return SamplerOptions(
            algo=self._algo, step_size=self._step_size, adapt_step_size=self._adapt_step_size,
            adapt_mass_matrix=self._adapt_mass_matrix,
            dense_mass="pooled" if (self._dense_mass == "pooled" or getattr(self, "_pooled", False))
            else bool(self._dense_mass),
            dense_blocks=list(self._dense_mass) if isinstance(self._dense_mass, list) and self._dense_mass else None,
            target_accept_prob=self._target_accept_prob, max_tree_depth=md,
            trajectory_length=self._trajectory_length, num_steps=self._num_steps,
            regularize_mass_matrix=self._regularize_mass_matrix,
            inverse_mass_matrix=self._inverse_mass_matrix,
            find_heuristic_step_size=self._find_heuristic_step_size)

    def bind_potential_fn(self, init_params, num_chains):
        """A callable ``potential_fn`` (hmc.py:127-130: a function of one chain's unconstrained
        values) is wrapped as a TorchPotential whose site structure is that of ``init_params``
        (required with ``potential_fn``, hmc.py:754-757); batched init_params carry a leading
        chain dimension when num_chains > 1.  No-op for models and Potential objects."""
        fn = self._potential_fn
        if fn is None or isinstance(fn, Potential):
            return
        if init_params is None:
            if self._potential is None:
                raise ValueError("Valid value of `init_params` must be provided with `potential_fn`.")
            return
        import torch

        from ..potentials import TorchPotential

        def one(v):
            v = torch.as_tensor(v)
            return v[0] if num_chains > 1 else v

        example = {k: one(v) for k, v in init_params.items()} if isinstance(init_params, dict) else one(init_params)
        old = self._potential
        if old is None or old.sites != TorchPotential(fn, example).sites:
            self._potential = TorchPotential(fn, example)

    def potential(self, model_args=(), model_kwargs=None) -> Potential:
        if self._potential_fn is not None and self._potential is None:
            raise ValueError("Valid value of `init_params` must be provided with `potential_fn`.")
        if isinstance(self._model, FusedModel):
            self._potential = self._model.potential(*model_args, **(model_kwargs or {}))
        elif self._model is not None:
            # model front end: trace the model and map it onto its fused kernel
            # (initialize_model, numpyro/infer/util.py:632-800)
            from ..frontend import potential_from_model

            self._potential = potential_from_model(self._model, model_args, model_kwargs)
        return self._potential

    def init_radius(self):
        s = self._init_strategy
        if s is init_to_uniform:
            return 2.0
        if isinstance(s, tuple) and s and s[0] == "uniform":
            return float(s[1])
        raise NotImplementedError("only init_to_uniform is supported")

    def make_engine(self, num_chains, model_args=(), model_kwargs=None, device=None, chain_offset=0,
                    sync_chains=False) -> Engine:
        return Engine(self.potential(model_args, model_kwargs), num_chains, self.options(), device=device,
                      chain_offset=chain_offset, sync_chains=sync_chains)

    def init(self, rng_key, num_warmup, init_params=None, model_args=(), model_kwargs={}, *,
             num_chains=None, chain_offset=0, device=None):
        """HMC.init (hmc.py:740-822), vectorized: initialises `num_chains` chains on the device
        (init_to_uniform with retries, or `init_params`) and returns their HMCState.

        The chain count is `num_chains`, else the leading dimension of a batch of keys
        (`random.split(key, C)`, as MCMC's vectorized path passes them) or of `init_params`,
        else 1.  Chain c draws from the Philox stream (seed of the first key, chain_offset + c),
        so a loop of `sample` calls reproduces `MCMC.run` with the same key bitwise."""
        import numpy as np
        import torch

        from ..random import key_to_seed

        keys = np.asarray(rng_key.cpu().numpy() if hasattr(rng_key, "cpu") else rng_key)
        if num_chains is None:
            if keys.ndim == 2:
                num_chains = keys.shape[0]
            elif init_params is not None and not isinstance(init_params, dict) and np.ndim(init_params) == 2:
                num_chains = int(np.shape(init_params)[0])
            elif isinstance(init_params, dict):
                num_chains = int(np.shape(next(iter(init_params.values())))[0])
            else:
                num_chains = 1
        seed = key_to_seed(keys)
        self.bind_potential_fn(init_params, int(num_chains))
        eng = self.make_engine(int(num_chains), model_args, model_kwargs, device=device,
                               chain_offset=chain_offset)
        ip = None
        if init_params is not None:
            ip = _flatten_init(eng.potential, init_params, int(num_chains))
            ip = torch.as_tensor(ip, dtype=torch.float32)
            if ip.dim() == 1:
                ip = ip[None, :].expand(eng.C, -1)
        with torch.cuda.device(eng.device):
            eng.initialize(seed, int(num_warmup), init_params=ip, radius=self.init_radius())
        self._engine, self._seed = eng, seed
        self._engine_args = _args_key(model_args, model_kwargs)
        self._sample_fn = self.sample
        return snapshot_state(eng, seed, keep_arena=False)

    def sample(self, state, model_args=(), model_kwargs=None):
        """One transition of every chain (sample_kernel, hmc.py:459-530) on the device; returns
        the new HMCState.  The engine advances in place: the returned state is current, the
        argument becomes a plain record (resuming from it needs a state with a device copy,
        e.g. MCMC.post_warmup_state)."""
        import torch

        _refuse_combined(state)
        eng = getattr(state, "_engine", None)
        if eng is None:
            if getattr(state, "_layout", None) is None:
                raise ValueError("state must come from init() or sample() of this kernel")
            # an unpickled state: resumed by an engine of this kernel for these model args
            # (the engine's bound data must be these model args: same layout is not enough)
            eng = getattr(self, "_engine", None)
            if (eng is None or eng.layout() != state._layout
                    or getattr(self, "_engine_args", None) != _args_key(model_args, model_kwargs)):
                C, chain_offset = state._layout[1], state._layout[4]
                eng = self.make_engine(C, model_args, model_kwargs, chain_offset=chain_offset)
                self._engine = eng
                self._engine_args = _args_key(model_args, model_kwargs)
        with torch.cuda.device(eng.device):
            restore_state(eng, state)
            eng.run(1, state.adapt_state.rng_key, collection_size=0)
        return snapshot_state(eng, state.adapt_state.rng_key, keep_arena=False)

    def postprocess_fn(self, model_args=(), model_kwargs=None):
        """Unconstrained site values -> constrained ones plus deterministic sites
        (infer/util.py:176-190 constrain_fn)."""
        import torch

        from ..potentials import POSITIVE

        pot = self.potential(model_args, model_kwargs)

        def fn(z):
            if not isinstance(z, dict):
                z = pot.unflatten(z)
            out = {}
            for name, _, tr in pot.sites:
                out[name] = torch.exp(z[name]) if tr == POSITIVE else z[name]
            out.update(pot.deterministic(out))
            return out

        return fn

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_sample_fn"] = None
        state["_engine"] = None
        state["_engine_args"] = None
        if self._model is not None:  # rebuilt from the model and its args by potential()
            state["_potential"] = None
        return state


class NUTS(HMC):
    """No-U-Turn Sampler (numpyro/infer/hmc.py:825-948)."""

    _algo = native.ALGO_NUTS

    def __init__(self, model=None, potential_fn=None, kinetic_fn=None, step_size=1.0,
                 inverse_mass_matrix=None, adapt_step_size=True, adapt_mass_matrix=True,
                 dense_mass=False, target_accept_prob=0.8, trajectory_length=None, max_tree_depth=10,
                 init_strategy=init_to_uniform, find_heuristic_step_size=False,
                 forward_mode_differentiation=False, regularize_mass_matrix=True):
        super().__init__(potential_fn=potential_fn, model=model, kinetic_fn=kinetic_fn,
                         step_size=step_size, inverse_mass_matrix=inverse_mass_matrix,
                         adapt_step_size=adapt_step_size, adapt_mass_matrix=adapt_mass_matrix,
                         dense_mass=dense_mass, target_accept_prob=target_accept_prob,
                         trajectory_length=trajectory_length, init_strategy=init_strategy,
                         find_heuristic_step_size=find_heuristic_step_size,
                         forward_mode_differentiation=forward_mode_differentiation,
                         regularize_mass_matrix=regularize_mass_matrix)
        self._max_tree_depth = max_tree_depth
