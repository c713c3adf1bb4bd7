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
    first).  Carries a device snapshot so it can be used as ``post_warmup_state``."""


HMCAdaptState = namedtuple(  # hmc_util.py:18-30
    "HMCAdaptState",
    ["step_size", "inverse_mass_matrix", "mass_matrix_sqrt", "mass_matrix_sqrt_inv", "ss_state",
     "mm_state", "window_idx", "rng_key"])


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


def init_to_uniform(site=None, radius=2):
    """Marker for the default init strategy (numpyro/infer/initialization.py:95-129)."""
    return ("uniform", float(radius))


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
            raise NotImplementedError("custom kinetic_fn: the engine uses the Euclidean kinetic energy")
        if find_heuristic_step_size:
            raise NotImplementedError("find_heuristic_step_size=True is not supported yet")
        if isinstance(dense_mass, (list, tuple)) and len(dense_mass) > 0:
            raise NotImplementedError("structured dense_mass (list of site groups) is not supported; "
                                      "use dense_mass=True for a full dense mass matrix")
        if model is not None and not isinstance(model, FusedModel):
            raise TypeError("`model` must be a fused model (numpyro_amd.potentials.*); arbitrary "
                            "Python models cannot run on the device engine")
        if potential_fn is not None and not isinstance(potential_fn, Potential):
            raise TypeError("`potential_fn` must be a numpyro_amd.potentials.Potential")
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
        self._potential = potential_fn
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
            adapt_mass_matrix=self._adapt_mass_matrix, dense_mass=bool(self._dense_mass),
            target_accept_prob=self._target_accept_prob, max_tree_depth=md,
            trajectory_length=self._trajectory_length, num_steps=self._num_steps,
            regularize_mass_matrix=self._regularize_mass_matrix,
            inverse_mass_matrix=self._inverse_mass_matrix)

    def potential(self, model_args=(), model_kwargs=None) -> Potential:
        if self._model is not None:
            self._potential = self._model.potential(*model_args, **(model_kwargs or {}))
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

    def init(self, rng_key, num_warmup, init_params=None, model_args=(), model_kwargs={}):
        raise NotImplementedError("drive the device engine through numpyro_amd.infer.MCMC")

    def sample(self, state, model_args, model_kwargs):
        raise NotImplementedError("drive the device engine through numpyro_amd.infer.MCMC")

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_sample_fn"] = None
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
