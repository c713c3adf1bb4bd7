"""numpyro.infer drop-in surface for the MI355X engine (MCMC, NUTS, HMC)."""
from .hmc import HMC, NUTS, HMCAdaptState, HMCState, MCMCKernel, init_to_uniform, pooled  # noqa: F401
from .mcmc import MCMC, shard_chains  # noqa: F401
from .predictive import Predictive  # noqa: F401

__all__ = ["HMC", "NUTS", "MCMC", "MCMCKernel", "HMCState", "HMCAdaptState", "init_to_uniform", "Predictive", "pooled"]
