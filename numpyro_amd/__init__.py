"""numpyro_amd: an MI355X-native NUTS/HMC engine behind numpyro's MCMC API.

Hot path: the vectorized-chain leapfrog + iterative NUTS tree (numpyro/infer/hmc_util.py)
as a device state machine (csrc/nuts.hip) driving fused potential+gradient HIP kernels
(csrc/potential_*.hip), reached through the C-ABI in include/numpyro_amd.h.
"""
__version__ = "0.1.0"

from . import diagnostics, random  # noqa: F401,E402
from . import distributions, jnp  # noqa: F401,E402
from .frontend import LocScaleReparam, reparam  # noqa: F401,E402
from .primitives import deterministic, plate, sample  # noqa: F401,E402
