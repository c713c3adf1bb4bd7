"""Per-phase cycle breakdown of the persistent wide kernel (k_wide_persistent): the library built
with -DNMX_PX_PROF (scripts/ab_build.py nuts.hip pxprof='-DNMX_PX_PROF') accumulates thread 0's
shader-clock cycles per phase of every leaf; this runs a short SV / funnel warmup through it and
prints the average cycles per leaf and each phase's share.
    python scripts/px_profile.py [sv|funnel] [chains]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numpyro_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath("build/ab/pxprof/libnumpyro_amd.so")
import torch  # noqa: E402

from numpyro_amd import datasets  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402

NAMES = ["leaf rows + wave sums", "reduction barrier wait", "leaf total (rows..fin+scalar rows)",
         "scalar logic (wave 0)", "apply rows", "end barrier wait", "whole leaf"]


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "sv"
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    lib = native.lib()
    fn = lib.nmx_debug_px_profile
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 16)()
    if which == "sv":
        model, args = P.stochastic_volatility, (datasets.sp500_synthetic(),)
    else:
        model, args = P.funnel, (10000,)
    mcmc = MCMC(NUTS(model), num_warmup=30, num_samples=5, num_chains=chains, progress_bar=False)
    mcmc.warmup(0, *args)
    torch.cuda.synchronize()
    native.check(fn(ctypes.addressof(buf)))  # reset after the warmup
    mcmc.run(1, *args)
    torch.cuda.synchronize()
    native.check(fn(ctypes.addressof(buf)))
    leaves = buf[7]
    whole = buf[6] / leaves
    print(f"{which} C={chains}: {leaves} leaves (thread 0 of each block), {whole:.0f} cycles per leaf")
    for i, n in enumerate(NAMES):
        print(f"  {n:40s} {buf[i] / leaves:10.0f} cycles  {buf[i] / buf[6]:6.1%}")


if __name__ == "__main__":
    main()
