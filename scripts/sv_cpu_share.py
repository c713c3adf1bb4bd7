"""CPU-baseline probe: the C NUTS restatement on stochastic volatility (32 chains, 6 s): leapfrog/s and
the potential share of its wall time (bench.py c4 CPU leg shape).  usage: python scripts/sv_cpu_share.py"""
import numpy as np, sys
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cpu_nuts as CN
from numpyro_amd import datasets
r = datasets.sp500_synthetic()
cn = CN.CpuNuts("sv", r)
D = cn.dim
C = 32
rs = np.random.RandomState(0)
z = np.zeros((C, D), np.float32); z[:, 0] = np.log(10.0); z[:, -1] = np.log(0.02); z[:, 1:-1] = np.log(np.abs(r).mean()) + 0.1 * rs.randn(C, D - 2)
from oracle import batched as OB
pe, g = OB.SVBatch(r)(z)
out = cn.run(z, g, pe, np.full(C, 0.02, np.float32), np.ones((C, D), np.float32), np.ones((C, D), np.float32), 1, 0, 1 << 14, min_transitions=0, seconds=6.0, keep_z=False)
print("threads", cn.threads(), "leapfrog/s", out["leapfrogs"] / out["wall_s"], "share", out["potential_s"] / out["wall_s"])
