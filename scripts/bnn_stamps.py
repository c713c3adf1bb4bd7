"""Per-phase cycles of k_bnn_c3 from the stamped experiment build (scripts/ab_bnn_stamps_src.py).
usage: NUMPYRO_AMD_LIB=build/abx_bnnst/st/libnumpyro_amd.so python scripts/bnn_stamps.py [chains]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import datasets, native  # noqa: E402
from numpyro_amd.potentials import BNN  # noqa: E402

NAMES = ["params + data to LDS", "h1 = tanh(X W1)", "P1 h2 = tanh(h1 W2)", "yhat, residual", "grad w3",
         "ga2", "P2 grad W2", "P3 ga1", "grad W1", "block sums + U"]
C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
X, Y = datasets.bnn_data(N=100, D_X=3)
dev = torch.device("cuda:0")
ldc = (C + 63) // 64 * 64
pot = BNN(X, Y, 69)
pot.bind(C, ldc, dev)
z = (0.3 * torch.randn(pot.dim, ldc, device=dev)).contiguous()
g = torch.zeros(pot.dim, ldc, device=dev)
pe = torch.zeros(ldc, device=dev)
ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=C, ldc=ldc)
s = native.stream_ptr()
for _ in range(5):
    pot.evaluate(ev, s)
torch.cuda.synchronize()
buf = np.zeros((1024, 12), np.uint64)
native.lib().nmx_x_bnn_stamps(ctypes.c_void_p(buf.ctypes.data))
n = int((buf[:, 0] > 0).sum())
d = np.diff(buf[:n, :11].astype(np.int64), axis=1)
med = np.median(d, axis=0)
tot = float(np.median(buf[:n, 10].astype(np.int64) - buf[:n, 0].astype(np.int64)))
print(f"k_bnn_c3 C={C}: {n} workgroups, median {tot:.0f} cycles per chain evaluation")
for i, nm in enumerate(NAMES):
    print(f"  {nm:24s} {med[i]:8.0f} cycles {100 * med[i] / tot:5.1f}%")
