"""Per-phase cycle shares of k_bnn (library built with -DNMX_BNN_PROF: scripts/ab_build.py
potential_bnn.hip bnnprof='-DNMX_BNN_PROF'): thread 0 of every workgroup adds its shader-clock
cycles per phase.  usage: python scripts/bnn_profile.py build/ab/bnnprof/libnumpyro_amd.so [chains]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numpyro_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

from numpyro_amd import datasets  # noqa: E402
from numpyro_amd.potentials import BNN  # noqa: E402

NAMES = ["params + data to LDS", "h1 = tanh(X W1)", "h2 = tanh(h1 W2) (MFMA)", "yhat, residual", "grad w3",
         "ga2 = gy w3 (1 - h2^2)", "grad W2 = h1^T ga2 (MFMA)", "ga1 = ga2 W2^T (MFMA)", "-",
         "grad W1 = X^T ga1", "block sums + U"]
C = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
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
lib = native.lib()
fn = lib.nmx_debug_bnn_profile
fn.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 16)()
for _ in range(3):
    pot.evaluate(ev, s)
torch.cuda.synchronize()
fn(buf)
for _ in range(20):
    pot.evaluate(ev, s)
torch.cuda.synchronize()
fn(buf)
tot = sum(buf[i] for i in range(11))
n = 20 * C
print(f"k_bnn C={C}: {tot / n:.0f} cycles per chain-evaluation (thread 0 of each workgroup)")
for i in range(11):
    if buf[i]:
        print(f"  {NAMES[i]:32s} {buf[i] / n:9.0f} cycles  {100.0 * buf[i] / tot:5.1f}%")
