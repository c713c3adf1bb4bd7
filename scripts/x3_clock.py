"""In-kernel clock of the covtype potential (MI355X_MICROARCH.md 'DVFS give-back' item 6): a
diagnostic build (-DNMX_X3_CLOCK, scripts/ab_build.py) stamps s_memtime / s_memrealtime around
k_logreg_x3's tile loop; after >= 3 s of back-to-back all-active launches on the synthetic covtype
data the clock is median(d memtime / d memrealtime) x 100 MHz over the last launch's workgroups.
usage: python scripts/x3_clock.py build/ab/clock/libnumpyro_amd.so [chains]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import datasets, native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
from numpyro_amd.potentials import LogisticRegression  # noqa: E402

C = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
dev = torch.device("cuda:0")
pot = LogisticRegression(torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev))
pot.bind(C, C, dev)
rs = np.random.RandomState(0)
Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.05 * rs.randn(C, D)).astype(np.float32)
z = torch.from_numpy(Z.T.copy()).to(dev)
g = torch.zeros(D, C, device=dev)
pe = torch.zeros(C, device=dev)
ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=C, ldc=C)
s = native.stream_ptr()
t_end = time.perf_counter() + 3.0
n = 0
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
while time.perf_counter() < t_end:
    for _ in range(20):
        pot.evaluate(ev, s)
    n += 20
    torch.cuda.synchronize()
a.record()
for _ in range(20):
    pot.evaluate(ev, s)
b.record()
b.synchronize()
ms = a.elapsed_time(b) / 20
host = (ctypes.c_ulonglong * (16384 * 2))()
native.lib().nmx_debug_x3_clock.restype = ctypes.c_int
native.check(native.lib().nmx_debug_x3_clock(host), "nmx_debug_x3_clock")
st = np.frombuffer(host, dtype=np.uint64).reshape(16384, 2).astype(np.float64)
ok = st[:, 1] > 0
ghz = st[ok, 0] / st[ok, 1] * 0.1
print(f"chains {C}: {n} warm launches, {ms:.3f} ms/launch (diagnostic build), {int(ok.sum())} workgroups stamped: "
      f"in-kernel clock median {np.median(ghz):.3f} GHz (p10 {np.percentile(ghz, 10):.3f}, p90 "
      f"{np.percentile(ghz, 90):.3f}); tile-loop real time median {np.median(st[ok, 1]) / 100:.1f} us")
