"""Tail-launch potential time vs row count (is the narrow / role-split form bound by where X
lives?): LogisticRegression on random N x 55 data, a compacted list of `n` chains in a 4096-wide
batch, 30 timed evaluations.  usage: python scripts/tail_rows_bench.py N [n] [lib]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402

if len(sys.argv) > 3:
    native.LIB_PATH = os.path.abspath(sys.argv[3])
from numpyro_amd.potentials import LogisticRegression  # noqa: E402

N = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda:0")
rs = np.random.RandomState(0)
X = torch.from_numpy(rs.randn(N, 55).astype(np.float32)).to(dev)
y = torch.from_numpy((rs.rand(N) < 0.4).astype(np.float32)).to(dev)
LDC = 4096
pot = LogisticRegression(X, y)
pot.bind(LDC, LDC, dev)
z = torch.from_numpy(0.05 * rs.randn(55, LDC).astype(np.float32)).to(dev)
g = torch.zeros(55, LDC, device=dev)
pe = torch.zeros(LDC, device=dev)
idx = torch.arange(LDC, dtype=torch.int32, device=dev)
cnt = torch.tensor([n], dtype=torch.int32, device=dev)
ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(idx),
                      active_count=native.ptr(cnt), num_chains=n, ldc=LDC)
s = native.stream_ptr()
for _ in range(3):
    pot.evaluate(ev, s)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(30):
    pot.evaluate(ev, s)
b.record()
b.synchronize()
ms = a.elapsed_time(b) / 30
S = native.lib().nmx_logreg_num_splits(N)
nt = (N + 31) // 32
print(f"N {N} n {n} splits {S} tiles/split {-(-nt // S)} eval {ms * 1e3:.1f} us "
      f"({ms * 1e3 / -(-nt // S):.2f} us per tile of a split)", flush=True)
