"""Per-iteration s_memtime stamps of the narrow tail form (experiment build only: the
stamped variant is generated from potential_logreg.hip into build/abx and never shipped).
usage: python scripts/narrow_stamps.py <lib> [N]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
from numpyro_amd.potentials import LogisticRegression  # noqa: E402

N = int(sys.argv[2]) if len(sys.argv) > 2 else 581012
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
cnt = torch.tensor([1], dtype=torch.int32, device=dev)
ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(idx),
                      active_count=native.ptr(cnt), num_chains=1, ldc=LDC)
s = native.stream_ptr()
for _ in range(20):
    pot.evaluate(ev, s)
torch.cuda.synchronize()
st = np.zeros((8, 8, 160, 4), np.uint64)
assert native.lib().nmx_x_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
st = st.astype(np.float64)
for wg in range(3):
    rt0, mt0 = st[wg, 0, 158, 0], st[wg, 0, 158, 1]
    rt1, mt1 = st[wg, 0, 159, 0], st[wg, 0, 159, 1]
    clk = (mt1 - mt0) / (rt1 - rt0) * 100e6
    print(f"WG {wg}: {(rt1 - rt0) / 100:.1f} us between the first and last stamps, clock {clk / 1e9:.2f} GHz")
    K = int(np.max(np.nonzero(st[wg, 0, :158, 3])[0])) + 1
    for w, name in ((0, "B0"), (1, "B1"), (2, "A0"), (3, "A1"), (4, "split4"), (5, "split5"), (6, "dma6"), (7, "dma7")):
        t = st[wg, w, 1:K - 1]
        bar = np.mean(t[:, 1] - t[:, 0])
        iss = np.mean(t[:, 2] - t[:, 1])
        work = np.mean(t[:, 3] - t[:, 2])
        it = np.mean(np.diff(st[wg, w, 1:K, 1]))
        print(f"  {name:6s} iterations {K}: cycles per iteration {it:7.0f} = barrier wait {bar:6.0f} + DMA issue "
              f"{iss:5.0f} + role work {work:6.0f}")
