"""Finalize phase stamps (experiment build): one chain listed, covtype-size rows."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
from numpyro_amd import datasets  # noqa: E402
from numpyro_amd.potentials import LogisticRegression  # noqa: E402

dev = torch.device("cuda:0")
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
pot = LogisticRegression(torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev))
LDC = 512
pot.bind(LDC, LDC, dev)
z = torch.zeros(D, LDC, device=dev)
g = torch.zeros(D, LDC, device=dev)
pe = torch.zeros(LDC, device=dev)
idx = torch.arange(LDC, dtype=torch.int32, device=dev)
cnt = torch.tensor([int(sys.argv[2]) if len(sys.argv) > 2 else 1], dtype=torch.int32, device=dev)
ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(idx),
                      active_count=native.ptr(cnt), num_chains=int(cnt.item()), ldc=LDC)
for _ in range(20):
    pot.evaluate(ev, native.stream_ptr())
torch.cuda.synchronize()
st = np.zeros((64, 4, 8), np.uint64)
assert native.lib().nmx_x_fin_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
st = st.astype(np.float64)
rows = [r for r in range(64) if st[r, 0, 0] > 0]
sums = np.array([[st[r, w, 1] - st[r, w, 0] for w in range(4)] for r in rows])
bar = np.array([[st[r, w, 2] - st[r, w, 1] for w in range(4)] for r in rows])
wall = np.array([(st[r, 0, 5] - st[r, 0, 4]) / 100 for r in rows])
span = (max(st[r, w, 5] for r in rows for w in range(4)) - min(st[r, w, 4] for r in rows for w in range(4))) / 100
slow = [(r, int(sums[i].max())) for i, r in enumerate(rows) if sums[i].max() > 2 * np.median(sums)]
print("slow blocks (row d, max wave cycles):", slow[:10])
print(f"blocks {len(rows)}: slot sums {sums.mean():.0f} cycles (max {sums.max():.0f}), barrier {bar.mean():.0f}; "
      f"block wall {wall.mean():.2f} us, span over blocks {span:.2f} us")
