"""Potential launch time with a compacted active list inside a wide batch (ldc = 4096), as in
the tail of a NUTS run, vs a dense batch of the same chains.
usage: python scripts/logreg_list_bench.py [counts] [lib]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import datasets, native
if len(sys.argv) > 2:
    native.LIB_PATH = os.path.abspath(sys.argv[2])
from numpyro_amd.potentials import LogisticRegression

counts = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,32,69,128,256,512").split(",")]
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
dev = torch.device("cuda:0")
LDC = 4096
pot = LogisticRegression(torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev))
pot.bind(LDC, LDC, dev)
rs = np.random.RandomState(0)
Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.05 * rs.randn(LDC, D)).astype(np.float32)
z = torch.from_numpy(Z.T.copy()).to(dev)
g = torch.zeros(D, LDC, device=dev); pe = torch.zeros(LDC, device=dev)
idx = torch.arange(LDC, dtype=torch.int32, device=dev)
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
s = native.stream_ptr()
for n in counts:
    cnt.fill_(n)
    # num_chains = the engine's bound on the list count (C - finished chains): the tight case
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(idx),
                          active_count=native.ptr(cnt), num_chains=n if os.environ.get("NO_HINT") is None else LDC,
                          ldc=LDC)
    for _ in range(3):
        pot.evaluate(ev, s)
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        pot.evaluate(ev, s)
    b.record(); b.synchronize()
    ms = a.elapsed_time(b) / 20
    print(f"active {n} of ldc {LDC}: {ms:.3f} ms/eval, "
          f"{4.0 * N * D * n / (ms * 1e-3) / 1e12:.1f} TFLOP/s", flush=True)
