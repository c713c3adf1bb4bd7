"""Time the fused logreg potential alone (all chains active).
usage: python scripts/bench_potential.py [ignored] [chains,...] [libnumpyro_amd.so of an A/B build]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import datasets, native
from numpyro_amd.potentials import LogisticRegression

if len(sys.argv) > 3:
    native.LIB_PATH = os.path.abspath(sys.argv[3])
variants = ["d"]
chains = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "4096,1024").split(",")]
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
dev = torch.device("cuda:0")
Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
for C in chains:
    ldc = (C + 63) // 64 * 64
    pot = LogisticRegression(Xd, yd)
    pot.bind(C, ldc, dev)
    rs = np.random.RandomState(0)
    Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.05 * rs.randn(C, D)).astype(np.float32)
    z = torch.zeros(D, ldc, device=dev); z[:, :C] = torch.from_numpy(Z.T.copy()).to(dev)
    g = torch.zeros(D, ldc, device=dev); pe = torch.zeros(ldc, device=dev)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=C, ldc=ldc)
    ref = None
    for v in variants:
        s = native.stream_ptr()
        for _ in range(3):
            pot.evaluate(ev, s)
        torch.cuda.synchronize()
        n = 20
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            pot.evaluate(ev, s)
        b.record(); b.synchronize()
        ms = a.elapsed_time(b) / n
        tf = 4.0 * N * D * C / (ms * 1e-3) / 1e12
        cur = (pe[:C].cpu().numpy().astype(np.float64), g[:, :C].cpu().numpy().astype(np.float64))
        if ref is None:
            ref = cur; err = (0.0, 0.0)
        else:
            err = (np.max(np.abs(cur[0] - ref[0]) / np.abs(ref[0])), np.max(np.abs(cur[1] - ref[1])) / np.max(np.abs(ref[1])))
        print(f"C={C} variant={v} {ms:.3f} ms/eval  {tf:.1f} TFLOP/s  frac={tf/(2500.0/6):.3f}  rel-diff-vs-first pe={err[0]:.2e} g={err[1]:.2e}", flush=True)
