"""Accuracy (vs a float64 evaluation on the GPU) and speed of logreg kernel variants at the
covtype shape.  usage: python scripts/logreg_variant_check.py 22,30 [chains=4096,1024,256]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import datasets, native
from numpyro_amd.potentials import LogisticRegression

variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["22", "30"]
chains = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "4096,1024,256").split(",")]
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
dev = torch.device("cuda:0")
Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
X64, y64 = Xd.double(), yd.double()
pot = None
for C in chains:
    ldc = (C + 63) // 64 * 64
    pot = LogisticRegression(Xd, yd)
    pot.bind(C, ldc, dev)
    rs = np.random.RandomState(0)
    Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.05 * rs.randn(C, D)).astype(np.float32)
    z = torch.zeros(D, ldc, device=dev); z[:, :C] = torch.from_numpy(Z.T.copy()).to(dev)
    g = torch.zeros(D, ldc, device=dev); pe = torch.zeros(ldc, device=dev)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=C, ldc=ldc)
    nref = min(C, 128)
    z64 = z[:, :nref].double()
    L = X64 @ z64
    pe64 = (torch.clamp(L, min=0) + torch.log1p(torch.exp(-L.abs())) - y64[:, None] * L).sum(0)
    pe64 += 0.5 * (z64 * z64).sum(0) + 0.5 * np.log(2 * np.pi) * D
    g64 = X64.T @ (torch.sigmoid(L) - y64[:, None]) + z64
    del L
    for v in variants:
        os.environ["NMX_LOGREG_VARIANT"] = v
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
        pe_err = ((pe[:nref].double() - pe64).abs() / pe64.abs()).max().item()
        gerr = ((g[:, :nref].double() - g64).abs().amax(0) / g64.abs().amax(0)).max().item()
        gmed = ((g[:, :nref].double() - g64).abs().amax(0) / g64.abs().amax(0)).median().item()
        print(f"C={C} variant={v} {ms:.3f} ms/eval {tf:.1f} TFLOP/s  vs f64: pe max rel {pe_err:.2e}  "
              f"grad max|err|/max|g| worst {gerr:.2e} median {gmed:.2e}", flush=True)
