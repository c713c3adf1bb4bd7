"""Debug the split-bf16 logreg layout: packed fragments vs a NumPy restatement, and the
kernel on a small problem vs float64."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import native
from numpyro_amd.native import lib, ptr
from numpyro_amd.potentials import LogisticRegression


def bf16_rne(x):
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    return (r.astype(np.uint32) << 16).view(np.float32)


def split3(v):
    b1 = bf16_rne(v); e1 = (v - b1).astype(np.float32)
    b2 = bf16_rne(e1); e2 = (e1 - b2).astype(np.float32)
    return b1, b2, bf16_rne(e2)


def expected(X, y, D):
    N = X.shape[0]
    KB, DT = (D + 15) // 16, (D + 31) // 32
    NP = 3 * KB + 6 * DT + 1
    nt = (N + 31) // 32
    Xp = np.zeros((nt * 32, 64), np.float32); Xp[:N, :D] = X
    yp = np.zeros(nt * 32, np.float32); yp[:N] = y
    P = split3(Xp)
    out = np.zeros((nt, NP, 64, 8), np.float32)
    lane = np.arange(64); r = lane & 31; h = lane >> 5
    for t in range(nt):
        for p in range(3):
            for kb in range(KB):
                for j in range(8):
                    out[t, p * KB + kb, :, j] = P[p][32 * t + r, 16 * kb + 8 * h + j]
            for dt in range(DT):
                for s in range(2):
                    for j in range(8):
                        row = 32 * t + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)
                        out[t, 3 * KB + p * 2 * DT + 2 * dt + s, :, j] = P[p][row, 32 * dt + r]
    return out, nt, NP


dev = torch.device("cuda:0")
rs = np.random.RandomState(0)
cases = [(100, 55, 64), (1000, 55, 128), (5000, 20, 64)]
if len(sys.argv) > 1:
    cases = [tuple(int(v) for v in c.split("x")) for c in sys.argv[1].split(",")]
for N, D, C in cases:
    X = rs.randn(N, D).astype(np.float32); y = (rs.rand(N) < 0.4).astype(np.float32)
    pot = LogisticRegression(torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev))
    pot.bind(C, C, dev)
    nt = (N + 31) // 32; NP = 3 * ((D + 15) // 16) + 6 * ((D + 31) // 32) + 1
    exp = expected(X[:32 * 64], y[:32 * 64], D)[0] if N <= 20000 else None
    nb = lib().nmx_logreg_packed_bytes(N, D)
    raw = pot.packed.view(torch.uint8)[nb - nt * NP * 1024: nb].cpu().numpy()
    got = raw.view(np.uint16).reshape(nt, NP, 64, 8).astype(np.uint32) << 16
    got = got.view(np.float32)
    for t in range(min(nt, 64) if exp is not None else 0):
        for i in range(NP - 1):
            if not np.array_equal(got[t, i], exp[t, i]):
                print("N", N, "tile", t, "piece", i, "mismatch", np.abs(got[t, i] - exp[t, i]).max()); break
    ylab = raw.reshape(nt, NP, 1024)[:, NP - 1, :128].copy().view(np.float32).reshape(nt, 2, 16)
    for t in range(min(nt, 64)):
        for hh in range(2):
            for ii in range(16):
                row = 32 * t + (ii & 3) + 8 * (ii >> 2) + 4 * hh
                want = y[row] if row < N else 0.0
                if ylab[t, hh, ii] != want:
                    print("label mismatch", t, hh, ii, ylab[t, hh, ii], want)
    print(f"N={N} D={D}: layout checked ({nt} tiles x {NP} pieces)", flush=True)
    Z = (0.1 * rs.randn(C, D)).astype(np.float32)
    z = torch.from_numpy(Z.T.copy()).to(dev)
    g = torch.zeros_like(z); pe = torch.zeros(C, device=dev)
    ev = native.EvalBatch(z=ptr(z), grad=ptr(g), pe=ptr(pe), num_chains=C, ldc=C)
    for v in ("22", "30"):
        os.environ["NMX_LOGREG_VARIANT"] = v
        pot.evaluate(ev, native.stream_ptr()); torch.cuda.synchronize()
        L = X.astype(np.float64) @ Z.T.astype(np.float64)
        pe64 = (np.maximum(L, 0) + np.log1p(np.exp(-np.abs(L))) - y[:, None] * L).sum(0) + 0.5 * (Z.astype(np.float64) ** 2).sum(1) + 0.5 * np.log(2 * np.pi) * D
        g64 = X.T.astype(np.float64) @ (1 / (1 + np.exp(-L)) - y[:, None]) + Z.T
        gg = g.cpu().numpy(); pp = pe.cpu().numpy()
        print(f"  variant {v}: pe rel err {np.max(np.abs(pp - pe64) / np.abs(pe64)):.2e}  grad err {np.max(np.abs(gg - g64)) / np.abs(g64).max():.2e}",
              "pe[:3]", pp[:3], pe64[:3], "g[:3,0]", gg[:3, 0], g64[:3, 0], flush=True)
