"""Per-split partials of the split-bf16 logreg kernel vs NumPy (debug)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import native
from numpyro_amd.native import lib, ptr
from numpyro_amd.potentials import LogisticRegression

N, D, C = [int(v) for v in sys.argv[1].split("x")]
os.environ["NMX_LOGREG_VARIANT"] = sys.argv[2] if len(sys.argv) > 2 else "30"
dev = torch.device("cuda:0")
rs = np.random.RandomState(0)
X = rs.randn(N, D).astype(np.float32); y = (rs.rand(N) < 0.4).astype(np.float32)
pot = LogisticRegression(torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev))
pot.bind(C, C, dev)
Z = (0.1 * rs.randn(C, D)).astype(np.float32)
z = torch.from_numpy(Z.T.copy()).to(dev)
g = torch.zeros_like(z); pe = torch.zeros(C, device=dev)
ev = native.EvalBatch(z=ptr(z), grad=ptr(g), pe=ptr(pe), num_chains=C, ldc=C)
pot.evaluate(ev, native.stream_ptr()); torch.cuda.synchronize()
nt = (N + 31) // 32
s = nt // 16 // 8 * 8; S = min(max(s, 8), 256)
per = (nt + S - 1) // S
ws = pot.workspace
gb = S * D * C * 4
gpart = ws.view(torch.uint8)[:gb].view(torch.float32).reshape(S, D, C).cpu().numpy()
off = (gb + 255) // 256 * 256
pep = ws.view(torch.uint8)[off:off + S * C * 8].view(torch.float64).reshape(S, C).cpu().numpy()
L = X.astype(np.float64) @ Z.T.astype(np.float64)
R = 1 / (1 + np.exp(-L)) - y[:, None]
T = 0.5 * np.abs(L) + np.log1p(np.exp(-np.abs(L)))
bad = []
for sp in range(S):
    r0, r1 = min(sp * per * 32, N), min((sp + 1) * per * 32, N)
    ge = X[r0:r1].T.astype(np.float64) @ R[r0:r1]
    pad = max(0, min((sp + 1) * per, nt) * 32 - max(r1, r0)) if (sp + 1) * per >= nt else 0
    pe_e = T[r0:r1].sum(0) + pad * np.log(2)
    eg = np.abs(gpart[sp] - ge).max() / max(np.abs(ge).max(), 1e-6)
    ep = np.abs(pep[sp] - pe_e).max() / max(np.abs(pe_e).max(), 1e-6)
    wrong_chains = np.where(np.abs(gpart[sp] - ge).max(0) > 1e-3 * max(np.abs(ge).max(), 1))[0]
    if eg > 1e-4 or ep > 1e-4 or not np.isfinite(eg):
        bad.append(sp)
        print(f"split {sp}: rows {r0}-{r1} grad err {eg:.2e} pe err {ep:.2e} bad chains {wrong_chains[:8]}... ({len(wrong_chains)})")
print("S", S, "per", per, "bad splits", len(bad), bad[:40])
