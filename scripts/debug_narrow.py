"""Narrow tail form vs the full kernel on one chain: per-split U partials and gradient slabs
(debugging aid).  usage: python scripts/debug_narrow.py [rows]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402
from numpyro_amd.potentials import LogisticRegression  # noqa: E402
from test_gpu_potentials import _eval, _eval_list  # noqa: E402

n_rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4001
dev = torch.device("cuda:0")
rs = np.random.RandomState(n_rows % 997)
X = rs.randn(n_rows, 55).astype(np.float32)
y = (rs.rand(n_rows) < 0.4).astype(np.float32)
Z = rs.randn(300, 55).astype(np.float32) * 0.05
pot = LogisticRegression(X, y)
S = native.lib().nmx_logreg_num_splits(n_rows)


def parts(C):
    ldc = (C + 63) // 64 * 64
    ws = pot.workspace
    gb = S * 55 * ldc * 4
    pe = ws[(gb + 255) // 256 * 256:].view(torch.float64)[:S * ldc].view(S, ldc)
    g = ws[:gb].view(torch.float32).view(S, 55, ldc)
    return pe.clone(), g.clone()


pe_a, g_a = _eval(pot, Z, dev)
pa, ga = parts(300)
for c in (0, 5):
    pe_b, g_b = _eval_list(pot, Z, [c], dev)
    pb, gb = parts(300)
    print(f"chain {c}: U full {pe_a[c]:.6f} narrow {pe_b[0]:.6f}; grad max diff {np.abs(g_a[c] - g_b[0]).max():.3g}")
    print("  U partial per split, full :", [f"{v:.4f}" for v in pa[:, c].tolist()])
    print("  U partial per split, narrow:", [f"{v:.4f}" for v in pb[:, 0].tolist()])
    print("  grad slab diff per split:", [f"{v:.3g}" for v in (ga[:, :, c] - gb[:, :, 0]).abs().amax(1).tolist()])
