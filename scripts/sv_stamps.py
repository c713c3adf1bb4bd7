"""Per-phase cycles of the persistent SV kernel from the stamped experiment build
(scripts/ab_sv_stamps_src.py): the config-4 run of scripts/bench_configs.py, then the phase totals
of the last k_wide_persistent launch, per workgroup, as seen by wave 0 (which runs the scalar
logic) and wave 1 (rows only).
usage: python scripts/sv_stamps.py LIB [chains] [warmup] [steps]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

from numpyro_amd import datasets, native  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
import bench_configs as BC  # noqa: E402

C = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
W = int(sys.argv[3]) if len(sys.argv) > 3 else 200
S = int(sys.argv[4]) if len(sys.argv) > 4 else 10
NPH = 12
NAMES = ["loop top (prev. iteration tail)", "leaf rows + wave sums", "U-turn checkpoint levels",
         "barrier: every wave's rows", "finish: scalar-site rows (wave 0)", "scalar NUTS logic (wave 0)",
         "barrier: decisions published", "apply rows", "barrier: rows written",
         "(of the finish) sums + fin()", "(of apply) take_leaf leaves", "(count) take_leaf leaves"]
r = datasets.sp500_synthetic()
BC.run_model("stochastic_volatility", P.stochastic_volatility, (r,), C, W, S, bytes_per_leapfrog=2 * (r.size + 2) * 4)
buf = np.zeros((8192, 2, NPH + 2), np.uint64)
assert native.lib().nmx_x_sv_stamps(ctypes.c_void_p(buf.ctypes.data)) == 0
n = min(C, 8192)
for w, nm in ((0, "wave 0"), (1, "wave 1")):
    acc = buf[:n, w, :NPH].astype(np.float64)
    nit = buf[:n, w, NPH].astype(np.float64)
    nleaf = buf[:n, w, NPH + 1].astype(np.float64)
    ok = nleaf > 0
    tot = acc[ok][:, :10].sum(axis=1)
    print(f"{nm}: {int(ok.sum())} workgroups, median {np.median(nit[ok]):.0f} iterations / "
          f"{np.median(nleaf[ok]):.0f} leaves per launch, median {np.median(tot / nleaf[ok]):.0f} cycles per leaf")
    per = np.median(acc[ok] / nleaf[ok, None], axis=0)
    for i in range(10):
        print(f"  {NAMES[i]:34s} {per[i]:8.0f} cycles/leaf {100 * per[i] / per[:10].sum():5.1f}%")
    tl = buf[:n, w, 11].astype(np.float64)
    ok2 = ok & (tl > 0) & (nleaf > tl)
    a_tl = np.median(acc[ok2, 10] / tl[ok2])
    a_other = np.median((acc[ok2, 7] - acc[ok2, 10]) / (nleaf[ok2] - tl[ok2]))
    print(f"  apply rows per leaf: take_leaf {a_tl:.0f} cycles, other leaves {a_other:.0f}; "
          f"take_leaf fraction {np.median(tl[ok2] / nleaf[ok2]):.2f}")
