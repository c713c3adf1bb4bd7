"""Debug: U terms of the narrow tail form along its pipeline (A wave -> split helper -> B wave)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
from numpyro_amd.potentials import LogisticRegression  # noqa: E402
from test_gpu_potentials import _eval_list  # noqa: E402

n_rows = 4001
rs = np.random.RandomState(n_rows % 997)
X = rs.randn(n_rows, 55).astype(np.float32)
y = (rs.rand(n_rows) < 0.4).astype(np.float32)
Z = rs.randn(300, 55).astype(np.float32) * 0.05
pot = LogisticRegression(X, y)
_eval_list(pot, Z, [0], torch.device("cuda:0"))
d = np.zeros((3, 8, 64, 64), np.uint64)
assert native.lib().nmx_x_dbg(d.ctypes.data_as(ctypes.c_void_p)) == 0
d = d.view(np.float64)
for wg in range(2):
    for i in range(16):
        print(wg, i, "A", d[0, wg, i, :3], "helper", d[1, wg, i, :3], "B", d[2, wg, i, :3])
