"""Phase timing of the launched fused step (k_nuts_step) from an experiment build with
s_memtime stamps (scripts/ab_step_stamps_src.py): covtype NUTS, the last launch of a run.
usage: python scripts/step_stamps.py <lib> [chains] [steps]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
from numpyro_amd import datasets  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402

C = int(sys.argv[2]) if len(sys.argv) > 2 else 512
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
X, y = datasets.covtype_synthetic(seed=0)
Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
mcmc = MCMC(NUTS(P.logistic_regression), num_warmup=200, num_samples=K, num_chains=C, progress_bar=False)
mcmc.warmup(0, Xd, yd)
names = ["begin", "leaf rows", "vblock", "leaf+tree", "apply", "vblock2", "end"]


def show(tag):
    st = np.zeros((1024, 12), np.uint64)
    assert native.lib().nmx_x_step_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
    nb = (C + 15) // 16
    st = st[:nb].astype(np.float64)
    d = np.diff(st[:, :8], axis=1)
    leaf = st[:, 8] > 0  # the block evaluated a leaf in the recorded launch
    rt = (st[:, 11] - st[:, 10]) / 100.0
    clk = (st[:, 7] - st[:, 0]) / np.maximum(st[:, 11] - st[:, 10], 1) * 100e6 / 1e9
    span = (st[leaf, 11].max() - st[leaf, 10].min()) / 100.0 if leaf.any() else 0.0
    print(f"{tag}: blocks {nb}, with a leaf {int(leaf.sum())}; span {span:.1f} us; block wall us median {np.median(rt):.1f} "
          f"max {rt.max():.1f}; clock {np.median(clk):.2f} GHz")
    for sel, lab in ((leaf, "leaf blocks"), (~leaf, "other blocks")):
        if sel.any():
            m = d[sel].mean(0)
            print(f"  {lab:12s} cycles: " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, m)) +
                  f"  (total {m.sum():.0f})")


mcmc.run(1, Xd, yd)
show("after a 1-transition run (last launch)")
mcmc.post_warmup_state = mcmc.last_state
mcmc.num_samples = K
mcmc.run(2, Xd, yd)
show(f"after a {K}-transition run (last launch)")
