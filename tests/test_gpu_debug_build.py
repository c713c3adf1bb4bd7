"""The debug build (numpyro_amd.build(debug=True): NMX_DCHECK bounds and invariant checks compiled
into every kernel, SURVEY.md §5 "race detection / sanitizers") runs each schedule -- fused step
with the covtype potential (full, tail and list forms), the launched wide step, the wide step
fused with a D-split model, the persistent one-wave schedule, per-chain and pooled dense mass,
the BNN -- in a subprocess (the library is loaded once per process) without a failed check."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import numpy as np, torch
from numpyro_amd import datasets, native
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS
assert native.LIB_PATH.endswith("libnumpyro_amd_debug.so"), native.LIB_PATH
native.lib()
rs = np.random.RandomState(0)

def run(model, args, C, W=30, S=10, **kw):
    m = MCMC(NUTS(model, **kw), num_warmup=W, num_samples=S, num_chains=C, progress_bar=False)
    m.run(1, *args, extra_fields=("num_steps",))
    ns = m.get_extra_fields()["num_steps"]
    assert int(ns.sum()) > 0
    return m

X = rs.randn(3000, 55).astype(np.float32)
y = (rs.rand(3000) < 0.4).astype(np.float32)
run(P.logistic_regression, (X, y), 300)                      # full + tail + list forms
run(P.diag_normal, (rs.randn(300).astype(np.float32), np.ones(300, np.float32)), 96)   # wide, launched
run(P.stochastic_volatility, (datasets.sp500_synthetic(T=400),), 96)                  # wide, fused model
run(P.eight_schools, (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y), 64)  # persistent
cov = np.eye(12) + 0.5
run(P.multivariate_normal, (None, cov), 64, dense_mass=True)   # per-chain dense
run(P.funnel, (300,), 64, dense_mass="pooled")                  # pooled dense, wide
Xb, Yb = datasets.bnn_data(N=30, D_X=3)
run(P.bnn, (Xb, Yb, 5), 64)
torch.cuda.synchronize()
# the mechanism itself: a violated check prints from the device (and only in this build)
assert native.lib().nmx_selftest_dcheck(7, native.stream_ptr()) == 1
torch.cuda.synchronize()
print("debug build ok")
"""


def test_debug_build_runs_every_schedule_without_a_failed_check():
    lib = os.path.join(ROOT, "numpyro_amd", "_lib", "libnumpyro_amd_debug.so")
    if not os.path.exists(lib):
        pytest.fail("debug library missing: run numpyro_amd.build(debug=True) (done by __graft_entry__.build())")
    env = dict(os.environ, NUMPYRO_AMD_DEBUG="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    fails = [ln for ln in out.splitlines() if "NMX_DCHECK failed" in ln]
    # exactly one: the probe's (no check failed in the runs above)
    assert len(fails) == 1 and "selftest.hip" in fails[0] and "value == 0" in fails[0], "\n".join(fails)[:3000]
    assert "debug build ok" in out
