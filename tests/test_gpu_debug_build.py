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


CARRY_SCRIPT = r"""
import os
import numpy as np, torch
from numpyro_amd import datasets, native
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS, HMC
assert native.LIB_PATH.endswith("libnumpyro_amd_debug.so"), native.LIB_PATH

def run(model, args, C, kernel=NUTS, sync=False, **kw):
    m = MCMC(kernel(model, **kw), num_warmup=30, num_samples=8, num_chains=C, progress_bar=False, sync_chains=sync)
    m.run(3, *args, extra_fields=("num_steps", "potential_energy"))
    ef = m.get_extra_fields(True)
    return ({k: v.cpu().numpy() for k, v in m.get_samples(True).items()},
            ef["num_steps"].cpu().numpy(), ef["potential_energy"].cpu().numpy(), m.last_run_stats["launches"])

cases = [("sv async", P.stochastic_volatility, (datasets.sp500_synthetic(T=400),), {}),
         ("sv lockstep", P.stochastic_volatility, (datasets.sp500_synthetic(T=400),), {"sync": True}),
         ("funnel hmc", P.funnel, (300,), {"kernel": HMC, "num_steps": 5})]
for name, model, args, kw in cases:
    os.environ.pop("NMX_PERSIST_CARRY", None)
    a = run(model, args, 48, **kw)
    os.environ["NMX_PERSIST_CARRY"] = "0"
    b = run(model, args, 48, **kw)
    assert a[3] > 0 and b[3] > 0
    for k in a[0]:
        np.testing.assert_array_equal(a[0][k], b[0][k], err_msg=name + " " + k)
    np.testing.assert_array_equal(a[1], b[1], err_msg=name)
    np.testing.assert_array_equal(a[2], b[2], err_msg=name)
    print(name, "bitwise equal:", int(a[1].sum()), "leapfrogs,", a[3], "launches")
print("carry ok")
"""


def test_persistent_lds_frontier_is_bitwise_the_arena_one():
    """k_wide_persistent keeps the chain's frontier (z_eval, g_eval, the moving end's momentum) in
    LDS when it fits (nuts.hip persist_carry); the debug build can turn that off
    (NMX_PERSIST_CARRY=0), and the draws, tree sizes and potential energies must not change: SV
    async (one launch per segment: the frontier loaded once and written back at the end), SV
    lockstep (one launch per transition: every transition crosses an exit and an entry) and HMC
    on the funnel (no tree: the leapfrog's frontier only)."""
    lib = os.path.join(ROOT, "numpyro_amd", "_lib", "libnumpyro_amd_debug.so")
    if not os.path.exists(lib):
        pytest.fail("debug library missing: run numpyro_amd.build(debug=True) (done by __graft_entry__.build())")
    env = dict(os.environ, NUMPYRO_AMD_DEBUG="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CARRY_SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=110)
    out = r.stdout + r.stderr
    print(out[-2000:])
    assert r.returncode == 0, out[-3000:]
    assert "carry ok" in out
    assert "NMX_DCHECK failed" not in out
