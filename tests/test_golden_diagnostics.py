"""Diagnostics against golden vectors produced by the reference's own numpyro/diagnostics.py
(tests/golden/make_diagnostics_golden.py; fixture tests/golden/diagnostics.npz).  Checks the
host implementation (numpyro_amd.diagnostics) and the rank-reduced one (numpyro_amd.shard, one
process here; the gloo world-2 test in test_shard.py ties it to the same numbers)."""
import os

import numpy as np
import pytest
import torch

from numpyro_amd import diagnostics as D
from numpyro_amd import shard

GOLDEN = np.load(os.path.join(os.path.dirname(__file__), "golden", "diagnostics.npz"))
CASES = sorted({k.split("/")[0] for k in GOLDEN.files})
RTOL = 1e-10  # float64 end to end; FFT length and reduction order match the reference


def g(case, key):
    return GOLDEN[f"{case}/{key}"]


@pytest.mark.parametrize("case", CASES)
def test_host_diagnostics_match_reference(case):
    x = g(case, "x")
    np.testing.assert_allclose(D.effective_sample_size(x), g(case, "ess"), rtol=RTOL)
    np.testing.assert_allclose(D.split_gelman_rubin(x), g(case, "split_gelman_rubin"), rtol=RTOL)
    if x.shape[0] >= 2:
        np.testing.assert_allclose(D.gelman_rubin(x), g(case, "gelman_rubin"), rtol=RTOL)
    flat = x.reshape((-1,) + x.shape[2:])
    np.testing.assert_array_equal(D.hpdi(flat, prob=0.9, axis=0), g(case, "hpdi90"))
    np.testing.assert_array_equal(D.hpdi(flat, prob=0.5, axis=0), g(case, "hpdi50"))
    np.testing.assert_allclose(D.autocorrelation(x[0], axis=0), g(case, "autocorrelation"), rtol=RTOL, atol=1e-14)
    np.testing.assert_allclose(D.autocovariance(x[0], axis=0, bias=False), g(case, "autocovariance_unbiased"),
                               rtol=RTOL, atol=1e-14)


@pytest.mark.parametrize("case", CASES)
def test_host_summary_matches_reference(case):
    s = D.summary({"v": g(case, "x")}, prob=0.9)["v"]
    keys = [k.split("/")[-1] for k in GOLDEN.files if k.startswith(f"{case}/summary/")]
    assert sorted(s.keys()) == sorted(keys)
    for k in keys:
        np.testing.assert_allclose(np.asarray(s[k]), g(case, f"summary/{k}"), rtol=RTOL, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("case", CASES)
def test_rank_reduced_diagnostics_match_reference(case):
    x = torch.as_tensor(g(case, "x"))
    np.testing.assert_allclose(shard.effective_sample_size(x).numpy(), g(case, "ess"), rtol=1e-9)
    np.testing.assert_allclose(shard.split_gelman_rubin(x).numpy(), g(case, "split_gelman_rubin"), rtol=1e-9)
    s = shard.summary({"v": x}, prob=0.9)["v"]
    for k in ("mean", "std", "median", "5.0%", "95.0%", "n_eff", "r_hat"):
        np.testing.assert_allclose(np.asarray(s[k]), g(case, f"summary/{k}"), rtol=1e-9, atol=1e-12, err_msg=k)
