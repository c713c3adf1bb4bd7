"""Predictive API checks that need no GPU (argument validation as numpy's
numpyro/infer/util.py:950-1015), and the oracle's predictive restatement against direct
formulas."""
import numpy as np
import pytest
import torch

from numpyro_amd import potentials as P
from numpyro_amd.infer import Predictive
from oracle import philox
from oracle import predictive as OPred


def test_predictive_argument_errors():
    with pytest.raises(ValueError):
        Predictive(P.logistic_regression)
    with pytest.raises(ValueError):
        Predictive(P.logistic_regression, {"coefs": torch.zeros(3, 2)}, guide=lambda: None)
    with pytest.raises(NotImplementedError):
        Predictive(P.logistic_regression, num_samples=10)  # prior predictive
    with pytest.raises(NotImplementedError):
        Predictive(P.diag_normal, {"x": torch.zeros(3, 9)})
    with pytest.raises(ValueError):
        Predictive(P.bnn, {"w1": torch.zeros(3, 2, 2), "w2": torch.zeros(4, 2, 2)})
    with pytest.warns(UserWarning):
        p = Predictive(P.logistic_regression, {"coefs": torch.zeros(5, 2)}, num_samples=7)
    assert p.num_samples == 5
    p = Predictive(P.logistic_regression, {"coefs": torch.zeros(2, 5, 3)}, batch_ndims=2)
    assert p.num_samples == 10 and p._batch_shape == (2, 5)


def test_oracle_predictive_streams():
    rs = np.random.RandomState(0)
    X = rs.randn(50, 4)
    coefs = rs.randn(3, 4)
    draws, p, u = OPred.predict_logreg(X, coefs, 9)
    assert draws.shape == (3, 50) and np.array_equal(draws, (u < p).astype(np.int32))
    w = philox.rng(9, 2, 0, philox.EV_PREDICT, 17, 0)
    assert u[2, 17] == philox.u01(w[0])
    loc = rs.randn(4, 6)
    scale = np.abs(rs.randn(6)) + 0.1
    y = OPred.predict_normal(loc, scale, 3)
    w = philox.rng(3, 1, 0, philox.EV_PREDICT, 5, 0)
    z, _ = philox.box_muller(w[0], w[1])
    np.testing.assert_allclose(y[1, 5], loc[1, 5] + scale[5] * float(z), rtol=1e-12)


def test_predictive_funnel_and_sv_sites():
    """examples/funnel.py:84-87: Predictive(reparam_model, samples, return_sites=["x", "y"])
    returns the deterministic x = exp(y / 2) x_decentered (reparam.py:140-142) and the given y;
    by default the deterministic site alone (util.py:870-877).  The centred funnel has neither an
    observed nor a deterministic site.  Stochastic volatility's observed r keeps its data (the
    returns also fix the series length, examples/stochastic_volatility.py:57-65)."""
    g = torch.Generator().manual_seed(0)
    xd, y = torch.randn(6, 9, generator=g), torch.randn(6, generator=g)
    out = Predictive(P.funnel_reparam, {"x_decentered": xd, "y": y}, return_sites=["x", "y"])(1, 10)
    torch.testing.assert_close(out["x"].cpu(), torch.exp(y / 2)[:, None] * xd)
    torch.testing.assert_close(out["y"].cpu(), y)
    out = Predictive(P.funnel_reparam, {"x_decentered": xd, "y": y})(1, 10)
    assert set(out) == {"x"}
    assert Predictive(P.funnel, {"x": xd, "y": y})(1, 10) == {}
    r = np.random.RandomState(1).randn(20).astype(np.float32)
    s = {"sigma": torch.rand(4, generator=g), "nu": torch.rand(4, generator=g) + 2, "s": torch.randn(4, 20, generator=g)}
    out = Predictive(P.stochastic_volatility, s)(2, r)
    assert out["r"].shape == (4, 20) and np.array_equal(out["r"][3].cpu().numpy(), r)
    with pytest.raises(ValueError, match="returns"):
        Predictive(P.stochastic_volatility, s)(2, None)
