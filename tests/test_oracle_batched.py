"""The chain-batched float32 potentials of the CPU comparator (oracle/batched.py) against the
float64 one-chain oracle potentials (oracle/potentials.py, themselves pinned against scipy and
finite differences), and the whitening identity of the dense-mass path."""
import numpy as np

from numpyro_amd import datasets
from oracle import batched as B
from oracle import potentials as OP


def _check(batch, ref, Z, rtol_pe=2e-5, rtol_g=1e-4):
    pe, G = batch(Z)
    assert pe.dtype == np.float32 and G.dtype == np.float32 and G.shape == Z.shape
    for b in range(Z.shape[0]):
        p, g = ref.pe_grad(Z[b].astype(np.float64))
        np.testing.assert_allclose(pe[b], p, rtol=rtol_pe, atol=1e-3)
        np.testing.assert_allclose(G[b], g, rtol=rtol_g, atol=rtol_g * np.abs(g).max())


def test_funnel_batch():
    rs = np.random.RandomState(0)
    Z = rs.randn(5, 300).astype(np.float32)
    Z[:, -1] *= 2.0
    _check(B.FunnelBatch(300), OP.Funnel(300), Z)


def test_sv_batch():
    r = datasets.sp500_synthetic(T=200)
    rs = np.random.RandomState(1)
    Z = np.concatenate([rs.randn(4, 1) * 0.3 + 2.0, np.cumsum(0.05 * rs.randn(4, 200), 1) - 4.0,
                        rs.randn(4, 1) * 0.3 - 3.0], axis=1).astype(np.float32)
    _check(B.SVBatch(r), OP.StochasticVolatility(r), Z)


def test_bnn_batch():
    X, Y = datasets.bnn_data(N=50, D_X=3)
    H = 7
    ref = OP.BNN(X, Y, H)
    Z = (0.5 * np.random.RandomState(2).randn(6, ref.dim)).astype(np.float32)
    _check(B.BNNBatch(X, Y, H), ref, Z)


def test_whitened_is_the_dense_change_of_variables():
    """U_w(w) = U(mu + T w), grad_w = T^T grad U: finite differences of U_w match grad_w."""
    rs = np.random.RandomState(3)
    D = 30
    A = rs.randn(D, D)
    T = np.triu(np.linalg.cholesky(A @ A.T / D + np.eye(D)).T)
    mu = rs.randn(D)
    f = B.Whitened(B.FunnelBatch(D), T, mu)
    W = (0.3 * rs.randn(2, D)).astype(np.float32)
    pe, G = f(W)
    ref = OP.Funnel(D)
    for b in range(2):
        p, g = ref.pe_grad(mu + T @ W[b].astype(np.float64))
        np.testing.assert_allclose(pe[b], p, rtol=1e-5)
        np.testing.assert_allclose(G[b], T.T @ g, rtol=1e-4, atol=1e-4 * np.abs(T.T @ g).max())
