"""ORACLE (test infrastructure only: bench.py's cpu_baseline legs of BASELINE configs 2-4 and
tests/) -- float32 potentials and gradients of the funnel, stochastic-volatility and BNN
models batched over chains in NumPy (the products on multithreaded BLAS), and the dense-mass
whitening around any of them.  They restate oracle/potentials.py (float64, one chain; pinned
against scipy.stats and finite differences in tests/test_oracle_potentials.py) for a batch
Z [B, D] -> (U [B], grad [B, D]), so that oracle/cpu_batched.run_chains can drive many of the
oracle's NUTS chains with one potential call per round: the CPU side of SURVEY.md §8d.

`dtype=np.float64` computes the same expressions in float64 (outputs rounded to float32): the
rounding reference of the parity calibration (oracle/parity.py), against which the float32
batch is "another float32 implementation" like the device.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import digamma, gammaln

F = np.float32
LOG_2PI = math.log(2 * math.pi)


class FunnelBatch:
    """examples/funnel.py:44-46 (centred), z = (x[K], y): U = y^2/18 + log(3 sqrt(2 pi))
    + sum_i [x_i^2 e^-y / 2 + y/2 + log(2 pi)/2] (Normal.log_prob, continuous.py:2200-2204)."""

    def __init__(self, dim, dtype=np.float32):
        self.dim, self.K = dim, dim - 1
        self.F = dtype

    def __call__(self, Z):
        F = self.F
        Z = np.asarray(Z, F)
        x, y = Z[:, :-1], Z[:, -1]
        e = np.exp(-y)
        xx = np.einsum("bk,bk->b", x, x)
        pe = y * y / F(18) + F(math.log(3.0) + 0.5 * LOG_2PI) + F(0.5) * e * xx + F(self.K) * (
            F(0.5) * y + F(0.5 * LOG_2PI))
        G = np.empty_like(Z)
        G[:, :-1] = x * e[:, None]
        G[:, -1] = y / F(9) + F(0.5 * self.K) - F(0.5) * e * xx
        return pe.astype(np.float32), G.astype(np.float32)


class SVBatch:
    """examples/stochastic_volatility.py:57-65, z = (log nu, s[T], log sigma): Exponential
    (continuous.py:473-475) + GaussianRandomWalk (:684-690) + StudentT (:2373-2384) with the
    ExpTransform log-Jacobians; gradient as oracle/potentials.py StochasticVolatility."""

    def __init__(self, returns, dtype=np.float32):
        self.F = dtype
        self.r2 = np.asarray(returns, np.float64).astype(dtype) ** 2
        self.T = self.r2.shape[0]
        self.dim = self.T + 2

    def __call__(self, Z):
        F = self.F
        Z = np.asarray(Z, F)
        a, s, b = Z[:, 0], Z[:, 1:-1], Z[:, -1]
        nu, sigma = np.exp(a), np.exp(b)
        T = self.T
        d = np.diff(s, axis=1, prepend=F(0))
        dd = np.einsum("bt,bt->b", d, d)
        q = self.r2[None, :] * np.exp(F(-2) * s) / nu[:, None]
        l1q = np.log1p(q)
        lg = (gammaln(F(0.5) * nu) - gammaln(F(0.5) * (nu + F(1)))).astype(F)
        lp = F(math.log(50.0)) - F(50) * sigma + b
        lp = lp - F(0.5) * dd / (sigma * sigma) - F(T) * b - F(0.5 * T * LOG_2PI)
        lp = lp + F(math.log(0.1)) - F(0.1) * nu + a
        lp = lp - F(0.5) * (nu + F(1)) * l1q.sum(1) - s.sum(1) - F(T) * (
            F(0.5) * a + F(0.5 * math.log(math.pi)) + lg)
        qq = q / (F(1) + q)
        d_next = np.concatenate([d[:, 1:], np.zeros((Z.shape[0], 1), F)], axis=1)
        gs = -(d - d_next) / (sigma * sigma)[:, None] + (nu + F(1))[:, None] * qq - F(1)
        gb = F(-50) * sigma + F(1) + dd / (sigma * sigma) - F(T)
        dg = (digamma(F(0.5) * (nu + F(1))) - digamma(F(0.5) * nu)).astype(F)
        ga = nu * (F(-0.1) + (-F(0.5) * l1q).sum(1) + F(0.5) * (nu + F(1)) / nu * qq.sum(1)
                   + F(T) * (-F(0.5) / nu + F(0.5) * dg)) + F(1)
        G = np.empty_like(Z)
        G[:, 0], G[:, 1:-1], G[:, -1] = -ga, -gs, -gb
        return (-lp).astype(np.float32), G.astype(np.float32)


class BNNBatch:
    """examples/bnn.py:43-74, z = (log prec, w1 [Dx, H], w2 [H, H], w3 [H, 1]): N(0, 1) weights,
    Gamma(3, 1) precision (continuous.py:515-524) + log-Jacobian, Y ~ N(tanh(tanh(X w1) w2) w3,
    1 / sqrt(prec)); the backward pass of oracle/potentials.py BNN over a batch of networks
    (batched matmuls)."""

    def __init__(self, X, Y, H, dtype=np.float32):
        self.F = dtype
        self.X = np.asarray(X, dtype)
        self.Y = np.asarray(Y, dtype).reshape(-1)
        self.N, self.Dx = self.X.shape
        self.H = int(H)
        self.dim = 1 + self.Dx * self.H + self.H * self.H + self.H

    def __call__(self, Z):
        F = self.F
        Z = np.asarray(Z, F)
        B, H, Dx, N = Z.shape[0], self.H, self.Dx, self.N
        u = Z[:, 0]
        o = 1
        w1 = Z[:, o:o + Dx * H].reshape(B, Dx, H); o += Dx * H
        w2 = Z[:, o:o + H * H].reshape(B, H, H); o += H * H
        w3 = Z[:, o:o + H].reshape(B, H, 1)
        p = np.exp(u)
        h1 = np.tanh(np.matmul(self.X[None], w1))           # [B, N, H]
        h2 = np.tanh(np.matmul(h1, w2))                      # [B, N, H]
        yhat = np.matmul(h2, w3)[:, :, 0]                    # [B, N]
        e = self.Y[None, :] - yhat
        ee = np.einsum("bn,bn->b", e, e)
        ww = np.einsum("bd,bd->b", Z[:, 1:], Z[:, 1:])
        lp = -F(0.5) * ww - F(0.5 * (self.dim - 1) * LOG_2PI)
        lp = lp + F(2) * u - p - F(gammaln(3.0)) + u
        lp = lp - F(0.5) * p * ee + F(0.5 * N) * u - F(0.5 * N * LOG_2PI)
        g_y = (-p[:, None] * e)[:, :, None]                  # dU / d yhat  [B, N, 1]
        gw3 = w3 + np.matmul(h2.transpose(0, 2, 1), g_y)
        ga2 = np.matmul(g_y, w3.transpose(0, 2, 1)) * (F(1) - h2 * h2)
        gw2 = w2 + np.matmul(h1.transpose(0, 2, 1), ga2)
        ga1 = np.matmul(ga2, w2.transpose(0, 2, 1)) * (F(1) - h1 * h1)
        gw1 = w1 + np.matmul(self.X.T[None], ga1)
        gu = -(F(3) - p + F(0.5 * N) - F(0.5) * p * ee)
        G = np.concatenate([gu[:, None], gw1.reshape(B, -1), gw2.reshape(B, -1), gw3.reshape(B, -1)], axis=1)
        return (-lp).astype(np.float32), G.astype(np.float32)


class Whitened:
    """Dense mass by whitening (numpyro_amd/dense.py): U_w(w) = U(mu + T w), grad_w = T^T
    grad_z, with T T^T = M^-1 -- dense-mass NUTS on z is identity-mass NUTS on w exactly
    (hmc.py:92-110, hmc_util.py:1183-1220).  The two products per call are [B, D] x [D, D]
    float32 GEMMs."""

    def __init__(self, base, T, mu, dtype=np.float32):
        self.base = base
        self.F = dtype
        self.Tt = np.ascontiguousarray(np.asarray(T, np.float64).T.astype(dtype))  # z = mu + w @ T^T
        self.T = np.ascontiguousarray(np.asarray(T, np.float64).astype(dtype))
        self.mu = np.asarray(mu, dtype)
        self.dim = base.dim

    def to_model(self, W):
        return self.mu[None, :] + np.asarray(W, self.F) @ self.Tt

    def __call__(self, W):
        # dtype float64 with a float64 base: the rounding reference of the parity calibration
        # (oracle/parity.py) -- positions, model and gradient product in float64, results rounded
        pe, G = self.base(self.to_model(W))
        return pe, (np.asarray(G, self.F) @ self.T).astype(np.float32)
