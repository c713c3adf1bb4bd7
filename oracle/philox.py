"""ORACLE (test infrastructure only) — Philox4x32-10 restated in NumPy.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this.

The reference draws its randomness from JAX's threefry2x32 key-splitting tree
(numpyro/infer/hmc.py:102,472-474; numpyro/infer/hmc_util.py:804,920,1005,1161-1162);
no reference test pins PRNG values, so the sampler's stream is
"parity unpinned" by construction.  The engine instead uses a counter-based Philox
keyed by (seed, global chain id, iteration, event, index); this module is the CPU
restatement of that stream, pinned by the Random123 known-answer vectors
(tests/test_philox.py), and used by the oracle sampler so that GPU and CPU chains
consume identical random numbers.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)

EV_MOMENTUM = 1
EV_DIRECTION = 2
EV_BIASED = 3
EV_LEAF = 4
EV_INIT = 5
EV_ACCEPT = 6
EV_PREDICT = 7
EV_HEURISTIC = 8


def philox4x32_10(ctr, key):
    """ctr: (..., 4) uint32, key: (..., 2) uint32 -> (..., 4) uint32."""
    c = np.asarray(ctr, dtype=np.uint32).astype(np.uint64)
    k = np.asarray(key, dtype=np.uint32).copy()
    c0, c1, c2, c3 = c[..., 0], c[..., 1], c[..., 2], c[..., 3]
    k0 = k[..., 0].astype(np.uint32)
    k1 = k[..., 1].astype(np.uint32)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0
            p1 = M1 * c2
            hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
            hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
            n0 = hi1 ^ c1 ^ k0.astype(np.uint64)
            n1 = lo1
            n2 = hi0 ^ c3 ^ k1.astype(np.uint64)
            n3 = lo0
            c0, c1, c2, c3 = n0, n1, n2, n3
            k0 = (k0 + W0).astype(np.uint32)
            k1 = (k1 + W1).astype(np.uint32)
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def rng(seed: int, chain, it, event: int, idx, sub):
    """Philox block of one sampler event (mirrors nmx_rng in csrc/nmx_common.h)."""
    chain, it, idx, sub = np.broadcast_arrays(
        np.asarray(chain, np.uint64), np.asarray(it, np.uint64),
        np.asarray(idx, np.uint64), np.asarray(sub, np.uint64))
    c2 = (np.uint64(event) << np.uint64(24)) | (idx & np.uint64(0x00FFFFFF))
    ctr = np.stack([chain, it, c2, sub], axis=-1).astype(np.uint32)
    seed = int(seed)
    key = np.broadcast_to(np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], np.uint32),
                          ctr.shape[:-1] + (2,))
    return philox4x32_10(ctr, key)


def u01(x):
    """[0,1) float32 from the top 24 bits (exact)."""
    return ((np.asarray(x, np.uint32) >> np.uint32(8)).astype(np.float32)
            * np.float32(5.9604644775390625e-08))


def u01_open0(x):
    """(0,1] float32."""
    return (((np.asarray(x, np.uint32) >> np.uint32(8)).astype(np.float32) + np.float32(1.0))
            * np.float32(5.9604644775390625e-08))


def box_muller(a, b):
    u1 = u01_open0(a).astype(np.float64)
    u2 = u01(b).astype(np.float64)
    rad = np.sqrt(-2.0 * np.log(u1))
    ang = 2.0 * np.pi * u2
    return (rad * np.cos(ang)).astype(np.float32), (rad * np.sin(ang)).astype(np.float32)


def normals(seed, chain, it, dim):
    """Momentum noise for one chain/iteration: dim N(0,1) draws (4 per Philox block)."""
    nblk = (dim + 3) // 4
    out = rng(seed, chain, it, EV_MOMENTUM, np.arange(nblk), 0)
    n0, n1 = box_muller(out[:, 0], out[:, 1])
    n2, n3 = box_muller(out[:, 2], out[:, 3])
    eps = np.stack([n0, n1, n2, n3], axis=-1).reshape(-1)[:dim]
    return eps


def heuristic_normals(seed, chain, it, attempt, dim):
    """find_reasonable_step_size momentum noise of one attempt (csrc/nuts.hip k_heur_propose)."""
    nblk = (dim + 3) // 4
    out = rng(seed, chain, it, EV_HEURISTIC, np.arange(nblk), attempt)
    n0, n1 = box_muller(out[:, 0], out[:, 1])
    n2, n3 = box_muller(out[:, 2], out[:, 3])
    return np.stack([n0, n1, n2, n3], axis=-1).reshape(-1)[:dim]


def uniform(seed, chain, it, event, idx=0, sub=0):
    return u01(rng(seed, chain, it, event, idx, sub)[..., 0])


def init_uniform(seed, chain, attempt, dim, radius=2.0):
    """init_to_uniform(radius) draw in unconstrained space (numpyro/infer/initialization.py:95-129)."""
    nblk = (dim + 3) // 4
    out = rng(seed, chain, 0, EV_INIT, np.arange(nblk), attempt)
    u = u01(out).reshape(-1)[:dim]
    return (np.float32(2.0 * radius) * u - np.float32(radius)).astype(np.float32)
