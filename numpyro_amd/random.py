"""PRNG keys.  The reference passes ``jax.random.PRNGKey(seed)`` (a uint32[2]); here a key
is the 64-bit Philox seed of csrc/nmx_common.h.  Any of: int, PRNGKey(seed), a length-2
uint32 array (JAX key layout, [hi, lo]) is accepted by MCMC.run."""
from __future__ import annotations

import numpy as np


def PRNGKey(seed: int):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed >> 32, seed & 0xFFFFFFFF], dtype=np.uint32)


def key_to_seed(key) -> int:
    if isinstance(key, (int, np.integer)):
        return int(key) & 0xFFFFFFFFFFFFFFFF
    a = np.asarray(key if not hasattr(key, "cpu") else key.cpu().numpy())
    if a.ndim == 0:
        return int(a) & 0xFFFFFFFFFFFFFFFF
    a = a.reshape(-1, a.shape[-1])[0] if a.ndim > 1 else a
    if a.size != 2:
        raise ValueError("a PRNG key is an int or a length-2 uint32 array")
    a = a.astype(np.uint64)
    return int((a[0] << np.uint64(32)) | a[1])


def split(key, num: int = 2):
    """Derive `num` independent keys (SplitMix64 over the seed)."""
    s = key_to_seed(key)
    out = []
    for i in range(num):
        z = (s + 0x9E3779B97F4A7C15 * (i + 1)) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out.append(PRNGKey(z))
    return np.stack(out)
