"""Generate tests/golden/diagnostics.npz from the REFERENCE's own numpyro/diagnostics.py.

Run in the build container only (it reads /root/reference, which does not exist on the GPU
box); the committed .npz is the fixture the tests use.  numpyro/diagnostics.py is plain
NumPy except for `jax.device_get` and `jax.tree.map/flatten` in summary(); those three are
provided here by a stand-in `jax` module of identity/dict helpers (nothing of jax's
arithmetic is involved).  The module is loaded by file path so numpyro/__init__.py (which
needs real jax) is never imported.

    python tests/golden/make_diagnostics_golden.py [/root/reference]
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference_diagnostics(ref_root):
    jax = types.ModuleType("jax")
    jax.device_get = lambda x: x
    tree = types.SimpleNamespace(
        map=lambda f, t: {k: f(v) for k, v in t.items()} if isinstance(t, dict) else f(t),
        flatten=lambda t: (list(t.values()) if isinstance(t, dict) else [t], None))
    jax.tree = tree
    saved = sys.modules.get("jax")
    sys.modules["jax"] = jax
    try:
        path = os.path.join(ref_root, "numpyro", "diagnostics.py")
        spec = importlib.util.spec_from_file_location("_ref_diagnostics", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        if saved is None:
            sys.modules.pop("jax", None)
        else:
            sys.modules["jax"] = saved
    return mod


def cases():
    """Seeded inputs: iid, AR(1), shifted chains, odd lengths, a multi-dim site, one chain."""
    rs = np.random.RandomState(20240601)
    out = {}
    out["iid"] = rs.randn(4, 1000)
    ar = np.zeros((3, 1501))
    e = rs.randn(3, 1501)
    for t in range(1, 1501):
        ar[:, t] = 0.8 * ar[:, t - 1] + e[:, t]
    out["ar1"] = ar
    sh = rs.randn(4, 200)
    sh[2:] += 1.5
    out["shifted"] = sh
    out["odd"] = rs.randn(5, 37) * np.array([1.0, 2.0, 0.5, 1.0, 3.0])[:, None]
    out["site3d"] = rs.standard_t(5, size=(2, 300, 3, 2))
    out["one_chain"] = rs.randn(1, 400)
    return out


def main():
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    ref = load_reference_diagnostics(ref_root)
    arrays = {}
    for name, x in cases().items():
        arrays[f"{name}/x"] = x
        arrays[f"{name}/ess"] = np.asarray(ref.effective_sample_size(x))
        if x.shape[0] >= 2:
            arrays[f"{name}/gelman_rubin"] = np.asarray(ref.gelman_rubin(x))
        arrays[f"{name}/split_gelman_rubin"] = np.asarray(ref.split_gelman_rubin(x))
        flat = x.reshape((-1,) + x.shape[2:])
        arrays[f"{name}/hpdi90"] = np.asarray(ref.hpdi(flat, prob=0.9, axis=0))
        arrays[f"{name}/hpdi50"] = np.asarray(ref.hpdi(flat, prob=0.5, axis=0))
        arrays[f"{name}/autocorrelation"] = np.asarray(ref.autocorrelation(x[0], axis=0))
        arrays[f"{name}/autocovariance_unbiased"] = np.asarray(ref.autocovariance(x[0], axis=0, bias=False))
        s = ref.summary({"v": x}, prob=0.9, group_by_chain=True)["v"]
        for k, v in s.items():
            arrays[f"{name}/summary/{k}"] = np.asarray(v)
    dst = os.path.join(HERE, "diagnostics.npz")
    np.savez_compressed(dst, **arrays)
    print(f"wrote {dst}: {len(arrays)} arrays")


if __name__ == "__main__":
    main()
