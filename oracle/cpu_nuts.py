"""ORACLE (test infrastructure only: bench.py's cpu_baseline legs and tests/) -- ctypes binding of
the C restatement of numpyro's NUTS sampling kernel with the benchmark models' potentials
(oracle/c/nuts_cpu.c): the CPU side of SURVEY.md §8d.  Chains resume a device state (sampling:
fixed step size, diagonal inverse mass; dense mass as identity-mass chains on whitened
coordinates with the device's T, mu) on the device's Philox stream, so they run the timed
workload's trees; tests/test_cpu_nuts.py pins the restatement against oracle/hmc_ref.py."""
from __future__ import annotations

import ctypes

import numpy as np

from . import build as _build

MODELS = {"covtype": 1, "funnel": 2, "sv": 3, "bnn": 4}


class _Model(ctypes.Structure):  # nmx_cpu_model
    _fields_ = [("model", ctypes.c_int), ("dim", ctypes.c_int), ("X", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("n", ctypes.c_long), ("bnn_dx", ctypes.c_int), ("bnn_h", ctypes.c_int), ("r2", ctypes.c_void_p),
                ("wT", ctypes.c_void_p), ("wmu", ctypes.c_void_p)]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _build.build()
        _LIB = ctypes.CDLL(_build.lib_path("nuts_cpu"))
        f = _LIB.nmx_cpu_nuts_run
        f.restype = ctypes.c_int
        vp = ctypes.c_void_p
        f.argtypes = [ctypes.POINTER(_Model), ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int,
                      ctypes.c_long, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_double, vp,
                      vp, vp, vp, vp]
        _LIB.nmx_cpu_threads.restype = ctypes.c_int
    return _LIB


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


class CpuNuts:
    """A model bound for the C sampler.  model: "covtype" (X [N, D], y [N]), "funnel" (dim),
    "sv" (returns [T]), "bnn" (X [N, Dx], Y [N], H); whitening=(T [D, D], mu [D]) for dense mass."""

    def __init__(self, model, *args, whitening=None):
        self.keep = []
        m = _Model()
        m.model = MODELS[model]
        if model == "covtype":
            X, y = _f32(args[0]), _f32(args[1])
            m.dim, m.X, m.y, m.n = X.shape[1], X.ctypes.data, y.ctypes.data, X.shape[0]
            self.keep += [X, y]
        elif model == "funnel":
            m.dim = int(args[0])
        elif model == "sv":
            r2 = _f32(np.asarray(args[0], np.float64).astype(np.float32) ** 2)
            m.dim, m.r2 = r2.shape[0] + 2, r2.ctypes.data
            self.keep.append(r2)
        elif model == "bnn":
            X, Y, H = _f32(args[0]), _f32(np.asarray(args[1]).reshape(-1)), int(args[2])
            m.n, m.bnn_dx, m.bnn_h = X.shape[0], X.shape[1], H
            m.dim = 1 + X.shape[1] * H + H * H + H
            m.X, m.y = X.ctypes.data, Y.ctypes.data
            self.keep += [X, Y]
        else:
            raise ValueError(model)
        if whitening is not None:
            T, mu = _f32(whitening[0]), _f32(whitening[1])
            m.wT, m.wmu = T.ctypes.data, mu.ctypes.data
            self.keep += [T, mu]
        self.m, self.dim = m, m.dim

    @staticmethod
    def threads():
        return int(lib().nmx_cpu_threads())

    def run(self, z, grad, pe, step_size, inv_mass, mass_sqrt, seed, it0, num_transitions, chain_offset=0,
            max_tree_depth=10, max_delta_energy=1000.0, min_transitions=None, seconds=1e30, keep_z=True,
            trace=False):
        """Chains [C] from a sampling state: z, grad [C, D], pe [C], step_size [C], inv_mass,
        mass_sqrt [C, D] (diagonal).  Returns {num_steps [C, T] (-1 past a chain's last), z [C, T,
        D] or None, done [C], leapfrogs, wall_s, potential_s, calls, trace}; with `trace` the
        per-leaf decision records in the device trace's layout [T, C, 2^depth, 8] (oracle/parity.py)."""
        C, D = np.shape(z)
        assert D == self.dim
        T = int(num_transitions)
        args = [_f32(z), _f32(grad), _f32(pe), _f32(step_size), _f32(inv_mass), _f32(mass_sqrt)]
        ns = np.empty((C, T), np.int32)
        zo = np.empty((C, T, D), np.float32) if keep_z else None
        done = np.empty(C, np.int32)
        st = np.empty(4, np.float64)
        tr = np.full((C, T, 1 << int(max_tree_depth), 8), np.nan, np.float32) if trace else None
        r = lib().nmx_cpu_nuts_run(ctypes.byref(self.m), C, *[a.ctypes.data for a in args], int(seed), int(it0),
                                   int(chain_offset), int(max_tree_depth), float(max_delta_energy), T,
                                   T if min_transitions is None else int(min_transitions), float(seconds),
                                   ns.ctypes.data, zo.ctypes.data if keep_z else None, done.ctypes.data,
                                   st.ctypes.data, tr.ctypes.data if trace else None)
        if r != 0:
            raise RuntimeError("nmx_cpu_nuts_run failed (bad arguments or allocation)")
        return {"num_steps": ns, "z": zo, "done": done, "leapfrogs": st[0], "wall_s": st[1], "potential_s": st[2],
                "calls": st[3], "trace": None if tr is None else np.ascontiguousarray(tr.transpose(1, 0, 2, 3))}
