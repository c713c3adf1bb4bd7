"""ORACLE (test infrastructure only: tests/ and bench.py's cpu_baseline leg) -- many chains of
the oracle's NUTS (oracle/hmc_ref.py) advanced together so that their potential
evaluations are batched into one call.

Each chain runs `NUTSOracle.sample` in its own Python thread; its `pe_grad(z)` blocks until
every chain still running has asked for an evaluation (or finished its transitions), then
one batched call evaluates them all.  Chains proceed independently (a chain whose tree ends
early starts its next transition), like the device engine's per-chain schedule; the batch
shrinks as chains finish.  A chain's trajectory is the oracle's own: the batching changes
only who computes the potential (tests/test_cpu_baseline.py checks this bitwise against
independent oracle chains).

`LogRegBatch` binds the batched C restatement of the covtype potential
(oracle/c/logreg_batch.c, OpenMP) -- the CPU comparator of bench.py.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import build as _build
from . import hmc_ref as H


class LogRegBatch:
    """pe_grad over a batch of chains: Z [B, D] -> (pe [B], grad [B, D]), float32, OpenMP."""

    def __init__(self, X, y):
        _build.build()
        self.lib = ctypes.CDLL(_build.lib_path("logreg_batch"))
        f = self.lib.nmx_cpu_logreg_pe_grad
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p,
                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        self.lib.nmx_cpu_threads.restype = ctypes.c_int
        self.X = np.ascontiguousarray(X, np.float32)
        self.y = np.ascontiguousarray(y, np.float32)
        self.N, self.D = self.X.shape

    def threads(self) -> int:
        return int(self.lib.nmx_cpu_threads())

    def __call__(self, Z):
        Z = np.asarray(Z, np.float32)
        B = Z.shape[0]
        Zt = np.ascontiguousarray(Z.T)
        pe = np.empty(B, np.float32)
        Gt = np.empty((self.D, B), np.float32)
        self.lib.nmx_cpu_logreg_pe_grad(self.X.ctypes.data, self.y.ctypes.data, self.N, self.D, Zt.ctypes.data, B,
                                        pe.ctypes.data, Gt.ctypes.data)
        return pe, np.ascontiguousarray(Gt.T)


class _Batcher:
    def __init__(self, pe_grad_batch, n):
        self.f = pe_grad_batch
        self.cv = threading.Condition()
        self.alive = n
        self.req = {}
        self.res = {}
        self.evals = 0
        self.calls = 0
        self.error = None

    def pe_grad(self, k, z):
        with self.cv:
            self.req[k] = z
            self.cv.notify_all()
            while k not in self.res and self.error is None:
                self.cv.wait()
            if self.error is not None:
                raise RuntimeError("batched evaluation failed") from self.error
            return self.res.pop(k)

    def done(self):
        with self.cv:
            self.alive -= 1
            self.cv.notify_all()

    def serve(self):
        while True:
            with self.cv:
                while self.alive > 0 and (len(self.req) < self.alive or not self.req):
                    self.cv.wait()
                if self.alive == 0:
                    return
                keys = sorted(self.req)
                Z = np.stack([self.req.pop(k) for k in keys])
            try:
                pe, g = self.f(Z)
            except Exception as e:  # noqa: BLE001  (propagated to every waiting chain)
                with self.cv:
                    self.error = e
                    self.cv.notify_all()
                raise
            with self.cv:
                for i, k in enumerate(keys):
                    self.res[k] = (np.float32(pe[i]), np.asarray(g[i], np.float32))
                self.evals += len(keys)
                self.calls += 1
                self.cv.notify_all()


def run_chains(pe_grad_batch, states, oracles, num_transitions):
    """Advance every (oracle, state) pair by `num_transitions` transitions with batched
    potential evaluations.  `oracles[k]` must have been built with pe_grad = None; it is bound
    here.  Returns (final states, per-chain list of states, potential evaluations, batched calls)."""
    n = len(states)
    b = _Batcher(pe_grad_batch, n)
    out = [None] * n
    hist = [[] for _ in range(n)]
    errs = []

    def work(k):
        try:
            o = oracles[k]
            fn = (lambda z, k=k: b.pe_grad(k, z))
            o.pe_grad = fn
            o.vv_init, o.vv_update = H.velocity_verlet(fn)
            st = states[k]
            for _ in range(num_transitions):
                st = o.sample(st)
                hist[k].append(st)
            out[k] = st
        except Exception as e:  # noqa: BLE001
            errs.append(e)
        finally:
            b.done()

    threads = [threading.Thread(target=work, args=(k,), daemon=True) for k in range(n)]
    for t in threads:
        t.start()
    b.serve()
    for t in threads:
        t.join()
    if errs:
        raise errs[0]
    return out, hist, b.evals, b.calls
