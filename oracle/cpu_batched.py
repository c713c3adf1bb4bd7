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
import time

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
        self.pot_s = 0.0  # seconds inside the batched potential
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
                t0 = time.perf_counter()
                pe, g = self.f(Z)
                self.pot_s += time.perf_counter() - t0
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


def run_chains(pe_grad_batch, states, oracles, num_transitions, deadline=None, record=False, stats=None,
               min_transitions=0):
    """Advance every (oracle, state) pair by `num_transitions` transitions with batched
    potential evaluations.  `oracles[k]` must have been built with pe_grad = None; it is bound
    here.  With `deadline` (a time.perf_counter() value) a chain starts no further transition
    once it has passed (chains run on continuously until then, so the batch stays full: the
    CPU comparator's fixed-batch mode); every chain still runs at least `min_transitions` (the
    parity legs need that many transitions of every chain).  With `record`, every history entry is (state,
    decisions of that transition: (kind, margin) list, see hmc_ref.record_decisions, per-leaf
    records, see hmc_ref.record_leaves and oracle/parity.py).  `stats`
    (a dict) receives the seconds spent inside the batched potential ("pot_s").
    Returns (final states, per-chain list of states, potential evaluations, batched calls)."""
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
            for i in range(num_transitions):
                if deadline is not None and i >= min_transitions and time.perf_counter() >= deadline:
                    break
                log = [] if record else None
                leaves = [] if record else None
                H.record_decisions(log)
                H.record_leaves(leaves)
                st = o.sample(st)
                hist[k].append((st, log, leaves) if record else st)
            H.record_decisions(None)
            H.record_leaves(None)
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
    if stats is not None:
        stats["pot_s"] = b.pot_s
    return out, hist, b.evals, b.calls


def chains_from_state(z, grad, pe, step_size, inverse_mass, mass_sqrt, it0, seed, num_warmup, chain_offset=0):
    """Oracle chains resuming a device state (arrays [C, ...] of the first C chains: position,
    gradient, potential energy, adapted step size, diagonal inverse mass and its square root,
    transition index it0 >= num_warmup, i.e. sampling), on the device's Philox stream `seed`.
    Returns (states, oracles) for run_chains; the oracles' next transitions are the ones the
    device ran from that state (bench.py's cpu_baseline leg, tests/test_gpu_nuts.py)."""
    oracles, states = [], []
    D = z.shape[1]
    for c in range(z.shape[0]):
        o = H.NUTSOracle(None, D, num_warmup, step_size=float(step_size[c]), inverse_mass_matrix=inverse_mass[c])
        wa = o.wa_init((z[c],), None, np.float32(step_size[c]), inverse_mass_matrix=inverse_mass[c],
                       mass_matrix_size=D)
        # the device's own square root (the same formula; taken as is so nothing is recomputed)
        wa = wa._replace(mass_matrix_sqrt=np.asarray(mass_sqrt[c], np.float32))
        oracles.append(o)
        states.append(H.HMCState(int(it0), np.asarray(z[c], np.float32), np.asarray(grad[c], np.float32),
                                 np.float32(pe[c]), None, None, None, 0, np.float32(0), np.float32(0), False, wa,
                                 (seed, chain_offset + c)))
    return states, oracles
