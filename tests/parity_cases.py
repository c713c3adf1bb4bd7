"""Shared parity machinery of the GPU tests (imported by tests/test_gpu_*.py; no tests here).

A device run and the oracle (oracle/hmc_ref.py) take the same transitions on the same Philox
stream.  The comparison is leaf-located (oracle/parity.py): a chain that leaves the reference's
path is checked at the first leaf where a decision differs, with that leaf's own bound, and a
draw that differs while every decision agrees is checked against a rounding calibration.

* reference: the oracle with the potential in rounded float64 -- the most accurate float32 NUTS;
* calibration: the same chains under a second float32 implementation of the potential (float32
  sums, or oracle/batched.py's NumPy batch) against that reference: how far rounding alone moves
  a float32 implementation;
* device: the engine's draws, tree sizes and per-leaf decision trace (Engine.set_trace) against
  the same reference; `report` requires every parting explained at its leaf, every draw within
  DRAW_MULT x the calibration's drift, and the whole record of the calibration's order
  (oracle/parity.py like_calibration).
"""
from __future__ import annotations

import numpy as np
import torch

from numpyro_amd import datasets, native
from numpyro_amd import potentials as P
from numpyro_amd.infer import HMC, NUTS
from oracle import hmc_ref as H
from oracle import parity as PR
from oracle import philox
from oracle import potentials as OP


def f32(pe_grad):
    """A potential's outputs rounded to float32 (the oracle's NUTS runs in float32)."""
    return lambda z: tuple(np.asarray(v, np.float32) if np.ndim(v) else np.float32(v) for v in pe_grad(z))


def fixed_step_case(model, dim, rs):
    """(model args, fused model, oracle potential, checked site, oracle-z extractor, step, min
    match, shared initial points or None for init_to_uniform)."""
    if model == "logreg":
        X = rs.randn(300, dim).astype(np.float32)
        beta = rs.randn(dim) * 0.5 / np.sqrt(dim)
        y = (rs.rand(300) < 1 / (1 + np.exp(-X @ beta))).astype(np.float32)
        return (X, y), P.logistic_regression, OP.LogisticRegression(X, y, dtype=np.float32), "coefs", \
            (lambda z: z), 0.02, 0.95, None
    if model == "diag_normal":
        mu = rs.randn(dim).astype(np.float32)
        sd = (0.5 + rs.rand(dim)).astype(np.float32)
        return (mu, sd), P.diag_normal, OP.IsoNormal(mu, sd, dtype=np.float32), "x", (lambda z: z), 0.05, 0.95, None
    if model == "funnel":
        return (dim,), P.funnel, OP.Funnel(dim, dtype=np.float32), "x", (lambda z: z[..., :-1]), 0.05, 0.9, None
    if model == "sv":
        r = datasets.sp500_synthetic(T=dim - 2)
        return (r,), P.stochastic_volatility, OP.StochasticVolatility(r, dtype=np.float32), "s", \
            (lambda z: z[..., 1:-1]), 0.005, 0.9, None
    if model == "bnn":
        # D = 5038 is BASELINE config 3 (examples/bnn.py: D_X = 3, N = 100, H = 69)
        H_ = {46: 5, 321: 16, 5038: 69}[dim]
        X, Y = datasets.bnn_data(N=100 if H_ == 69 else 30, D_X=3)
        o = 1 + 3 * H_
        # shared well-conditioned start (small weights, prec ~ e): from U(-2, 2) the tanh
        # layers saturate and |U| ~ 1e3, where fp32 energy rounding flips leaf choices; the
        # hidden-to-hidden weights scale with 1/sqrt(H) so the second layer stays unsaturated
        z0 = (0.3 * rs.randn(64, dim)).astype(np.float32)
        z0[:, o:] *= np.float32(min(1.0, np.sqrt(5.0 / H_)))
        z0[:, 0] = 1.0
        return (X, Y, H_), P.bnn, OP.BNN(X, Y, H_, dtype=np.float32), "w2", \
            (lambda z: z[..., o:o + H_ * H_]), 0.01, 0.9, z0
    raise ValueError(model)


def second_f32(model, dim, ref):
    """Another float32 implementation of the model's potential (the calibration side): the
    NumPy float32 batch of oracle/batched.py where it exists, else float32 arithmetic of the
    oracle's own expressions."""
    from oracle import batched as OB

    if model == "sv":
        b = OB.SVBatch(ref.returns if hasattr(ref, "returns") else datasets.sp500_synthetic(T=dim - 2))
    elif model == "funnel":
        b = OB.FunnelBatch(dim)
    elif model == "bnn":
        b = OB.BNNBatch(ref.X, ref.Y, ref.H)
    elif model == "logreg":
        return f32(OP.LogisticRegression(ref.X, ref.y, dtype=np.float32).pe_grad)
    elif model == "diag_normal":
        mu, sd = ref.mu.astype(np.float32), ref.sd.astype(np.float32)

        def pe_grad(z):
            d = (np.asarray(z, np.float32) - mu) / sd
            return np.float32(np.float32(0.5) * np.dot(d, d)), (d / sd).astype(np.float32)
        return pe_grad
    else:
        raise ValueError(model)
    return lambda z: (lambda pe, g: (np.float32(pe[0]), g[0]))(*b(np.asarray(z, np.float32)[None]))


def reference_f64(model, ref):
    """The reference potential: the oracle's expressions in float64, rounded to float32."""
    if model == "logreg":
        return f32(OP.LogisticRegression(ref.X, ref.y, dtype=np.float64).pe_grad)
    return f32(ref.pe_grad)  # the other oracle potentials compute in float64 and round


def traced(o, s, T):
    """T oracle transitions from state s with their decision logs and leaf records."""
    hist = []
    for _ in range(T):
        log, leaves = [], []
        H.record_decisions(log)
        H.record_leaves(leaves)
        try:
            s = o.sample(s)
        finally:
            H.record_decisions(None)
            H.record_leaves(None)
        hist.append((s, log, leaves))
    return hist


def oracle_runs(pe_grad, dim, C, T, seed, step, z0, algo="NUTS", **kw):
    """Fixed-step oracle chains from init_to_uniform (or the shared z0), traced."""
    hist = []
    for c in range(C):
        o = H.NUTSOracle(pe_grad, dim, 0, algo=algo, step_size=step, adapt_step_size=False,
                         adapt_mass_matrix=False, **kw)
        zc = philox.init_uniform(seed, c, 0, dim) if z0 is None else z0[c]
        hist.append(traced(o, o.init(zc, seed, c), T))
    return hist


def as_trace(hist, L=1024):
    """An oracle run in the device's trace layout (oracle/parity.py oracle_to_trace): the second
    side of a calibration comparison.  Returns (trace [T, C, L, 8], num_steps [C, T], z [C, T, D])."""
    C, T = len(hist), min(len(h) for h in hist)
    tr = np.full((T, C, L, 8), np.nan, np.float32)
    ns = np.zeros((C, T), np.int64)
    z = np.zeros((C, T, np.size(hist[0][0][0].z)))
    for c, h in enumerate(hist):
        for t in range(T):
            st, _, leaves = h[t]
            tr[t, c] = PR.oracle_to_trace(leaves, L)
            ns[c, t] = st.num_steps
            z[c, t] = st.z
    return tr, ns, z


def report(par, label, cal=None, frac=None):
    """Every located parting explained at its leaf, every draw mismatch bounded by the
    calibration's drift (without a calibration a draw mismatch fails), and with `cal` the whole
    record of the calibration's order; prints each parting and the drift statistics."""
    if cal is not None:
        PR.bound_draws(par, cal)
    for m in par["mismatches"]:
        print(f"[{label}] " + PR.describe(m))
    if cal is not None:
        for m in cal["mismatches"]:
            print(f"[{label}] calibration: " + PR.describe(m))
        for m in cal.get("partings_after_draw", []):
            print(f"[{label}] calibration: chain {m['chain']}: after its draw, parts at transition {m['transition']} "
                  f"leaf {m['leaf']} on {m['kind']} ({'rounding flip' if m['explained'] else 'NOT explained'})")
    w = par["worst_dE"]
    print(f"[{label}] {par['matched']}/{par['chains']} chains reproduce the reference over {par['transitions']} "
          f"chain-transitions; leaf-energy discrepancy <= {par['max_dE_err']:.2e} (relative {par['max_dE_rel']:.2e}"
          + ("" if w is None else f", at chain {w['chain']} transition {w['transition']} leaf {w['leaf']}: dE "
             f"{w['dev']:.6g} vs {w['oracle']:.6g}, U {w['pe']:.6g}") + ")")
    bad = [m for m in par["mismatches"] if not m["explained"]]
    assert not bad, f"[{label}] partings not explained by rounding: {[PR.describe(m) for m in bad]}"
    if cal is not None:
        ok, msg = PR.like_calibration(par, cal)
        print(f"[{label}] {msg}")
        assert ok, f"[{label}] {msg}"
    if frac is not None:
        assert par["matched"] >= int(frac * par["chains"]), f"[{label}] {par['matched']}/{par['chains']} matched"


def engine_fixed(model, dim, C, T, seed, k, trace=True, dense_matrix=None, max_tree_depth=10, algo="NUTS",
                 **extra):
    """A fixed-step engine run of the case (trace of the first k chains on): (engine, oracle
    potential, step, min match, z0, num_steps [C, T], draws [C, T, D] (model space,
    constrained), samples, fields)."""
    rs = np.random.RandomState(dim)
    args, fm, ref, site, extract, step, frac, z0 = fixed_step_case(model, dim, rs)
    kw = dict(step_size=step, adapt_step_size=False, adapt_mass_matrix=False, **extra)
    if algo == "NUTS":
        kw["max_tree_depth"] = max_tree_depth
    if dense_matrix is not None:
        kw.update(dense_mass=True, inverse_mass_matrix=dense_matrix)
    eng = (NUTS if algo == "NUTS" else HMC)(fm, **kw).make_engine(C, args)
    ip = None if z0 is None else torch.from_numpy(z0[:C])
    eng.initialize(seed, 0, init_params=ip)
    if trace:
        eng.set_trace(k, 0, T)
    samples, fields, _ = eng.run(T, seed)
    ns = fields[:, native.COLLECT.index("num_steps"), :C].t().round().to(torch.int64).cpu().numpy()
    z = samples[:, :, :C].permute(2, 0, 1).to(torch.float64).cpu().numpy()  # [C, T, D] model space, constrained
    return eng, ref, step, frac, z0, ns, z, samples, fields


def constrain_fn(eng):
    """The device collects constrained draws (ExpTransform sites): map oracle draws likewise."""
    pos = eng.model_potential.transform_codes().cpu().numpy().astype(bool)
    return lambda zz: np.where(pos, np.exp(np.asarray(zz, np.float64)), zz)
