"""Leaf-level parity: the device's per-leaf decision trace (nmx_nuts_config.trace,
Engine.set_trace) against the oracle's leaf records (oracle.hmc_ref.record_leaves) on the same
Philox stream, for every step schedule -- the fused step (dim < 257), the persistent wide
kernel (k_wide_persistent), the launched D-slice kernels and the chain-row dense step
(k_chain_step, BASELINE configs 2 and 3).

A chain whose tree size or draw leaves the oracle's is located at the first leaf where a
decision differs (oracle/parity.py): the parting must be a rounding flip there -- the shared
uniform between the two transition probabilities, with their difference within what the
leaf-energy discrepancy measured up to that leaf allows, or U-turn dots of opposite sign within
the measured dot rounding, or delta energies on either side of the divergence threshold.  Not
the closest decision anywhere in the transition: the decision at the parting leaf, with that
leaf's bound (hmc_util.py:984-1085 _iterative_build_subtree, :1088-1180 build_tree)."""
import numpy as np
import pytest
import torch

from numpyro_amd import datasets, native
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS
from oracle import hmc_ref as H
from oracle import parity as PR
from oracle import philox

pytestmark = pytest.mark.gpu


def _traced(o, s, T):
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


def _f32(pe_grad):
    return lambda z: tuple(np.asarray(v, np.float32) if np.ndim(v) else np.float32(v) for v in pe_grad(z))


def _as_trace(hist, L=1024):
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


def _report(par, label, cal=None, frac=None):
    """Every located parting explained at its leaf; with `cal` (the same comparison between the
    oracle and another float32 oracle) the device's spread must be of the calibration's order."""
    for m in par["mismatches"]:
        print(f"[{label}] " + PR.describe(m))
    print(f"[{label}] {par['matched']}/{par['chains']} chains reproduce the oracle over {par['transitions']} "
          f"chain-transitions; leaf-energy discrepancy on matched paths <= {par['max_dE_err']:.2e}")
    bad = [m for m in par["mismatches"] if not m["explained"] and m["kind"] != "draw"]
    assert not bad, f"[{label}] partings not explained by rounding at their leaf: {bad}"
    if cal is not None:
        ok, msg = PR.like_calibration(par, cal)
        print(f"[{label}] {msg}")
        assert ok, f"[{label}] {msg}"
    if frac is not None:
        assert par["matched"] >= int(frac * par["chains"])


def _oracle_runs(pe_grad, dim, C, T, seed, step, z0, **kw):
    hist = []
    for c in range(C):
        o = H.NUTSOracle(pe_grad, dim, 0, step_size=step, adapt_step_size=False, adapt_mass_matrix=False, **kw)
        zc = philox.init_uniform(seed, c, 0, dim) if z0 is None else z0[c]
        hist.append(_traced(o, o.init(zc, seed, c), T))
    return hist


def _second_f32(model, dim, ref):
    """Another float32 implementation of the model's potential (the calibration side): the
    NumPy float32 batch of oracle/batched.py where it exists, else float32 sums (the oracle's
    logistic regression at dtype float32, against which `ref` is taken in rounded float64)."""
    from oracle import batched as OB

    if model == "sv":
        b = OB.SVBatch(ref.returns if hasattr(ref, "returns") else datasets.sp500_synthetic(T=dim - 2))
    elif model == "funnel":
        b = OB.FunnelBatch(dim)
    elif model == "bnn":
        b = OB.BNNBatch(ref.X, ref.Y, ref.H)
    else:
        return None
    return lambda z: (lambda pe, g: (np.float32(pe[0]), g[0]))(*b(np.asarray(z, np.float32)[None]))


def _engine_fixed(model, dim, C, T, seed, k, trace=True, dense_matrix=None, max_tree_depth=10):
    from test_gpu_nuts import _fixed_step_case

    rs = np.random.RandomState(dim)
    args, fm, ref, site, extract, step, frac, z0 = _fixed_step_case(model, dim, rs)
    kw = dict(step_size=step, adapt_step_size=False, adapt_mass_matrix=False, max_tree_depth=max_tree_depth)
    if dense_matrix is not None:
        kw.update(dense_mass=True, inverse_mass_matrix=dense_matrix)
    eng = NUTS(fm, **kw).make_engine(C, args)
    ip = None if z0 is None else torch.from_numpy(z0[:C])
    eng.initialize(seed, 0, init_params=ip)
    if trace:
        eng.set_trace(k, 0, T)
    samples, fields, _ = eng.run(T, seed)
    ns = fields[:, native.COLLECT.index("num_steps"), :C].t().round().to(torch.int64).cpu().numpy()
    z = samples[:, :, :C].permute(2, 0, 1).to(torch.float64).cpu().numpy()  # [C, T, D] model space, constrained
    return eng, ref, step, frac, z0, ns, z, samples, fields


@pytest.mark.parametrize("model,dim", [("logreg", 40), ("sv", 302), ("funnel", 600), ("bnn", 321)])
def test_traced_fixed_step_parity(device, model, dim):
    """Fixed step, no adaptation: fused step (logreg D=40), persistent wide kernel (SV D=302,
    funnel D=600) and the launched D-slice schedule (BNN D=321); every parting located at its
    leaf and explained there."""
    seed, C, T = 77, 64, 3
    eng, ref, step, frac, z0, ns, z, _, _ = _engine_fixed(model, dim, C, T, seed, C)
    tr = eng.trace_records()
    if model == "logreg":  # the reference side in rounded float64, calibrated against float32 sums
        from oracle import potentials as OP
        ref32, ref = ref, OP.LogisticRegression(ref.X, ref.y, dtype=np.float64)
        second = _f32(ref32.pe_grad)
    else:
        second = _second_f32(model, dim, ref)
    hist = _oracle_runs(_f32(ref.pe_grad), dim, C, T, seed, step, z0)
    # the device collects constrained draws (ExpTransform sites): map the oracle's likewise
    pos = eng.model_potential.transform_codes().cpu().numpy().astype(bool)
    constrain = lambda zz: np.where(pos, np.exp(np.asarray(zz, np.float64)), zz)  # noqa: E731
    par = PR.compare_traced(hist, tr, ns, z, atol=1e-3, rtol=1e-3, to_model=constrain)
    # rounding calibration: the same comparison between the oracle and another float32 oracle
    ctr, cns, cz = _as_trace(_oracle_runs(second, dim, C, T, seed, step, z0))
    cal = PR.compare_traced(hist, ctr, cns, cz, atol=1e-3, rtol=1e-3)
    _report(par, f"traced {model} D={dim}", cal=cal)
    # a matched chain's leaves: every tree's length recorded, the last one ends the transition
    for c in range(C):
        for t in range(T):
            n = int(ns[c, t])
            assert np.all(np.isfinite(tr[t, c, :n, PR.T_FLAGS])) and np.all(np.isnan(tr[t, c, n:, PR.T_FLAGS]))
            assert int(tr[t, c, n - 1, PR.T_FLAGS]) & PR.TF_ITER_DONE


def test_trace_leaves_results_unchanged(device):
    """Recording the trace changes no draw or field (persistent wide and fused schedules)."""
    for model, dim in (("sv", 302), ("logreg", 40)):
        a = _engine_fixed(model, dim, 64, 2, 5, 64, trace=True)
        b = _engine_fixed(model, dim, 64, 2, 5, 64, trace=False)
        assert torch.equal(a[7], b[7]) and torch.equal(a[8], b[8])


def test_dense_chain_step_matches_oracle_dense_mass(device):
    """BASELINE configs 2-3's dense schedule (k_chain_step on the chain-row arena, whitening
    GEMMs k_gemm_x3 packing the listed chains' rows) against the oracle's dense-mass NUTS in model
    coordinates (momentum mass_matrix_sqrt @ eps, kinetic energy r.M^-1 r, U-turn dots with M^-1:
    hmc.py:92-110, hmc_util.py:1183-1220): funnel D = 600, a given dense matrix, fixed step."""
    seed, C, T, D = 31, 48, 3, 600
    rs = np.random.RandomState(1)
    a = rs.randn(D, D) / 60.0
    M = (a @ a.T + np.eye(D)).astype(np.float32)
    eng, ref, step, frac, _, ns, z, _, _ = _engine_fixed("funnel", D, C, T, seed, C, dense_matrix=M, max_tree_depth=7)
    assert eng.dense and eng.crow and not eng.chain_dense  # the k_chain_step schedule
    tr = eng.trace_records()
    kw = dict(dense_mass=True, inverse_mass_matrix=M, max_tree_depth=7)
    hist = _oracle_runs(_f32(ref.pe_grad), D, C, T, seed, step, None, **kw)
    par = PR.compare_traced(hist, tr, ns, z, atol=2e-3, rtol=2e-3)
    ctr, cns, cz = _as_trace(_oracle_runs(_second_f32("funnel", D, ref), D, C, T, seed, step, None, **kw))
    cal = PR.compare_traced(hist, ctr, cns, cz, atol=2e-3, rtol=2e-3)
    _report(par, "dense chain-row step funnel D=600", cal=cal)


def test_bnn_pooled_dense_config3_matches_oracle(device):
    """BASELINE config 3's workload (examples/bnn.py: D_X = 3, N = 100, H = 69, D = 5038) with
    dense_mass='pooled' on the k_chain_step schedule: device adaptation (W = 30: one middle window,
    the pooled matrix re-expressed at its end), then 2 traced sampling transitions of 16 chains.
    The oracle resumes each chain from the device's post-warmup state in the device's whitened
    coordinates (identity mass, the device's pooled T and mu teacher-forced: oracle/batched.py
    Whitened) on the same stream.  Trees of up to 1023 leapfrogs of a tanh network: f32 rounding
    grows along them, so chains may part -- each must part at a leaf where the decision is a
    rounding flip of that leaf."""
    from oracle import batched as OB
    from oracle import cpu_batched as CB

    Hh, C, W, T, k, seed = 69, 64, 30, 2, 16, 3
    X, Y = datasets.bnn_data(N=100, D_X=3)
    mcmc = MCMC(NUTS(P.bnn, dense_mass="pooled"), num_warmup=W, num_samples=T, num_chains=C,
                postprocess_fn=lambda z: z)
    mcmc.warmup(seed, X, Y, Hh)
    eng = mcmc._engine
    assert eng.dense and eng.crow and eng.D == 5038
    st = {n: eng.chain_state(n)[:k].detach().cpu().numpy().copy() for n in ("z", "zgrad", "pe", "step_size")}
    wt = eng.potential.whitening
    f = OB.Whitened(OB.BNNBatch(X, Y, Hh), wt.T.cpu().numpy(), wt.mu.cpu().numpy())
    eng.set_trace(k, eng.iteration, T)
    mcmc.run(seed + 1, X, Y, Hh, extra_fields=("num_steps",))
    ns = mcmc.get_extra_fields(group_by_chain=True)["num_steps"][:k].cpu().numpy()
    zdev = mcmc._samples[:, :, :k].permute(2, 0, 1).to(torch.float64).cpu().numpy()  # model space
    ones = np.ones_like(st["z"])
    states, oracles = CB.chains_from_state(st["z"], st["zgrad"], st["pe"], st["step_size"], ones, ones, W,
                                           seed + 1, W)
    _, hist, evals, _ = CB.run_chains(f, states, oracles, T, record=True)
    to_model = lambda w: f.to_model(np.asarray(w)[None])[0]  # noqa: E731
    par = PR.compare_traced(hist, eng.trace_records(), ns, zdev, atol=1e-3, rtol=1e-3, to_model=to_model)
    print(f"[bnn pooled dense D=5038] {evals} oracle leapfrogs, device trees {ns.tolist()}")
    # rounding calibration: the oracle in rounded float64 (network and whitening) from the same
    # states, against the float32 oracle the device was compared with
    f64 = OB.Whitened(OB.BNNBatch(X, Y, Hh, dtype=np.float64), wt.T.cpu().numpy(), wt.mu.cpu().numpy(),
                      dtype=np.float64)
    states, oracles = CB.chains_from_state(st["z"], st["zgrad"], st["pe"], st["step_size"], ones, ones, W,
                                           seed + 1, W)
    _, hist64, _, _ = CB.run_chains(f64, states, oracles, T, record=True)
    ctr, cns, cz = _as_trace(hist64)
    cal = PR.compare_traced(hist, ctr, cns, np.stack([[to_model(w) for w in cc] for cc in cz]), atol=1e-3,
                            rtol=1e-3, to_model=to_model)
    _report(par, "bnn pooled dense D=5038", cal=cal)
