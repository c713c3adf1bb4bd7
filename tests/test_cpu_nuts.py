"""The C restatement of the NUTS sampling kernel (oracle/c/nuts_cpu.c, the CPU baseline of
bench.py) against the NumPy oracle (oracle/hmc_ref.py) on the same Philox stream: chains
resumed from the same sampling state take the same trees and draws up to float32 rounding (the C
potentials are float32 arithmetic with double reductions, the oracle's the rounded float64
expressions), for every benchmark model and for dense mass as whitened identity-mass chains."""
import numpy as np
import pytest

from oracle import batched as OB
from oracle import cpu_batched as CB
from oracle import cpu_nuts as CN
from oracle import potentials as OP


def _case(model, rs):
    if model == "covtype":
        X = rs.randn(3000, 8).astype(np.float32)
        X[:, -1] = 1.0
        beta = rs.randn(8) * 0.5
        y = (rs.rand(3000) < 1 / (1 + np.exp(-X @ beta))).astype(np.float32)
        r64 = OP.LogisticRegression(X.astype(np.float64), y.astype(np.float64), dtype=np.float64)
        f = lambda Z: tuple(np.asarray(v, np.float32) for v in r64.pe_grad_batch(Z))  # noqa: E731
        z0 = (beta + 0.02 * rs.randn(16, 8)).astype(np.float32)
        return CN.CpuNuts("covtype", X, y), f, z0, 0.02
    if model == "funnel":
        b = OB.FunnelBatch(40, dtype=np.float64)
        z0 = (0.5 * rs.randn(16, 40)).astype(np.float32)
        return CN.CpuNuts("funnel", 40), b, z0, 0.1
    if model == "sv":
        from numpyro_amd import datasets
        r = datasets.sp500_synthetic(T=60)
        b = OB.SVBatch(r, dtype=np.float64)
        z0 = np.concatenate([np.full((16, 1), 2.0), np.log(np.abs(r) + 1e-2)[None].repeat(16, 0)
                             + 0.1 * rs.randn(16, 60), np.full((16, 1), -3.0)], 1).astype(np.float32)
        return CN.CpuNuts("sv", r), b, z0, 0.01
    if model == "bnn":
        from numpyro_amd import datasets
        X, Y = datasets.bnn_data(N=30, D_X=3)
        b = OB.BNNBatch(X, Y, 5, dtype=np.float64)
        z0 = (0.3 * rs.randn(16, b.dim)).astype(np.float32)
        z0[:, 0] = 1.0
        return CN.CpuNuts("bnn", X, Y, 5), b, z0, 0.01
    if model == "funnel_dense":
        D = 30
        a = rs.randn(D, D) / 10
        T = np.linalg.cholesky(a @ a.T + np.eye(D)).T.astype(np.float32)  # upper triangular, like the device's
        mu = (0.1 * rs.randn(D)).astype(np.float32)
        b = OB.Whitened(OB.FunnelBatch(D, dtype=np.float64), T, mu, dtype=np.float64)
        z0 = (0.3 * rs.randn(16, D)).astype(np.float32)
        return CN.CpuNuts("funnel", D, whitening=(T, mu)), b, z0, 0.05
    raise ValueError(model)


@pytest.mark.parametrize("model", ["covtype", "funnel", "sv", "bnn", "funnel_dense"])
def test_c_nuts_matches_oracle(model):
    rs = np.random.RandomState(5)
    cn, f64, z0, step = _case(model, rs)
    C, D = z0.shape
    T, seed, it0 = 3, 1234, 50
    pe0, g0 = f64(z0)
    ss = np.full(C, step, np.float32)
    im = (0.5 + rs.rand(C, D)).astype(np.float32) if model != "funnel_dense" else np.ones((C, D), np.float32)
    msq = (1.0 / np.sqrt(im)).astype(np.float32)
    # the BNN's tanh network amplifies rounding along trees of 255-1023 leapfrogs: shorter trees
    md = 6 if model == "bnn" else 10
    out = cn.run(z0, g0, pe0, ss, im, msq, seed, it0, T, chain_offset=7, max_tree_depth=md)
    states, oracles = CB.chains_from_state(z0, g0, pe0, ss, im, msq, it0, seed, 10, chain_offset=7)
    for o in oracles:
        o.max_treedepth = (md, md)
    _, hist, evals, _ = CB.run_chains(f64, states, oracles, T)
    assert int(out["leapfrogs"]) > 0 and np.all(out["done"] == T)
    match, exact_trees = 0, 0
    for c in range(C):
        ns = np.array([s.num_steps for s in hist[c]])
        zs = np.stack([s.z for s in hist[c]])
        exact_trees += int(np.array_equal(ns, out["num_steps"][c]))
        if np.array_equal(ns, out["num_steps"][c]) and np.allclose(zs, out["z"][c], rtol=1e-3, atol=1e-4):
            match += 1
    print(f"[C NUTS {model}] {match}/{C} chains take the oracle's trees and draws over {T} transitions "
          f"({int(out['leapfrogs'])} C leapfrogs, {evals} oracle)")
    assert match >= int(0.8 * C), (match, out["num_steps"], [[s.num_steps for s in h] for h in hist])


def test_c_nuts_deadline_and_min_transitions():
    rs = np.random.RandomState(1)
    cn, f64, z0, step = _case("funnel", rs)
    C, D = z0.shape
    pe0, g0 = f64(z0)
    one = np.ones((C, D), np.float32)
    out = cn.run(z0, g0, pe0, np.full(C, step, np.float32), one, one, 3, 0, 50, min_transitions=2, seconds=0.0)
    assert np.all(out["done"] == 2) and np.all(out["num_steps"][:, 2:] == -1) and np.all(out["num_steps"][:, :2] > 0)
    assert out["leapfrogs"] == out["num_steps"][:, :2].sum()


@pytest.mark.parametrize("model", ["funnel", "sv", "funnel_dense"])
def test_c_nuts_trace_matches_oracle_leaf_records(model):
    """The C sampler's per-leaf decision trace (the device trace's layout) against the oracle's leaf
    records (oracle.hmc_ref.record_leaves) on the same chains: every leaf of every matched chain
    takes the same decisions (oracle/parity.py locate finds no parting), its delta energy agrees to
    float32 rounding; the trace can stand in for a second float32 oracle in a calibration."""
    from oracle import parity as PR

    rs = np.random.RandomState(5)
    cn, f64, z0, step = _case(model, rs)
    C, D = z0.shape
    T, seed, it0 = 3, 99, 20
    pe0, g0 = f64(z0)
    one = np.ones((C, D), np.float32)
    ss = np.full(C, step, np.float32)
    out = cn.run(z0, g0, pe0, ss, one, one, seed, it0, T, trace=True)
    states, oracles = CB.chains_from_state(z0, g0, pe0, ss, one, one, it0, seed, 10)
    _, hist, _, _ = CB.run_chains(f64, states, oracles, T, record=True)
    par = PR.compare_traced(hist, out["trace"], out["num_steps"], out["z"].astype(np.float64), atol=1e-4, rtol=1e-3)
    for m in par["mismatches"]:
        print(PR.describe(m))
    assert par["matched"] >= C - 2 and all(m["explained"] or m["kind"] == "draw" for m in par["mismatches"])
    for c in range(C):
        for t in range(T):
            n = int(out["num_steps"][c, t])
            tr = out["trace"][t, c]
            assert np.all(np.isfinite(tr[:n, PR.T_FLAGS])) and np.all(np.isnan(tr[n:, PR.T_FLAGS]))
            assert int(tr[n - 1, PR.T_FLAGS]) & PR.TF_ITER_DONE
    assert par["max_dE_rel"] < 1e-5
