"""The CPU comparator of bench.py (CPU side 2): the batched C restatement of
the covtype potential (oracle/c/logreg_batch.c) against the float64 oracle, and the batched
multi-chain driver (oracle/cpu_batched.py) against independent oracle chains, bitwise."""
import numpy as np

from oracle import cpu_batched as CB
from oracle import hmc_ref as H
from oracle import philox
from oracle import potentials as OP


def _data(N=3000, D=55, seed=0):
    rs = np.random.RandomState(seed)
    X = rs.randn(N, D).astype(np.float32)
    beta = rs.randn(D) * 0.3
    y = (rs.rand(N) < 1 / (1 + np.exp(-X @ beta))).astype(np.float32)
    return X, y


def test_logreg_batch_matches_fp64():
    X, y = _data()
    Z = (0.2 * np.random.RandomState(1).randn(37, X.shape[1])).astype(np.float32)
    pe, g = CB.LogRegBatch(X, y)(Z)
    pe_r, g_r = OP.LogisticRegression(X, y).pe_grad_batch(Z)
    np.testing.assert_allclose(pe, pe_r, rtol=1e-5)
    scale = np.abs(X).T @ np.ones(X.shape[0]) + np.abs(Z)  # |X|^T |sigmoid - y| bound
    assert np.all(np.abs(g - g_r) <= 1e-5 * scale)


def test_batched_chains_are_the_oracle_chains():
    """Batching the potential calls of 6 chains changes nothing: each chain's states equal an
    independent oracle run (per-row evaluation with the oracle's own f32 potential)."""
    X, y = _data(N=200, D=5, seed=2)
    ref = OP.LogisticRegression(X, y, dtype=np.float32)

    def rowwise(Z):
        out = [ref.pe_grad(z) for z in Z]
        return np.array([o[0] for o in out], np.float32), np.stack([o[1] for o in out])

    seed, n, W, T = 5, 6, 10, 14
    oracles, states, indep = [], [], []
    for c in range(n):
        o = H.NUTSOracle(ref.pe_grad, 5, W)
        states.append(o.init(philox.init_uniform(seed, c, 0, 5), seed, c))
        oracles.append(H.NUTSOracle(None, 5, W))
        s = states[-1]
        hist = []
        for _ in range(T):
            s = o.sample(s)
            hist.append(s)
        indep.append(hist)
    _, hist, evals, calls = CB.run_chains(rowwise, states, oracles, T)
    assert evals == sum(s.num_steps for h in indep for s in h)
    assert calls < evals
    for c in range(n):
        for a, b in zip(hist[c], indep[c]):
            assert a.num_steps == b.num_steps
            np.testing.assert_array_equal(a.z, b.z)
            assert a.adapt_state.step_size == b.adapt_state.step_size


def test_fixed_batch_mode_and_path_comparison():
    """run_chains(deadline=...) keeps every chain running until the deadline (the CPU
    comparator's fixed batch) and at least `min_transitions`; record=True returns each
    transition's decisions and leaf records, and compare_traced reports a chain whose tree sizes
    or draws leave the reference's."""
    import time

    from oracle import parity as PR

    X, y = _data(N=200, D=5, seed=3)
    ref = OP.LogisticRegression(X, y, dtype=np.float32)

    def rowwise(Z):
        out = [ref.pe_grad(z) for z in Z]
        return np.array([o[0] for o in out], np.float32), np.stack([o[1] for o in out])

    seed, n, W = 9, 4, 10
    mk = lambda: ([H.NUTSOracle(ref.pe_grad, 5, W).init(philox.init_uniform(seed, c, 0, 5), seed, c)  # noqa: E731
                   for c in range(n)], [H.NUTSOracle(None, 5, W) for _ in range(n)])
    states, oracles = mk()
    t0 = time.perf_counter()
    _, hist, evals, _ = CB.run_chains(rowwise, states, oracles, 1 << 30, deadline=t0 + 0.5, record=True)
    assert all(len(h) >= 2 for h in hist) and evals > 0
    st, log, leaves = hist[0][0]
    assert isinstance(log, list) and all(k in H.TIE for k, _ in log)
    assert len(leaves) == st.num_steps and leaves[-1]["iter_done"]
    states, oracles = mk()
    _, h3, _, _ = CB.run_chains(rowwise, states, oracles, 1 << 30, deadline=time.perf_counter(), min_transitions=3)
    assert all(len(h) == 3 for h in h3)
    T = min(len(h) for h in hist)
    tr = np.full((T, n, 1024, 8), np.nan, np.float32)
    for c, h in enumerate(hist):
        for t in range(T):
            tr[t, c] = PR.oracle_to_trace(h[t][2], 1024)
    ns = np.array([[h[t][0].num_steps for t in range(T)] for h in hist])
    zs = np.array([[h[t][0].z for t in range(T)] for h in hist], np.float64)
    par = PR.compare_traced(hist, tr, ns, zs, atol=0.0)
    assert par["matched"] == n and par["transitions"] == n * T and not par["mismatches"]
    zs_bad = zs.copy()
    zs_bad[1, 1, 0] += 1e-3
    par = PR.compare_traced(hist, tr, ns, zs_bad, atol=0.0)
    assert par["matched"] == n - 1 and (par["mismatches"][0]["chain"], par["mismatches"][0]["transition"]) == (1, 1)
    assert par["mismatches"][0]["kind"] == "draw" and not par["mismatches"][0]["explained"]


def test_bench_valu_roofline_from_the_committed_profile():
    """bench.py's c4 VALU fraction: profiled VALU wave-instructions per chain-leapfrog x rate over
    1024 SIMDs x 0.5 instructions per cycle at the profiled clock (profiles/r05/sv_valu.json)."""
    import bench

    r = bench._valu_roofline("profiles/r05/sv_valu.json", 33.0e6)
    assert r is not None and r["unit"] == "G VALU wave-instr/s"
    assert np.isclose(r["achieved"], r["insts_per_leapfrog"] * 33.0e6 / 1e9)
    assert np.isclose(r["peak"], 1024 * 0.5 * r["clock_ghz"])
    assert 0.05 < r["frac"] < 1.0
    assert bench._valu_roofline("profiles/r05/no_such_profile.json", 1.0) is None
