"""The first-parting-leaf parity machinery (oracle/parity.py) on oracle-vs-oracle runs: two
oracle runs whose potentials differ by a rounding-sized perturbation part only at decisions
the leaf energies explain, and a decision flipped far from its tie is reported as not
explained (the check has teeth).  The device side of these records is nmx_nuts_config.trace
(tests/test_gpu_parity_trace.py)."""
import math

import numpy as np

from oracle import cpu_batched as CB
from oracle import hmc_ref as H
from oracle import parity as PR
from oracle import philox
from oracle import potentials as OP


def _case(N=400, D=6, seed=11):
    rs = np.random.RandomState(seed)
    X = rs.randn(N, D).astype(np.float32)
    beta = rs.randn(D) * 0.4
    y = (rs.rand(N) < 1 / (1 + np.exp(-X @ beta))).astype(np.float32)
    return OP.LogisticRegression(X, y, dtype=np.float32), D


def _run(pe_grad, D, n, seed, T, step):
    states, oracles = [], []
    for c in range(n):
        o = H.NUTSOracle(pe_grad, D, 0, step_size=step, adapt_step_size=False, adapt_mass_matrix=False)
        states.append(o.init(philox.init_uniform(seed, c, 0, D) * np.float32(0.1), seed, c))
        oracles.append(H.NUTSOracle(None, D, 0, step_size=step, adapt_step_size=False, adapt_mass_matrix=False))

    def batch(Z):
        out = [pe_grad(z) for z in Z]
        return np.array([o[0] for o in out], np.float32), np.stack([o[1] for o in out])

    _, hist, _, _ = CB.run_chains(batch, states, oracles, T, record=True)
    return hist


def _as_device(hist, T, L=1024):
    n = len(hist)
    tr = np.full((T, n, L, 8), np.nan, np.float32)
    ns = np.zeros((n, T), np.int64)
    z = np.zeros((n, T, hist[0][0][0].z.shape[0]))
    for c, h in enumerate(hist):
        for t in range(T):
            st, _, leaves = h[t]
            tr[t, c] = PR.oracle_to_trace(leaves, L)
            ns[c, t] = st.num_steps
            z[c, t] = st.z
    return tr, ns, z


def test_leaf_records_follow_the_tree():
    ref, D = _case()
    hist = _run(ref.pe_grad, D, 4, 3, 3, 0.05)
    for h in hist:
        for st, _, leaves in h:
            assert len(leaves) == st.num_steps
            assert leaves[-1]["iter_done"] and not any(r["iter_done"] for r in leaves[:-1])
            # subtree ends: sizes 1, 2, 4, ... (or cut short by a U-turn / divergence)
            ends = [i for i, r in enumerate(leaves) if r["done_sub"]]
            assert ends[0] == 0 and all(r["p_leaf"] == -1.0 for r in leaves[:1])


def test_identical_runs_match_leaf_for_leaf():
    ref, D = _case()
    T = 3
    hist = _run(ref.pe_grad, D, 6, 5, T, 0.05)
    tr, ns, z = _as_device(hist, T)
    par = PR.compare_traced(hist, tr, ns, z, atol=0.0)
    assert par["matched"] == 6 and not par["mismatches"] and par["max_dE_err"] == 0.0
    for c, h in enumerate(hist):
        for t in range(T):
            assert PR.locate(tr[t, c], h[t][2]) is None


def test_energy_perturbation_parts_only_at_explained_leaves():
    """Every leaf energy perturbed by a deterministic function of the position of size <= 5e-3
    (gradients untouched, so the trajectories stay the same): transition probabilities move by
    up to ~1e-3, some chains part, and each must do so at a leaf where the shared uniform falls
    between the two probabilities, within the bound the measured leaf-energy discrepancy
    allows."""
    ref, D = _case(N=600)

    def perturbed(z):
        u, g = ref.pe_grad(z)
        return np.float32(u + np.float32(5e-3) * np.float32(np.sin(1e4 * float(z[0]) + 3e3 * float(z[1])))), g

    T, n = 8, 32
    a = _run(ref.pe_grad, D, n, 9, T, 0.08)
    b = _run(perturbed, D, n, 9, T, 0.08)
    tr, ns, z = _as_device(b, T)
    par = PR.compare_traced(a, tr, ns, z, atol=0.0)
    for m in par["mismatches"]:
        print(PR.describe(m))
    assert 0 < par["max_dE_err"] <= 1.1e-2  # two perturbed energies per dE
    assert par["mismatches"], "the perturbation flipped no decision: the test would be vacuous"
    assert all(m["explained"] for m in par["mismatches"]), par["mismatches"]


def test_flip_far_from_a_tie_is_not_explained():
    ref, D = _case()
    hist = _run(ref.pe_grad, D, 4, 7, 2, 0.05)
    for c, h in enumerate(hist):
        leaves = h[0][2]
        # a leaf with an in-subtree transition whose uniform is far from its probability
        cand = [i for i, r in enumerate(leaves) if r["p_leaf"] >= 0 and abs(r["u_leaf"] - r["p_leaf"]) > 0.05]
        if not cand:
            continue
        i = cand[0]
        dev = PR.oracle_to_trace(leaves, 1024)
        dev[i, PR.T_FLAGS] = float(int(dev[i, PR.T_FLAGS]) ^ PR.TF_TAKE_LEAF)
        loc = PR.locate(dev, leaves)
        assert loc["leaf"] == i and loc["kind"] == "take_leaf" and not loc["explained"]
        return
    raise AssertionError("no leaf with a clear transition decision")


def test_calibration_between_two_float32_implementations():
    """like_calibration: two float32 implementations of one potential (float32 sums vs rounded
    float64) compared with a third are of the same order; a record with an unexplained parting
    or far fewer matched chains is not."""
    from oracle import potentials as OP

    rs = np.random.RandomState(4)
    X = rs.randn(500, 5).astype(np.float32)
    y = (rs.rand(500) < 0.5).astype(np.float32)
    r32 = OP.LogisticRegression(X, y, dtype=np.float32)
    r64 = OP.LogisticRegression(X, y, dtype=np.float64)
    f64 = lambda z: tuple(np.asarray(v, np.float32) for v in r64.pe_grad(z))  # noqa: E731
    T, n = 4, 12
    ref = _run(f64, 5, n, 2, T, 0.1)
    a = _run(r32.pe_grad, 5, n, 2, T, 0.1)
    tr, ns, z = _as_device(a, T)
    par = PR.compare_traced(ref, tr, ns, z, atol=1e-4, rtol=1e-4)
    ok, msg = PR.like_calibration(par, par)
    assert ok, msg
    bad = dict(par, matched=0, mismatches=par["mismatches"] + [{"kind": "take_leaf", "explained": False}])
    assert not PR.like_calibration(bad, par)[0]


def test_draw_mismatch_needs_a_calibration_and_is_bounded_by_it():
    """A transition whose decisions all agree but whose draw differs (kind `draw`) is explained
    only by a rounding calibration: within DRAW_MULT x the calibration's drift on that chain and
    transition.  A corrupted proposal (every decision equal, the draw moved far beyond the drift
    rounding produces) is reported as unexplained -- with or without a calibration."""
    rs = np.random.RandomState(4)
    X = rs.randn(500, 5).astype(np.float32)
    y = (rs.rand(500) < 0.5).astype(np.float32)
    r32 = OP.LogisticRegression(X, y, dtype=np.float32)
    r64 = OP.LogisticRegression(X, y, dtype=np.float64)
    f64 = lambda z: tuple(np.asarray(v, np.float32) for v in r64.pe_grad(z))  # noqa: E731
    T, n = 3, 8
    ref = _run(f64, 5, n, 2, T, 0.1)
    cal_tr, cal_ns, cal_z = _as_device(_run(r32.pe_grad, 5, n, 2, T, 0.1), T)
    cal = PR.compare_traced(ref, cal_tr, cal_ns, cal_z, atol=1e-6, rtol=0.0)
    # the "device": the calibration's own run with one draw corrupted by 1e-2
    z_bad = cal_z.copy()
    z_bad[3, 1, 2] += 1e-2
    par = PR.compare_traced(ref, cal_tr, cal_ns, z_bad, atol=1e-6, rtol=0.0)
    draws = [m for m in par["mismatches"] if m["kind"] == "draw"]
    assert any(m["chain"] == 3 and m["transition"] <= 1 for m in draws)
    assert PR.counts(par)["unexplained"] >= 1  # no calibration: a draw is never explained
    PR.bound_draws(par, cal)
    bad = [m for m in par["mismatches"] if m["chain"] == 3]
    assert bad and not bad[0]["explained"] and bad[0]["ratio"] > PR.DRAW_MULT, bad
    ok, msg = PR.like_calibration(par, cal)
    assert not ok, msg
    # the calibration against itself: every draw mismatch it has is its own drift (ratio 1)
    same = PR.compare_traced(ref, cal_tr, cal_ns, cal_z, atol=1e-6, rtol=0.0)
    PR.bound_draws(same, cal)
    assert all(m["explained"] for m in same["mismatches"] if m["kind"] == "draw")
    assert same["draw_drift"]["geo_mean_ratio"] == 1.0
    ok, msg = PR.like_calibration(same, cal)
    assert ok, msg


def test_draw_bound_uses_the_calibrations_typical_drift_at_that_transition():
    """A chain whose own calibration drift is small is bounded by the calibration's median drift
    over chains at the same transition (chaotic trajectories spread single-chain drifts over two
    orders of magnitude); the paired geometric mean is judged at its lower 95% bound."""
    drift = [{"chain": c, "transition": 1, "tree": 7, "drift": d, "dz": d}
             for c, d in enumerate([1.0, 30.0, 50.0, 80.0, 200.0])]
    cal = {"drift": drift, "mismatches": [], "matched": 0}
    par = {"drift": [], "mismatches": [{"kind": "draw", "chain": 0, "transition": 1,
                                        "tree_oracle": 7, "drift": 60.0, "dz": 60.0}]}
    PR.bound_draws(par, cal)
    m = par["mismatches"][0]
    assert m["explained"] and m["cal_drift"] == 50.0 and "median" in m["cal_basis"], m
    # far beyond the typical drift: still unexplained
    par = {"drift": [], "mismatches": [dict(par["mismatches"][0], drift=1e4, dz=1e4)]}
    PR.bound_draws(par, cal)
    assert not par["mismatches"][0]["explained"]
    # paired drift: 3 pairs whose geometric mean is above 2x but whose spread cannot exclude 1x
    dev = {"drift": [dict(d, drift=d["drift"] * f) for d, f in zip(drift, [0.5, 1.0, 20.0])],
           "mismatches": []}
    st = PR.drift_stats(dev, cal)
    assert st["geo_mean_ratio"] > PR.DRIFT_GEO_MAX and st["geo_mean_lo95"] <= PR.DRIFT_GEO_MAX, st
    # the same ratio on every pair is judged at face value
    dev = {"drift": [dict(d, drift=d["drift"] * 3.0) for d in drift], "mismatches": []}
    st = PR.drift_stats(dev, cal)
    assert st["geo_mean_lo95"] > PR.DRIFT_GEO_MAX, st


def test_draw_on_a_chain_where_the_calibration_flipped_is_rounding_sensitive():
    """Where the second float32 implementation itself parted from the reference on a chain by a
    located rounding flip (at or before the draw's transition), a device draw that stayed on the
    reference's path there is explained and counted apart (draws_on_parted); a calibration that
    left the path only by a draw of its own earlier bounds by its largest drift at that tree size."""
    drift = [{"chain": 0, "transition": 0, "tree": 1023, "drift": 2.0, "dz": 2.0},
             {"chain": 1, "transition": 0, "tree": 1023, "drift": 5.0, "dz": 5.0},
             {"chain": 1, "transition": 1, "tree": 1023, "drift": 9.0, "dz": 9.0}]
    flip = {"kind": "take_leaf", "leaf": 521, "chain": 0, "transition": 1, "explained": True}
    cal = {"drift": drift, "mismatches": [flip], "matched": 1}
    draw = {"kind": "draw", "chain": 0, "transition": 1, "tree_oracle": 1023, "drift": 67.8, "dz": 0.09,
            "leaf": None, "margin": 0.09}
    par = {"drift": [], "mismatches": [dict(draw)]}
    PR.bound_draws(par, cal)
    m = par["mismatches"][0]
    assert m["explained"] and m["cal_drift"] == math.inf and "parted" in m["cal_basis"], m
    assert par["draw_drift"]["draws_on_parted"] == 1
    assert "rounding-sensitive" in PR.describe(m)
    # a flip the calibration could not explain does not make the chain rounding-sensitive
    cal_bad = dict(cal, mismatches=[dict(flip, explained=False)])
    par = {"drift": [], "mismatches": [dict(draw)]}
    PR.bound_draws(par, cal_bad)
    m = par["mismatches"][0]
    assert not m["explained"] and m["cal_basis"] == "largest at this tree size", m
    # a flip at a later transition does not cover an earlier draw
    cal_late = dict(cal, mismatches=[dict(flip, transition=2)])
    par = {"drift": [], "mismatches": [dict(draw)]}
    PR.bound_draws(par, cal_late)
    assert not par["mismatches"][0]["explained"]


def test_calibration_drift_is_followed_through_its_own_draws():
    """compare_traced(through_draws=True) keeps recording a chain's drift after its first `draw`
    mismatch (same decisions, draws apart) while the decisions keep agreeing, with one mismatch per
    chain as before; so a device draw later on that chain is bounded by the calibration's own drift
    there."""
    rs = np.random.RandomState(4)
    X = rs.randn(500, 5).astype(np.float32)
    y = (rs.rand(500) < 0.5).astype(np.float32)
    r32 = OP.LogisticRegression(X, y, dtype=np.float32)
    r64 = OP.LogisticRegression(X, y, dtype=np.float64)
    f64 = lambda z: tuple(np.asarray(v, np.float32) for v in r64.pe_grad(z))  # noqa: E731
    T, n = 3, 8
    ref = _run(f64, 5, n, 2, T, 0.1)
    cal_tr, cal_ns, cal_z = _as_device(_run(r32.pe_grad, 5, n, 2, T, 0.1), T)
    plain = PR.compare_traced(ref, cal_tr, cal_ns, cal_z, atol=1e-7, rtol=0.0)
    thru = PR.compare_traced(ref, cal_tr, cal_ns, cal_z, atol=1e-7, rtol=0.0, through_draws=True)
    draws = [m for m in plain["mismatches"] if m["kind"] == "draw" and m["transition"] < T - 1]
    assert draws, "the tolerance is below float32 drift: every chain has a draw mismatch"
    assert len(thru["mismatches"]) == len(plain["mismatches"]) and thru["matched"] == plain["matched"]
    keys = {(d["chain"], d["transition"]) for d in thru["drift"]}
    for m in draws:
        assert (m["chain"], m["transition"] + 1) in keys
    assert len(thru["drift"]) > len(plain["drift"])


def test_calibration_flip_after_its_draw_marks_the_chain_rounding_sensitive():
    """A calibration that drew apart at transition 0 (a draw) and flipped a decision at transition 1
    lists the flip in partings_after_draw; a device draw at transition 1 on that chain is then
    explained as a rounding-sensitive chain."""
    cal = {"drift": [{"chain": 0, "transition": 0, "tree": 1023, "drift": 2.1, "dz": 0.002}],
           "mismatches": [{"kind": "draw", "leaf": None, "chain": 0, "transition": 0, "explained": False}],
           "partings_after_draw": [{"chain": 0, "transition": 1, "kind": "take_leaf", "leaf": 17,
                                    "explained": True}], "matched": 0}
    par = {"drift": [], "mismatches": [{"kind": "draw", "chain": 0, "transition": 1, "tree_oracle": 1023,
                                        "drift": 67.8, "dz": 0.09, "leaf": None, "margin": 0.09}]}
    PR.bound_draws(par, cal)
    assert par["mismatches"][0]["explained"] and par["draw_drift"]["draws_on_parted"] == 1
