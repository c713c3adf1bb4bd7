"""ORACLE (test infrastructure only: tests/ and bench.py's parity legs) -- locate where a device
NUTS transition parts from the oracle's, leaf by leaf.

The device records, for listed chains, the quantities each leaf's decisions are taken on
(nmx_nuts_config.trace: delta energy, in-subtree transition probability, the smallest iterative
U-turn dot, at a subtree end the biased transition probability and the whole-tree dot, and the
decisions taken); the oracle records the same per leaf (oracle.hmc_ref.record_leaves), plus the
uniforms of its transition draws (the same Philox stream as the device) and the magnitudes of
the U-turn dots' terms.

Up to the first leaf where a decision differs, device and oracle integrate the same
trajectory (positions depend only on the doubling directions and the step, not on which leaf
is the proposal), so every earlier leaf measures how far f32 rounding has carried the two
apart: dE_err = max |dE_dev - dE_oracle| over the leaves up to the parting one.  A parting is a
rounding flip -- `explained` -- when:

* a transition draw (hmc_util.py:749-764): the shared uniform lies between the two
  probabilities and they differ by no more than the leaf energies can move them.  The in-subtree
  probability is sigmoid(w_new - w_sub) with w_sub a logaddexp of leaf weights (both
  1-Lipschitz in the largest leaf-energy change), so it moves by <= 2 dE_err / 4; the biased one
  min(1, exp(w_sub - w_tree)) moves by <= p * 2 dE_err.  Bound: twice those, plus 1e-6 for the
  probability's own f32 rounding;
* an HMC Metropolis accept (hmc.py:401-414, one record per transition): as the biased
  transition, the probability min(1, exp(-dE)) moving by <= p * 2 dE_err;
* a divergence (hmc_util.py:872): the two delta energies lie on either side of
  max_delta_energy;
* a U-turn (hmc_util.py:735-746): the two smallest dots have different signs and differ by no
  more than max(4 x the largest relative dot discrepancy seen at the earlier leaves, 1e-5) x the
  magnitude of the dot's terms.

A transition whose decisions all agree but whose draw differs is reported as `draw`: the same
leaf was selected, but the positions drifted apart along the trajectory (leapfrog dynamics of a
tanh network or a stiff posterior amplify rounding over hundreds of leaves).  A draw has a
bound too: it is explained only by a rounding calibration (below) -- when the device's drift
at that chain and transition is within DRAW_MULT x the calibration's drift there, or x the
calibration's median drift over its chains at that transition where that is larger (chaotic
trajectories spread single-chain drifts over two orders of magnitude).  Where the calibration
itself left the reference's path on that chain by a located rounding flip (at this transition or
before), the chain's trajectory is rounding-sensitive beyond what a drift bound measures, and a
device that stayed on the path is explained (reported as such, counted apart in the drift
statistics' `draws_on_parted`); where the calibration left the path otherwise (a draw of its own at
an earlier transition), its largest drift at the same tree size stands in.  Without a calibration a draw mismatch is unexplained: a bug that corrupts
the proposal (the whitening's to_model, the collection) while every decision stays equal
cannot pass as drift.  Drift is measured in tolerance units, max_i |z_i - ref_i| / (atol +
rtol |ref_i|), so a draw mismatch has drift > 1.

Calibration.  How far rounding alone carries two float32 implementations of the same
algorithm apart is measured, not assumed: `compare_traced` run between the reference oracle
(potential in rounded float64, the most accurate float32 NUTS) and a second oracle whose
potential is a float32 implementation (oracle/batched.py's NumPy batch, or float32 sums) gives
the spread rounding alone produces -- matched chains, located partings, the drift of every
transition whose decisions agree (followed through the calibration's own draw mismatches,
compare_traced(through_draws=True): a draw leaves a chain on the reference's path), the relative
leaf-energy discrepancy.  The device is compared
with the same reference; `bound_draws` explains (or not) its draw mismatches by the
calibration's drift, and `like_calibration` requires its whole record to be of the
calibration's order: drift distributions compared pairwise on the (chain, transition) pairs both
reached on the reference's path (geometric mean of the ratios <= DRIFT_GEO_MAX, at its lower
95% bound when the pairs are few), leaf-energy
discrepancies relative to the energies' magnitude (tests/test_gpu_parity_trace.py, bench.py's
config legs)."""
from __future__ import annotations

import math

import numpy as np

# enum nmx_trace_field / nmx_trace_flag (include/numpyro_amd.h)
T_DE, T_P_LEAF, T_DOT_SUB, T_P_BIASED, T_DOT_TREE, T_FLAGS, T_PE, T_LEAF = range(8)
TF_TAKE_LEAF, TF_TURN_SUB, TF_DIVERGE, TF_DONE_SUB, TF_TAKE_BIASED, TF_TURN_TREE, TF_ITER_DONE = (
    1, 2, 4, 8, 16, 32, 64)

DOT_FLOOR = 1e-5  # relative f32 rounding of a U-turn dot over D <= 1e4 terms
P_FLOOR = 1e-6  # f32 rounding of a transition probability itself
DRAW_MULT = 4.0  # a draw mismatch is explained when its drift <= DRAW_MULT x the calibration's there
DRIFT_GEO_MAX = 2.0  # like_calibration: geometric mean of paired device / calibration drifts
DRIFT_FLOOR = 1e-2  # drift (tolerance units) below which a ratio is not taken (floored on both sides)
DE_REL_MULT = 10.0  # like_calibration: relative leaf-energy discrepancy vs the calibration's


def _dev_flags(rec):
    f = int(rec[T_FLAGS])
    return {"take_leaf": bool(f & TF_TAKE_LEAF), "turn_sub": bool(f & TF_TURN_SUB),
            "diverge": bool(f & TF_DIVERGE), "done_sub": bool(f & TF_DONE_SUB),
            "take_biased": bool(f & TF_TAKE_BIASED), "turn_tree": bool(f & TF_TURN_TREE),
            "iter_done": bool(f & TF_ITER_DONE)}


# decision kinds in the order a leaf takes them (csrc/nuts.hip leaf_phase / tree_phase)
_ORDER = ("diverge", "turn_sub", "take_leaf", "done_sub", "turn_tree", "take_biased", "iter_done")


def locate(dev, orc, max_delta_energy=1000.0):
    """dev: [L, 8] device trace of one transition (rows past its tree are NaN); orc: the
    oracle's leaf records of the same transition.  Returns None when every common leaf takes
    the same decisions, else {leaf, kind, dev, oracle, u, margin, bound, dE_err, explained}."""
    n = min(len(orc), int(np.sum(np.isfinite(dev[:, T_FLAGS]))))
    de_err, rel_dot = 0.0, 0.0
    for i in range(n):
        d, o = dev[i], orc[i]
        df = _dev_flags(d)
        de_err = max(de_err, abs(float(d[T_DE]) - o["dE"])) if np.isfinite(o["dE"]) else de_err
        full = o["done_sub"] and not o["turn_sub"] and not o["diverge"] and math.isfinite(o["dot_tree"])
        diff = None
        for k in _ORDER:
            if k == "turn_tree" and not full:
                continue
            if k == "take_biased" and not (o["done_sub"] and df["done_sub"]):
                continue
            if df[k] != o[k]:
                diff = k
                break
        if diff is None:
            # the leaf agreed: its dots measure the rounding of the U-turn dots so far
            for dk, sk in (("dot_sub", "scale_sub"), ("dot_tree", "scale_tree")):
                dv = float(d[T_DOT_SUB if dk == "dot_sub" else T_DOT_TREE])
                if math.isfinite(o[dk]) and math.isfinite(dv) and o[sk] > 0:
                    rel_dot = max(rel_dot, abs(dv - o[dk]) / o[sk])
            continue
        out = {"leaf": i, "kind": diff, "dE_err": de_err}
        if diff in ("take_leaf", "take_biased"):
            pk, uk = ("p_leaf", "u_leaf") if diff == "take_leaf" else ("p_biased", "u_biased")
            pd, po, u = float(d[T_P_LEAF if diff == "take_leaf" else T_P_BIASED]), o[pk], o[uk]
            # in-subtree sigmoid: 1-Lipschitz in the leaf energies (x 2 for the logaddexp);
            # biased / HMC Metropolis min(1, exp(-dE)): slope p per unit of energy
            slope = 1.0 if diff == "take_leaf" and not o.get("hmc") else 4.0 * max(pd, po)
            if o.get("hmc"):
                diff = out["kind"] = "accept"
            bound = slope * de_err + P_FLOOR
            out.update(dev=pd, oracle=po, u=u, margin=abs(u - po), bound=bound,
                       explained=bool((pd - u) * (po - u) <= 0 and abs(pd - po) <= bound))
        elif diff == "diverge":
            ed, eo = float(d[T_DE]), o["dE"]
            out.update(dev=ed, oracle=eo, u=None, margin=abs(eo - max_delta_energy), bound=abs(ed - eo),
                       explained=bool((ed - max_delta_energy) * (eo - max_delta_energy) <= 0))
        elif diff in ("turn_sub", "turn_tree"):
            dk, sk = ("dot_sub", "scale_sub") if diff == "turn_sub" else ("dot_tree", "scale_tree")
            dv, ov, sc = float(d[T_DOT_SUB if diff == "turn_sub" else T_DOT_TREE]), o[dk], o[sk]
            bound = max(4.0 * rel_dot, DOT_FLOOR) * sc
            out.update(dev=dv, oracle=ov, u=None, margin=abs(ov), bound=bound,
                       explained=bool((dv <= 0) != (ov <= 0) and abs(dv - ov) <= bound))
        else:  # done_sub / iter_done differ without a differing cause: a bookkeeping bug
            out.update(dev=None, oracle=None, u=None, margin=None, bound=None, explained=False)
        return out
    return None


def _drift(z, ref, atol, rtol):
    """Largest coordinate difference in tolerance units (atol + rtol |ref|); raw when both are 0."""
    den = atol + rtol * np.abs(ref)
    d = np.abs(z - ref)
    return float(np.max(d / den)) if np.all(den > 0) else float(np.max(d))


def compare_traced(hist, dev_trace, dev_num_steps, dev_z, atol, rtol=0.0, to_model=None, max_delta_energy=1000.0,
                   through_draws=False):
    """Per-chain parity of oracle histories (oracle.cpu_batched.run_chains(record=True): entries
    (state, decisions, leaves)) with the device's transitions from the same state, each
    mismatch located at its parting leaf.  dev_trace [T, chains, L, 8] is the engine's decision
    trace (Engine.set_trace) over the same transitions.  A chain matches while tree sizes are
    equal and draws agree to atol + rtol |z|.  Returns {chains, transitions, matched,
    max_abs_dz, max_dE_err, max_dE_rel, worst_dE, drift, mismatches: [{chain, transition,
    tree_dev, tree_oracle, leaf, kind, dev, oracle, u, margin, bound, dE_err, explained}],
    explained}.  `drift` lists every transition whose decisions all agree (matched, or the
    chain's `draw` mismatch): {chain, transition, tree, drift (tolerance units), dz}.
    `worst_dE` locates the largest leaf-energy discrepancy on the common leaves (chain,
    transition, leaf, the two delta energies, the leaf's potential energy and the discrepancy
    relative to |U_leaf| + |dE|, the magnitude the energies' rounding scales with).

    through_draws (for a rounding calibration): a chain's comparison goes on past its first
    `draw` mismatch (same tree, every decision equal: still on the reference's path), recording
    the drift of each later transition whose decisions agree, up to a located parting (not recorded
    again: one mismatch per chain either way; such partings are listed in `partings_after_draw`).
    A device draw at a later transition on that chain then has the calibration's own drift there as
    its bound, or -- where the calibration flipped there -- the chain counts as rounding-sensitive
    (bound_draws)."""
    matched, transitions, max_dz, max_de, mism, drift, later = 0, 0, 0.0, 0.0, [], [], []
    worst, max_rel = None, 0.0
    for c, h in enumerate(hist):
        T = min(len(h), dev_num_steps.shape[1], dev_trace.shape[0])
        transitions += T
        ok = True
        for t in range(T):
            st, _, leaves = h[t]
            z = np.asarray(st.z, np.float64) if to_model is None else np.asarray(to_model(st.z), np.float64)
            ref = np.asarray(dev_z[c, t], np.float64)
            dz = float(np.max(np.abs(z - ref) - rtol * np.abs(ref)))
            dr = _drift(z, ref, atol, rtol)
            dev = dev_trace[t, c]
            n = min(len(leaves), int(st.num_steps))
            de = []
            for i in range(n):
                ed, eo = float(dev[i, T_DE]), leaves[i]["dE"]
                if not (np.isfinite(ed) and np.isfinite(eo)):
                    continue
                err = abs(ed - eo)
                de.append(err)
                rel = err / max(1.0, abs(float(leaves[i]["pe"])) + abs(eo))
                if worst is None or rel > worst["rel"]:
                    worst = {"chain": c, "transition": t, "leaf": i, "dev": ed, "oracle": eo,
                             "pe": float(leaves[i]["pe"]), "err": err, "rel": rel}
                max_rel = max(max_rel, rel)
            if st.num_steps != int(dev_num_steps[c, t]) or dz > atol:
                loc = locate(dev, leaves, max_delta_energy)
                same_tree = st.num_steps == int(dev_num_steps[c, t])
                if loc is None:
                    loc = {"leaf": None, "kind": "draw", "dev": None, "oracle": None, "u": None, "margin": dz,
                           "bound": atol, "dE_err": max(de) if de else 0.0, "explained": False, "drift": dr}
                    drift.append({"chain": c, "transition": t, "tree": int(st.num_steps), "drift": dr, "dz": dz})
                elif not ok:
                    # through_draws: a located parting after the chain's draw ends its record (kept
                    # apart: bound_draws reads it as the calibration leaving the path there)
                    later.append({"chain": c, "transition": t, "kind": loc["kind"], "leaf": loc["leaf"],
                                  "explained": loc["explained"]})
                    break
                loc.update(chain=c, transition=t, tree_dev=int(dev_num_steps[c, t]), tree_oracle=int(st.num_steps))
                if ok:
                    mism.append(loc)
                ok = False
                if through_draws and loc["kind"] == "draw" and same_tree:
                    continue
                break
            drift.append({"chain": c, "transition": t, "tree": int(st.num_steps), "drift": dr, "dz": dz})
            max_dz = max(max_dz, dz)
            if de:
                max_de = max(max_de, max(de))
        if ok:
            matched += 1
    return {"chains": len(hist), "transitions": transitions, "matched": matched, "max_abs_dz": max_dz,
            "max_dE_err": max_de, "max_dE_rel": max_rel, "worst_dE": worst, "drift": drift,
            "mismatches": mism, "explained": sum(1 for m in mism if m["explained"]), "partings_after_draw": later}


def bound_draws(par, cal, mult=DRAW_MULT):
    """Explain (or not) the `draw` mismatches of the device record `par` by the rounding
    calibration `cal` (compare_traced of a second float32 oracle against the same reference):
    a draw is a rounding drift when the device's drift is within `mult` x the calibration's on
    the same chain and transition; where the calibration left the reference's path on that chain
    by a located rounding flip at or before that transition, the draw is explained (ratio 0,
    cal_drift inf: the chain is rounding-sensitive); where it left it by a draw of its own, its
    largest drift at the same tree size (any tree size if none) stands in.  Sets
    cal_drift / ratio / explained on each draw and par["draw_drift"] (paired drift statistics,
    see drift_stats); returns par."""
    at = {(d["chain"], d["transition"]): d["drift"] for d in cal["drift"]}
    # transitions at which the calibration itself left the reference's path by a located rounding
    # flip (chain -> first such transition)
    cal_parted = {}
    for cm in cal.get("mismatches", []) + cal.get("partings_after_draw", []):
        if cm.get("leaf") is not None and cm.get("explained"):
            cal_parted[cm["chain"]] = min(cal_parted.get(cm["chain"], cm["transition"]), cm["transition"])
    by_tree, by_t = {}, {}
    for d in cal["drift"]:
        by_tree[d["tree"]] = max(by_tree.get(d["tree"], 0.0), d["drift"])
        by_t.setdefault(d["transition"], []).append(d["drift"])
    typical = {t: float(np.median(v)) for t, v in by_t.items()}
    top = max((d["drift"] for d in cal["drift"]), default=0.0)
    for m in par["mismatches"]:
        if m["kind"] != "draw":
            continue
        key = (m["chain"], m["transition"])
        if key in at:
            # a chaotic trajectory's drift varies by two orders of magnitude between chains at the
            # same transition (BNN c3: 1.05 to 198 tolerance units), so a chain whose own
            # calibration drift happens to be small is bounded by the calibration's typical drift
            # at that transition instead
            ref, how = at[key], "same chain and transition"
            med = typical.get(m["transition"], 0.0)
            if med > ref:
                ref, how = med, "median of the calibration's chains at this transition"
        elif cal_parted.get(m["chain"], math.inf) <= m["transition"]:
            # the second float32 implementation could not follow the reference on this chain (a
            # rounding flip at its own leaf, at this transition or before): the trajectory is
            # rounding-sensitive beyond what a drift bound measures, and the device, still on the
            # reference's path, drifts less than an implementation that left it
            m["cal_drift"], m["cal_basis"] = math.inf, (f"the calibration itself parted on this chain "
                                                         f"(rounding flip at transition {cal_parted[m['chain']]})")
            m["ratio"], m["bound"], m["explained"] = 0.0, math.inf, True
            continue
        elif m["tree_oracle"] in by_tree:
            ref, how = by_tree[m["tree_oracle"]], "largest at this tree size"
        else:
            ref, how = top, "largest of the calibration"
        m["cal_drift"], m["cal_basis"] = ref, how
        m["ratio"] = m["drift"] / ref if ref > 0 else math.inf
        m["bound"] = mult * ref
        m["explained"] = bool(m["ratio"] <= mult)
    par["explained"] = sum(1 for m in par["mismatches"] if m["explained"])
    par["draw_drift"] = drift_stats(par, cal)
    return par


def drift_stats(par, cal):
    """Paired drift of the device and the calibration on the (chain, transition) pairs where both
    took the reference's decisions: {pairs, geo_mean_ratio, median_dev, median_cal, max_dev,
    max_cal, draws, max_draw_ratio}.  Drifts in tolerance units; ratios floored at DRIFT_FLOOR units
    on both sides: drift below 1% of the tolerance is bit-level agreement, whose ratio says nothing
    (two float32 implementations of a diagonal normal differ there by 2x from a reciprocal)."""
    a = {(d["chain"], d["transition"]): d["drift"] for d in par["drift"]}
    b = {(d["chain"], d["transition"]): d["drift"] for d in cal["drift"]}
    keys = sorted(set(a) & set(b))
    fl = DRIFT_FLOOR
    r = [math.log(max(a[k], fl) / max(b[k], fl)) for k in keys]
    draws = [m for m in par["mismatches"] if m["kind"] == "draw"]
    # the geometric mean's lower 95% bound (2 standard errors of the mean log ratio): a chaotic
    # pair's log ratio has a spread of ~1 or more, so a few pairs cannot tell 2x from 1x
    lo = None
    if len(r) >= 2:
        mu, sd = sum(r) / len(r), float(np.std(r, ddof=1))
        lo = math.exp(mu - 2.0 * sd / math.sqrt(len(r)))
    elif r:
        lo = math.exp(r[0])
    return {"pairs": len(keys), "geo_mean_ratio": math.exp(sum(r) / len(r)) if r else None,
            "geo_mean_lo95": lo,
            "median_dev": float(np.median([a[k] for k in keys])) if keys else None,
            "median_cal": float(np.median([b[k] for k in keys])) if keys else None,
            "max_dev": max((a[k] for k in keys), default=None), "max_cal": max((b[k] for k in keys), default=None),
            "draws": len(draws), "max_draw_ratio": max((m.get("ratio", math.inf) for m in draws), default=None),
            "draws_on_parted": sum(1 for m in draws if m.get("cal_drift") == math.inf)}


def oracle_to_trace(leaves, L):
    """The device trace layout [L, 8] of one transition's oracle leaf records (NaN past the
    tree): lets tests run `locate` on two oracle runs."""
    out = np.full((L, 8), np.nan, np.float32)
    for i, o in enumerate(leaves[:L]):
        f = ((TF_TAKE_LEAF if o["take_leaf"] else 0) | (TF_TURN_SUB if o["turn_sub"] else 0) |
             (TF_DIVERGE if o["diverge"] else 0) | (TF_DONE_SUB if o["done_sub"] else 0) |
             (TF_TAKE_BIASED if o["take_biased"] else 0) | (TF_TURN_TREE if o["turn_tree"] else 0) |
             (TF_ITER_DONE if o["iter_done"] else 0))
        out[i] = [o["dE"], o["p_leaf"], o["dot_sub"], o["p_biased"], o["dot_tree"], f, o["pe"], i]
    return out


def describe(m):
    """One line per located mismatch (test / bench stderr)."""
    if m["leaf"] is None:
        cal = "" if "cal_drift" not in m else (
            f"; drift {m['drift']:.3g} vs calibration {m['cal_drift']:.3g} ({m['cal_basis']}) = {m['ratio']:.3g}x "
            f"-> {'rounding drift' if m['explained'] else 'NOT explained by rounding'}")
        if m.get("cal_drift") == math.inf:
            cal = f"; drift {m['drift']:.3g} where {m['cal_basis']} -> rounding-sensitive chain"
        if "cal_drift" not in m:
            cal = "; no rounding calibration -> NOT explained"
        return (f"chain {m['chain']}: transition {m['transition']} draws differ by {m['margin']:.3g} with every "
                f"decision equal{cal}")
    val = "" if m["dev"] is None else f" dev {m['dev']:.6g} oracle {m['oracle']:.6g}"
    u = "" if m["u"] is None else f" u {m['u']:.6g}"
    b = "" if m["bound"] is None else f" bound {m['bound']:.3g}"
    return (f"chain {m['chain']}: transition {m['transition']} (tree {m['tree_dev']} dev / {m['tree_oracle']} "
            f"oracle) parts at leaf {m['leaf']} on {m['kind']}:{val}{u}{b}, leaf-energy discrepancy up to it "
            f"{m['dE_err']:.3g} -> {'rounding flip' if m['explained'] else 'NOT explained by rounding'}")


def counts(par):
    """{matched, chains, <kind>: n, unexplained} of a compare_traced record (a draw counts as
    unexplained unless bound_draws explained it by a calibration)."""
    out = {"chains": par["chains"], "matched": par["matched"], "unexplained": 0}
    for m in par["mismatches"]:
        out[m["kind"]] = out.get(m["kind"], 0) + 1
        out["unexplained"] += 0 if m["explained"] else 1
    return out


def like_calibration(dev, cal, slack=None):
    """(ok, message): the device-vs-reference record `dev` is of the same order as the rounding
    calibration `cal` (a second float32 oracle vs the same reference, same chains): its draws
    bounded by the calibration's drift (bound_draws) and every located parting explained at its
    leaf; matched chains within `slack` (default max(4, chains / 10)) of the calibration's; the
    paired drift's geometric-mean ratio <= DRIFT_GEO_MAX (its lower 95% bound, over few pairs);
    and the largest relative leaf-energy
    discrepancy within DE_REL_MULT x the calibration's (floor 1e-7, a few float32 ulps)."""
    if "draw_drift" not in dev:
        bound_draws(dev, cal)
    if "draw_drift" not in cal:
        bound_draws(cal, cal)  # the calibration's own draws are the rounding drift (ratio 1)
    a, b = counts(dev), counts(cal)
    slack = max(4, dev["chains"] // 10) if slack is None else slack
    g = dev["draw_drift"]["geo_mean_ratio"]
    rel_ok = dev["max_dE_rel"] <= DE_REL_MULT * max(cal["max_dE_rel"], 1e-7)
    msg = (f"device {a} (max dE err {dev['max_dE_err']:.3g}, relative {dev['max_dE_rel']:.3g}) vs rounding "
           f"calibration {b} (max dE err {cal['max_dE_err']:.3g}, relative {cal['max_dE_rel']:.3g}); paired drift "
           f"{dev['draw_drift']['pairs']} transitions, geometric-mean ratio "
           f"{'n/a' if g is None else format(g, '.3g')} (lower 95% bound "
           f"{'n/a' if dev['draw_drift'].get('geo_mean_lo95') is None else format(dev['draw_drift']['geo_mean_lo95'], '.3g')}), median {dev['draw_drift']['median_dev']} vs "
           f"{dev['draw_drift']['median_cal']} tolerance units")
    lo = dev["draw_drift"].get("geo_mean_lo95")
    ok = (a["unexplained"] == 0 and a["matched"] >= b["matched"] - slack and rel_ok
          and (lo is None or lo <= DRIFT_GEO_MAX))
    return ok, msg
