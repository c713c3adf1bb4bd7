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
* a divergence (hmc_util.py:872): the two delta energies lie on either side of
  max_delta_energy;
* a U-turn (hmc_util.py:735-746): the two smallest dots have different signs and differ by no
  more than max(4 x the largest relative dot discrepancy seen at the earlier leaves, 1e-5) x the
  magnitude of the dot's terms.

A transition whose decisions all agree but whose draw differs is reported as `draw`: the same
leaf was selected, but the positions drifted apart along the trajectory (leapfrog dynamics of a
tanh network or a stiff posterior amplify rounding over hundreds of leaves).

Calibration.  How far rounding alone carries two float32 implementations of the same
algorithm apart is measured, not assumed: `compare_traced` run between the oracle and a second
oracle whose potential is another float32 implementation (oracle/batched.py's NumPy batch vs
oracle/potentials.py's rounded float64, or float32 vs rounded float64 sums) gives the reference
spread of matched chains, located partings and drift; `like_calibration` requires the device's
to be of the same order (tests/test_gpu_parity_trace.py)."""
from __future__ import annotations

import math

import numpy as np

# enum nmx_trace_field / nmx_trace_flag (include/numpyro_amd.h)
T_DE, T_P_LEAF, T_DOT_SUB, T_P_BIASED, T_DOT_TREE, T_FLAGS, T_PE, T_LEAF = range(8)
TF_TAKE_LEAF, TF_TURN_SUB, TF_DIVERGE, TF_DONE_SUB, TF_TAKE_BIASED, TF_TURN_TREE, TF_ITER_DONE = (
    1, 2, 4, 8, 16, 32, 64)

DOT_FLOOR = 1e-5  # relative f32 rounding of a U-turn dot over D <= 1e4 terms
P_FLOOR = 1e-6  # f32 rounding of a transition probability itself


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
            slope = 1.0 if diff == "take_leaf" else 4.0 * max(pd, po)
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


def compare_traced(hist, dev_trace, dev_num_steps, dev_z, atol, rtol=0.0, to_model=None, max_delta_energy=1000.0):
    """Per-chain parity of oracle histories (oracle.cpu_batched.run_chains(record=True): entries
    (state, decisions, leaves)) with the device's transitions from the same state, each
    mismatch located at its parting leaf.  dev_trace [T, chains, L, 8] is the engine's decision
    trace (Engine.set_trace) over the same transitions.  A chain matches while tree sizes are
    equal and draws agree to atol + rtol |z|.  Returns {chains, transitions, matched,
    max_abs_dz, max_dE_err, mismatches: [{chain, transition, tree_dev, tree_oracle, leaf, kind,
    dev, oracle, u, margin, bound, dE_err, explained}], explained}."""
    matched, transitions, max_dz, max_de, mism = 0, 0, 0.0, 0.0, []
    for c, h in enumerate(hist):
        T = min(len(h), dev_num_steps.shape[1], dev_trace.shape[0])
        transitions += T
        ok = True
        for t in range(T):
            st, _, leaves = h[t]
            z = np.asarray(st.z, np.float64) if to_model is None else np.asarray(to_model(st.z), np.float64)
            ref = np.asarray(dev_z[c, t], np.float64)
            dz = float(np.max(np.abs(z - ref) - rtol * np.abs(ref)))
            dev = dev_trace[t, c]
            n = min(len(leaves), int(st.num_steps))
            de = [abs(float(dev[i, T_DE]) - leaves[i]["dE"]) for i in range(n)
                  if np.isfinite(dev[i, T_DE]) and np.isfinite(leaves[i]["dE"])]
            if st.num_steps != int(dev_num_steps[c, t]) or dz > atol:
                loc = locate(dev, leaves, max_delta_energy)
                if loc is None:
                    loc = {"leaf": None, "kind": "draw", "dev": None, "oracle": None, "u": None, "margin": dz,
                           "bound": atol, "dE_err": max(de) if de else 0.0, "explained": False}
                loc.update(chain=c, transition=t, tree_dev=int(dev_num_steps[c, t]), tree_oracle=int(st.num_steps))
                mism.append(loc)
                ok = False
                break
            max_dz = max(max_dz, dz)
            if de:
                max_de = max(max_de, max(de))
        if ok:
            matched += 1
    return {"chains": len(hist), "transitions": transitions, "matched": matched, "max_abs_dz": max_dz,
            "max_dE_err": max_de, "mismatches": mism, "explained": sum(1 for m in mism if m["explained"])}


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
        return (f"chain {m['chain']}: transition {m['transition']} draws differ by {m['margin']:.3g} with every "
                f"decision equal")
    val = "" if m["dev"] is None else f" dev {m['dev']:.6g} oracle {m['oracle']:.6g}"
    u = "" if m["u"] is None else f" u {m['u']:.6g}"
    b = "" if m["bound"] is None else f" bound {m['bound']:.3g}"
    return (f"chain {m['chain']}: transition {m['transition']} (tree {m['tree_dev']} dev / {m['tree_oracle']} "
            f"oracle) parts at leaf {m['leaf']} on {m['kind']}:{val}{u}{b}, leaf-energy discrepancy up to it "
            f"{m['dE_err']:.3g} -> {'rounding flip' if m['explained'] else 'NOT explained by rounding'}")


def counts(par):
    """{matched, chains, <kind>: n, unexplained} of a compare_traced record."""
    out = {"chains": par["chains"], "matched": par["matched"], "unexplained": 0}
    for m in par["mismatches"]:
        out[m["kind"]] = out.get(m["kind"], 0) + 1
        out["unexplained"] += 0 if (m["explained"] or m["kind"] == "draw") else 1
    return out


def like_calibration(dev, cal, slack=None):
    """(ok, message): the device-vs-oracle record `dev` is of the same order as the rounding
    calibration `cal` (oracle vs another float32 oracle on the same chains): every located
    parting explained at its leaf, matched chains within `slack` (default max(4, chains / 10))
    of the calibration's, and the largest leaf-energy discrepancy on matched paths within 10x
    of the calibration's (floor 1e-3)."""
    a, b = counts(dev), counts(cal)
    slack = max(4, dev["chains"] // 10) if slack is None else slack
    msg = (f"device {a} (max dE err {dev['max_dE_err']:.3g}) vs rounding calibration {b} "
           f"(max dE err {cal['max_dE_err']:.3g})")
    ok = (a["unexplained"] == 0 and a["matched"] >= b["matched"] - slack
          and dev["max_dE_err"] <= 10.0 * max(cal["max_dE_err"], 1e-3))
    return ok, msg
