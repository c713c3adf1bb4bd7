"""Benchmark: NUTS leapfrog steps/s over vectorized chains of the covtype logistic
regression (BASELINE.json metric), one process per GPU.

A "step" is one MCMC transition of every chain (one NUTS tree each).  Protocol (SURVEY.md
§8d): `--adapt` warmup/adaptation transitions (mcmc.warmup: dual averaging + diagonal mass,
default 200, untimed setup like data loading), then `--warmup` untimed sampling transitions,
then exactly `--steps` sampling transitions timed (mcmc.run), bracketed by barrier +
synchronize on every rank; value = sum(num_steps) over all chains and ranks / max-over-ranks
wall time (useful leapfrogs, inputs resident in HBM).  Timing adapted chains matters: with
the step size still at its initial value most trees are one divergent leaf.

Launch for N GPUs:  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, Peak FP32 (matrix), dense
MI355X_BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md, Peak BF16 MFMA, dense
MI355X_HBM_PEAK_GBS = 8000.0
# The covtype kernel (k_logreg_x3, potential_logreg.hip) runs each f32 product as six bf16
# MFMA products of three-term splits: its f32-equivalent ceiling is the bf16 MFMA peak / 6.
SPLIT_PRODUCTS = 6


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100, help="timed sampling transitions")
    p.add_argument("--warmup", type=int, default=5, help="untimed sampling transitions after adaptation")
    p.add_argument("--adapt", type=int, default=200, help="untimed adaptation (warmup) transitions")
    p.add_argument("--chains", type=int, default=4096, help="total chains over all GPUs")
    p.add_argument("--rows", type=int, default=581012)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--design", default="iid", choices=["iid", "structured"],
                   help="synthetic covtype design: iid N(0,1) columns (default) or the real data's structure "
                        "(one-hot groups collinear with the intercept: depth-saturated trees, datasets.covtype_structured)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (headline)")
    p.add_argument("--config-cpu-seconds", type=float, default=8.0, help="CPU baseline budget per config")
    p.add_argument("--cpu-chains", type=int, default=64, help="chains of the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--sync-chains", action="store_true", help="reference lockstep schedule")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"))
    p.add_argument("--configs", default="c2,c3,c4",
                   help="BASELINE.json secondary configs measured after the headline (comma list of c2 funnel-10k "
                        "dense, c3 BNN dense, c4 stochastic volatility; 'none' skips); c2/c3 are one-GPU configs "
                        "and run at --gpus 1 only, c4 shards its 8192 chains over the ranks")
    p.add_argument("--lib", default=None, help="(experiments) load this build of the library instead")
    p.add_argument("--chain-groups", type=int, default=None,
                   help="(experiments) chain groups on their own streams (Engine.chain_groups)")
    return p.parse_args()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _c_baseline(cn, st, seed, it0, seconds, chain_offset=0, flop=None):
    """Time the C restatement of NUTS (oracle/c/nuts_cpu.c, OpenMP) on `st`'s chains resumed from
    the GPU's state on the GPU's stream, running continuously for `seconds` (every chain starts
    its next transition at once: a fixed batch; stopped at the deadline, every evaluated leapfrog
    counted); the CPU baseline record."""
    out = cn.run(st["z"], st["zgrad"], st["pe"], st["step_size"], st["inv_mass"], st["mass_sqrt"], seed, it0,
                 1 << 14, chain_offset=chain_offset, min_transitions=0, seconds=seconds, keep_z=False)
    leap, wall, pot = out["leapfrogs"], out["wall_s"], out["potential_s"]
    rec = {"value": leap / wall, "unit": "leapfrog/s", "cores": cn.threads(), "kind": "port",
           "potential_only": {"value": leap / pot, "unit": "leapfrog/s",
                              "basis": "the same leapfrogs over the seconds inside the batched potential calls"},
           "potential_share": pot / wall, "transitions": int(out["done"].sum()), "leapfrogs": int(leap),
           "wall_s": wall, "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
           "threads_note": "OpenMP threads = the GPU box's CPU share (OMP_NUM_THREADS; nproc is the whole host)"}
    if flop is not None:
        rec["potential_gflops"] = flop * leap / pot / 1e9
    return rec


def _gpu_state(state, chains):
    cols = lambda t: t[:chains].detach().cpu().numpy().copy()  # noqa: E731
    return {"z": cols(state.z["coefs"]), "zgrad": cols(state.z_grad), "pe": cols(state.potential_energy),
            "step_size": cols(state.adapt_state.step_size), "inv_mass": cols(state.adapt_state.inverse_mass_matrix),
            "mass_sqrt": cols(state.adapt_state.mass_matrix_sqrt)}


def cpu_baseline(X, y, state, seed, it0, num_warmup, chains, seconds, dev_ns=None, dev_z=None, dev_trace=None):
    """CPU comparator (SURVEY.md §8d CPU side 2): the C restatement of the NUTS sampling kernel
    (oracle/c/nuts_cpu.c: the per-chain tree state machine in C, OpenMP over chains; the covtype
    potential's two GEMMs over the full data batched over the chains, register-blocked AVX-512,
    oracle/c/logreg_batch.c), `chains` chains started from the GPU's adapted state of the first
    chains on the same Philox stream, so they run the timed workload's trees; running continuously
    for `seconds`.  Returns leapfrogs/s, the potential-only rate and the potential's share.

    Full-size parity (with dev_ns [chains, T] / dev_z [chains, T, D], the GPU's timed
    transitions of those chains, and dev_trace, their per-leaf decision trace): the NumPy oracle
    (oracle/hmc_ref.py, the C float32 potential) runs the same T transitions from the same state;
    tree sizes and draws are compared with the GPU's, every chain that leaves the GPU's path is
    located at its parting leaf; the C restatement's own T transitions are compared too."""
    import numpy as np

    from oracle import cpu_batched as CB
    from oracle import cpu_nuts as CN

    D = X.shape[1]
    st = _gpu_state(state, chains)
    cn = CN.CpuNuts("covtype", X, y)
    cn.run(st["z"], st["zgrad"], st["pe"], st["step_size"], st["inv_mass"], st["mass_sqrt"], seed, it0, 1,
           max_tree_depth=1)  # untimed: OpenMP pool, first touch
    out = _c_baseline(cn, st, seed, it0, seconds, flop=4.0 * X.shape[0] * D)
    out["sample"] = (f"reduced C={chains}: {chains} chains of the timed workload (GPU-adapted state, same stream) "
                     f"run continuously for {out['wall_s']:.1f}s: {out['transitions']} transitions = "
                     f"{out['leapfrogs']} leapfrogs; C restatement of NUTS (oracle/c/nuts_cpu.c) with the covtype "
                     f"potential batched over chains (oracle/c/logreg_batch.c, register-blocked AVX-512, full "
                     f"{X.shape[0]}x{D} f32 data)")
    if dev_ns is not None:
        T = dev_ns.shape[1]
        resume = lambda: CB.chains_from_state(st["z"], st["zgrad"], st["pe"], st["step_size"],  # noqa: E731
                                              st["inv_mass"], st["mass_sqrt"], it0, seed, num_warmup)
        _, hist, _, _ = CB.run_chains(CB.LogRegBatch(X, y), *resume(), T, record=True)
        par = _located_parity(hist, dev_trace, dev_ns[:chains], dev_z[:chains], atol=1e-4, label="parity")
        par["basis"] = ("oracle NUTS (NumPy, oracle/hmc_ref.py, with the C float32 potential over the full data) vs "
                        "the GPU's timed transitions of the same chains from the same state on the same Philox stream: "
                        "equal tree sizes and draws within 1e-4 per transition; a chain that parts is located at the "
                        "first leaf where a decision differs (device decision trace vs oracle leaf records, "
                        "oracle/parity.py) and checked there; a draw that differs with every decision equal is "
                        "checked against the rounding calibration (the device and the C float32 oracle each against "
                        "the float64-potential oracle on that chain: device drift <= DRAW_MULT x the C oracle's)")
        draws = [m for m in par["mismatches"] if m["kind"] == "draw"]
        if draws:
            _headline_draw_calibration(par, draws, X, y, hist, dev_trace, dev_ns[:chains], dev_z[:chains], D, resume)
        # the C restatement over the same transitions: a second, independent float32 implementation
        c = cn.run(st["z"], st["zgrad"], st["pe"], st["step_size"], st["inv_mass"], st["mass_sqrt"], seed, it0, T)
        ok = [bool(np.array_equal(c["num_steps"][i], dev_ns[i]) and np.allclose(c["z"][i], dev_z[i], atol=1e-4))
              for i in range(chains)]
        par["c_restatement"] = {"chains": chains, "matched": int(sum(ok)),
                                "basis": "oracle/c/nuts_cpu.c chains (same state, same stream) vs the GPU's timed "
                                         "transitions: equal tree sizes and draws within 1e-4"}
        out["parity"] = par
    return out


def _headline_draw_calibration(par, draws, X, y, hist, dev_trace, dev_ns, dev_z, D, resume):
    """The headline's draw mismatches bounded by a rounding calibration (oracle/parity.py
    bound_draws): on the chains with a `draw` mismatch only, the oracle with the potential in
    rounded float64 (the reference) re-runs their transitions; the device and the C float32
    oracle are each compared with it, and the device's drift must be within DRAW_MULT x the C
    oracle's at that transition."""
    import numpy as np

    from oracle import cpu_batched as CB
    from oracle import parity as PR
    from oracle import potentials as OP

    chains = sorted({m["chain"] for m in draws})
    T = max(m["transition"] for m in draws) + 1
    r64 = OP.LogisticRegression(X.astype(np.float64), y.astype(np.float64), dtype=np.float64)
    f64 = lambda Z: tuple(np.asarray(v, np.float32) for v in r64.pe_grad_batch(Z))  # noqa: E731
    states, oracles = resume()
    _, h64, _, _ = CB.run_chains(f64, [states[c] for c in chains], [oracles[c] for c in chains], T, record=True)
    del r64
    sub32 = [hist[c][:T] for c in chains]
    ctr, cns, cz = _oracle_trace(sub32, dev_trace.shape[2])
    cal = PR.compare_traced(h64, ctr, cns, cz, atol=1e-4, through_draws=True)
    dev = PR.compare_traced(h64, dev_trace[:T, chains], dev_ns[chains, :T], dev_z[chains, :T], atol=1e-4)
    PR.bound_draws(dev, cal)
    for m in par["mismatches"]:
        if m["kind"] != "draw":
            continue
        sub = [d for d in dev["mismatches"] if chains[d["chain"]] == m["chain"]]
        if sub and sub[0]["kind"] == "draw":
            for k in ("cal_drift", "cal_basis", "ratio", "bound", "explained"):
                m[k] = sub[0][k]
            m["drift_vs_f64"] = sub[0]["drift"]
        elif sub:  # vs the float64 reference the device parts at a located decision: judged there
            m["explained"], m["vs_f64"] = sub[0]["explained"], sub[0]["kind"]
        print(f"[parity] chain {m['chain']} draw drift vs the float64 reference: " +
              (PR.describe(sub[0]) if sub else "device matches the float64 reference"), file=sys.stderr)
        if not sub:  # the device is on the float64 reference's path: the C float32 oracle drifted
            m["explained"], m["ratio"] = True, 0.0
    c = PR.counts(par)
    par["unexplained"] = c["unexplained"]
    par["draw_drift"] = dev["draw_drift"]


def _located_parity(hist, dev_trace, dev_ns, dev_z, atol, rtol=0.0, to_model=None, label="parity"):
    """Leaf-located parity record (oracle/parity.py compare_traced), JSON-ready; each parting is
    printed to stderr with its leaf, decision, the two values, the shared uniform and the bound."""
    import numpy as np

    from oracle import parity as PR

    par = PR.compare_traced(hist, dev_trace, dev_ns, dev_z, atol=atol, rtol=rtol, to_model=to_model)
    for m in par["mismatches"]:
        print(f"[{label}] " + PR.describe(m), file=sys.stderr)
    par["mismatches"] = [{k: (float(v) if isinstance(v, (np.floating, float)) else v) for k, v in m.items()}
                         for m in par["mismatches"]]
    # one classification for the device record and its rounding calibration (oracle/parity.py
    # counts): per kind of parting ("take_leaf", "turning", ... located at their leaf; "draw" = every
    # decision equal, the positions drifted), and unexplained = a located parting outside its
    # leaf's bound, or a decision the trace cannot place
    c = PR.counts(par)
    par["kinds"] = {k: v for k, v in c.items() if k not in ("chains", "matched", "unexplained")}
    par["unexplained"] = c["unexplained"]
    par.pop("drift")  # per-transition drifts: summarised by bound_draws / drift_stats where calibrated
    return par


# BASELINE.json configs[2..4]: (model, args, chains (total), adaptation transitions, timed
# transitions, dense mass, roofline basis, CPU-comparator potential).  Each runs in an adapted
# regime (mcmc.warmup with the reference's window schedule), the timed transitions after it.
def _config_specs():
    import numpy as np

    from numpyro_amd import datasets
    from numpyro_amd import potentials as P
    from oracle import batched as OB

    X, Y = datasets.bnn_data(N=100, D_X=3)
    H = 69
    D_bnn = 1 + 3 * H + H * H + H
    r = datasets.sp500_synthetic()
    return {
        "c2": dict(name="funnel D=10000, dense mass (pooled), examples/funnel.py", model=P.funnel, args=(10000,),
                   chains=4096, warmup=CONFIG_WARMUP["c2"], steps=5, dense="pooled", one_gpu=True,
                   flop=2.0 * 10000 * 10000, basis="2 D^2 FLOP per chain-leapfrog (z = mu + T w, g_w = T^T g_z)",
                   cpu=lambda dt=np.float32: OB.FunnelBatch(10000, dtype=dt), cpu_chains=16,
                   c_model="funnel", c_args=(10000,)),
        "c3": dict(name="BNN D_X=3 N=100 H=69 (D=5038), dense mass (pooled), examples/bnn.py", model=P.bnn,
                   args=(X, Y, H), chains=2048, warmup=CONFIG_WARMUP["c3"], steps=5, dense="pooled", one_gpu=True,
                   flop=2.0 * D_bnn * D_bnn + 6.0 * 100 * H * H + 6.0 * 100 * 3 * H,
                   basis="2 D^2 (whitening) + 6 N H^2 + 6 N Dx H (network) FLOP per chain-leapfrog",
                   cpu=lambda dt=np.float32: OB.BNNBatch(X, Y, H, dtype=dt), cpu_chains=16, parity_transitions=2,
                   c_model="bnn", c_args=(X, Y, H)),
        "c4": dict(name="stochastic volatility T=2517 (D=2519), diag mass, examples/stochastic_volatility.py",
                   model=P.stochastic_volatility, args=(r,), chains=8192, warmup=CONFIG_WARMUP["c4"],
                   steps=10, dense=False, one_gpu=False, bytes=7 * 4 * 2519,
                   basis="7 D x 4 B per chain-leapfrog (z, r, g read + write, inverse mass read; SURVEY §8d)",
                   valu_profile="profiles/r05/sv_valu.json",
                   cpu=lambda dt=np.float32: OB.SVBatch(r, dtype=dt), cpu_chains=32,
                   c_model="sv", c_args=(r,)),
    }


# chains of the C restatement's timed CPU run (the GPU's first chains): enough for the batched
# potentials (covtype's and the whitening's GEMMs) to stream their operand once per many chains
TIMING_CHAINS = 64

# adaptation transitions per config (the reference examples use 1000; bounded so that the
# default bench run stays within a few minutes)
CONFIG_WARMUP = {"c2": 100, "c3": 100, "c4": 200}


def cpu_baseline_config(sp, eng, seed, dev_ns, dev_z, seconds, dev_trace):
    """CPU side of a secondary config (SURVEY.md §8d CPU side 2): `cpu_chains` chains of the C
    restatement of NUTS (oracle/c/nuts_cpu.c, the config's potential in C; dense mass as whitened
    identity-mass chains with the GPU's pooled T, mu) resumed from the GPU's adapted state of the
    first chains on the same Philox stream, running continuously for `seconds`.

    Parity over the first T timed transitions (T = min(steps, sp["parity_transitions"])): the
    reference is the NumPy oracle (oracle/hmc_ref.py) with the potential in rounded float64
    (oracle/batched.py, float64) from the same states; the device's transitions (decision trace
    dev_trace), the NumPy oracle with the float32 batched potential (the rounding calibration) and
    the C restatement (its own decision trace) are each compared with it (oracle/parity.py):
    partings located at their leaf, draws with every decision equal bounded by the calibration's
    drift there, the device's record compared with the calibration's by like_calibration."""
    import numpy as np

    from oracle import batched as OB
    from oracle import cpu_batched as CB
    from oracle import cpu_nuts as CN
    from oracle import parity as PR

    k = min(sp["cpu_chains"], eng.C)
    kt = min(TIMING_CHAINS, eng.C)
    stt = {n: eng.chain_state(n)[:kt].detach().cpu().numpy().copy()
           for n in ("z", "zgrad", "pe", "step_size", "inv_mass", "mass_sqrt")}
    to_model, whiten = None, None
    if eng.dense:
        wt = eng.potential.whitening
        whiten = (wt.T.cpu().numpy(), wt.mu.cpu().numpy())
        stt["inv_mass"] = np.ones_like(stt["z"])  # identity mass on w (unit_mass on the device)
        stt["mass_sqrt"] = np.ones_like(stt["z"])
        f32w = OB.Whitened(sp["cpu"](), *whiten)
        to_model = lambda w: f32w.to_model(np.asarray(w)[None])[0]  # noqa: E731
    st = {n: v[:k] for n, v in stt.items()}  # the parity chains: the first k of them
    cn = CN.CpuNuts(sp["c_model"], *sp["c_args"], whitening=whiten)
    out = _c_baseline(cn, stt, seed, eng.iteration, seconds, chain_offset=eng.chain_offset)
    out["sample"] = (f"reduced C={kt}: {kt} chains of the timed workload (GPU-adapted state, same stream) run "
                     f"continuously for {out['wall_s']:.1f}s: {out['transitions']} transitions = {out['leapfrogs']} "
                     f"leapfrogs; C restatement of NUTS (oracle/c/nuts_cpu.c) with the model's potential in C" +
                     ("; dense mass as the whitened identity-mass chain with the GPU's pooled T, mu (two GEMMs per "
                      "evaluation, OpenMP)" if eng.dense else ""))
    T = min(dev_ns.shape[1], sp.get("parity_transitions", dev_ns.shape[1]))
    label = f"parity {sp['name'].split(',')[0]}"
    f64 = sp["cpu"](np.float64)
    if eng.dense:
        f64 = OB.Whitened(f64, *whiten, dtype=np.float64)
    states, oracles = CB.chains_from_state(st["z"], st["zgrad"], st["pe"], st["step_size"], st["inv_mass"],
                                           st["mass_sqrt"], eng.iteration, seed, eng.num_warmup,
                                           chain_offset=eng.chain_offset)
    t64 = time.perf_counter()
    _, hist64, _, _ = CB.run_chains(f64, states, oracles, T, record=True)
    t64 = time.perf_counter() - t64
    # rounding calibration: the NumPy oracle with the float32 batched potential (oracle/batched.py),
    # the same chains and transitions -- the plain float32 implementation the tests calibrate with
    f32 = sp["cpu"]()
    if eng.dense:
        f32 = OB.Whitened(f32, *whiten)
    states, oracles = CB.chains_from_state(st["z"], st["zgrad"], st["pe"], st["step_size"], st["inv_mass"],
                                           st["mass_sqrt"], eng.iteration, seed, eng.num_warmup,
                                           chain_offset=eng.chain_offset)
    _, hist32, _, _ = CB.run_chains(f32, states, oracles, T, record=True)
    L = dev_trace.shape[2]
    ctr, cns, cz = _oracle_trace(hist32, L)
    if to_model is not None:
        cz = np.stack([[to_model(w) for w in cc] for cc in cz])
    cal = PR.compare_traced(hist64, ctr, cns, cz, atol=1e-3, rtol=1e-3, to_model=to_model, through_draws=True)
    PR.bound_draws(cal, cal)
    # the C restatement over the same transitions (float32 potentials in C, double reductions in the
    # sampler): a third implementation, reported beside the calibration
    c = cn.run(st["z"], st["zgrad"], st["pe"], st["step_size"], st["inv_mass"], st["mass_sqrt"], seed, eng.iteration,
               T, chain_offset=eng.chain_offset, trace=True)
    ccz = c["z"].astype(np.float64)
    if to_model is not None:
        ccz = np.stack([[to_model(w) for w in cc] for cc in ccz])
    crec = PR.compare_traced(hist64, c["trace"][:, :, :L], c["num_steps"], ccz, atol=1e-3, rtol=1e-3,
                             to_model=to_model)
    PR.bound_draws(crec, cal)
    par = _located_parity(hist64, dev_trace, dev_ns[:k, :T], dev_z[:k, :T], atol=1e-3, rtol=1e-3,
                          to_model=to_model, label=label)
    dev_full = PR.compare_traced(hist64, dev_trace, dev_ns[:k, :T], dev_z[:k, :T], atol=1e-3, rtol=1e-3,
                                 to_model=to_model)
    ok, msg = PR.like_calibration(dev_full, cal)
    for m in dev_full["mismatches"]:
        if m["kind"] == "draw":
            print(f"[{label}] " + PR.describe(m), file=sys.stderr)
    print(f"[{label}] {msg}", file=sys.stderr)
    _adopt_draw_bounds(par, dev_full)
    par["basis"] = ("the GPU's timed transitions vs the NumPy oracle NUTS with the potential in rounded float64 (the "
                    f"reference), same chains from the same state on the same Philox stream, first {T} transitions "
                    "per chain; partings located at their leaf; draws with every decision equal bounded by the "
                    f"calibration's drift (DRAW_MULT = {PR.DRAW_MULT})")
    par["calibration"] = {"basis": "the NumPy oracle with the float32 batched potential (oracle/batched.py) vs the "
                                   "same reference", **PR.counts(cal),
                          "max_dE_err": cal["max_dE_err"], "max_dE_rel": cal["max_dE_rel"],
                          "device_like_calibration": ok}
    par["c_restatement"] = {"basis": "oracle/c/nuts_cpu.c (float32 potentials in C, its own decision trace) vs the "
                                     "same reference, its draws bounded by the same calibration", **PR.counts(crec),
                            "max_dE_rel": crec["max_dE_rel"],
                            "geo_mean_drift_ratio": crec["draw_drift"]["geo_mean_ratio"]}
    par["draw_drift"] = dev_full["draw_drift"]
    par["max_dE_rel"], par["worst_dE"] = dev_full["max_dE_rel"], dev_full["worst_dE"]
    par["transitions_per_chain"] = T
    par["reference_seconds"] = t64
    return out, par


def _adopt_draw_bounds(par, full):
    """Copy bound_draws' verdict on each draw mismatch from the full record into the JSON one."""
    import numpy as np

    from oracle import parity as PR

    by = {(m["chain"], m["transition"]): m for m in full["mismatches"]}
    for m in par["mismatches"]:
        f = by.get((m["chain"], m["transition"]))
        if f is not None and m["kind"] == "draw":
            for k in ("cal_drift", "cal_basis", "ratio", "bound", "explained", "drift"):
                if k in f:
                    m[k] = float(f[k]) if isinstance(f[k], (float, np.floating)) else f[k]
    c = PR.counts(par)
    par["unexplained"] = c["unexplained"]


def _oracle_trace(hist, L):
    """An oracle run in the device trace layout (oracle/parity.py oracle_to_trace)."""
    import numpy as np

    from oracle import parity as PR

    C, T = len(hist), min(len(h) for h in hist)
    tr = np.full((T, C, L, 8), np.nan, np.float32)
    ns = np.zeros((C, T), np.int64)
    z = np.zeros((C, T, np.size(hist[0][0][0].z)))
    for c, h in enumerate(hist):
        for t in range(T):
            st_, _, leaves = h[t]
            tr[t, c] = PR.oracle_to_trace(leaves, L)
            ns[c, t] = st_.num_steps
            z[c, t] = st_.z
    return tr, ns, z


def _valu_roofline(path, rank_rate):
    """VALU issue fraction of a kernel that the HBM basis does not bound: the profiled VALU
    wave-instructions per chain-leapfrog (rocprofv3 SQ_INSTS_VALU over the kernel's dispatches,
    committed under profiles/) x this rank's leapfrog rate, against the SIMDs' issue peak of
    one wave64 VALU instruction per 2 cycles (256 CUs x 4 SIMDs, MI355X_MICROARCH.md) at the
    effective clock profiled with it (GRBM_GUI_ACTIVE / 8 / kernel time)."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), path)) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None
    per, clk = prof["valu_wave_insts_per_leapfrog"], prof["effective_clock_ghz"]
    achieved = per * rank_rate / 1e9
    peak = 256 * 4 * 0.5 * clk
    return {"achieved": achieved, "peak": peak, "unit": "G VALU wave-instr/s", "frac": achieved / peak,
            "insts_per_leapfrog": per, "salu_per_leapfrog": prof.get("salu_per_leapfrog"), "clock_ghz": clk,
            "profile_frac": prof.get("valu_issue_frac"), "source": path,
            "basis": "profiled VALU wave-instructions per chain-leapfrog x this rank's leapfrog rate / (1024 SIMDs "
                     "x 0.5 instr/cycle x profiled clock)"}


def secondary_configs(which, rank, world, device, cpu_seconds):
    """Leapfrogs/s of the BASELINE.json secondary configs on synthetic data of their shape:
    adaptation (untimed; its tree sizes and divergences reported), then `steps` transitions
    timed between barrier + synchronize (max over ranks); value = sum(num_steps) over all
    ranks / wall.  At one rank each config also gets its CPU comparator and parity record."""
    import torch
    import torch.distributed as dist

    from numpyro_amd import shard
    from numpyro_amd.infer import MCMC, NUTS, shard_chains
    from numpyro_amd.random import key_to_seed

    out = {}
    specs = _config_specs()
    for key in [k.strip() for k in which.split(",") if k.strip() and k.strip() != "none"]:
        sp = specs[key]
        if sp["one_gpu"] and world > 1:
            continue
        lo, hi = shard_chains(sp["chains"], rank, world)
        # postprocess_fn: the draws stay unconstrained (model coordinates), as the CPU
        # comparator's chains hold them
        # vectorized: this rank's chains on its own GPU (chain_method="parallel" would spread a
        # single process over every visible GPU)
        mcmc = MCMC(NUTS(sp["model"], dense_mass=sp["dense"]), num_warmup=sp["warmup"], num_samples=sp["steps"],
                    num_chains=hi - lo, chain_offset=lo, progress_bar=False, postprocess_fn=_identity,
                    chain_method="vectorized")
        t0 = time.perf_counter()
        mcmc._fields_only = True  # the adaptation's tree sizes and divergences, not its draws
        mcmc.warmup(7, *sp["args"], collect_warmup=True, extra_fields=("num_steps", "diverging"))
        mcmc._fields_only = False
        torch.cuda.synchronize()
        setup_s = time.perf_counter() - t0
        wf = mcmc.get_extra_fields(group_by_chain=True)
        w_ns = wf["num_steps"].to(torch.float64)
        wst = torch.tensor([w_ns.sum().item(), float(wf["diverging"].sum().item())], dtype=torch.float64,
                           device=device)
        # the potential launches (dense: whitening products + model kernel + column packing)
        # timed with HIP events on their stream inside the timed region, as for the headline
        eng = mcmc._engine
        pot = eng.potential
        orig_eval, evs = pot.evaluate, []

        def timed_eval(ev, s, *rest, _orig=orig_eval):
            st = _ext_stream(s)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            _orig(ev, s, *rest)
            b.record(st)
            evs.append((a, b))

        pot.evaluate = timed_eval
        parity_leg = world == 1 and rank == 0 and cpu_seconds > 0
        if parity_leg:  # decision trace of the CPU comparator's chains (parity located per leaf)
            eng.set_trace(min(sp["cpu_chains"], eng.C), eng.iteration, sp["steps"])
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mcmc.run(8, *sp["args"], extra_fields=("num_steps", "diverging", "potential_energy"))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        pot.evaluate = orig_eval
        pot_ms = sum(a.elapsed_time(b) for a, b in evs)
        ef = mcmc.get_extra_fields(group_by_chain=True)
        st = torch.tensor([ef["num_steps"].to(torch.float64).sum().item(), wall,
                           float(ef["diverging"].sum().item())], dtype=torch.float64, device=device)
        if world > 1:
            tot, mx = st.clone(), st.clone()
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(wst)
            leap, wall, div = tot[0].item(), mx[1].item(), tot[2].item()
        else:
            leap, div = st[0].item(), st[2].item()
        n_ch, W = sp["chains"], sp["warmup"]
        r = {"workload": sp["name"], "num_chains": n_ch, "warmup": W, "steps": sp["steps"],
             "value": leap / wall, "unit": "leapfrog/s", "ms_per_step": wall * 1e3 / sp["steps"],
             "mean_tree_size": leap / (n_ch * sp["steps"]), "divergent_frac": div / (n_ch * sp["steps"]),
             "adapt_wall_s": setup_s, "adapt_leapfrogs": wst[0].item(),
             "adapt_leapfrog_per_s": wst[0].item() / setup_s, "adapt_mean_tree_size": wst[0].item() / (n_ch * W),
             "adapt_divergent_frac": wst[1].item() / (n_ch * W), "dense_mass": sp["dense"] or False}
        if "flop" in sp:
            tf = sp["flop"] * leap / wall / 1e12
            peak = MI355X_BF16_MFMA_PEAK_TFLOPS / SPLIT_PRODUCTS
            r["roofline"] = {"bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s", "frac": tf / peak,
                             "basis": sp["basis"] + " over the sampling wall time (split-bf16 whitening GEMMs)"}
            if pot_ms > 0:  # the potential launches alone (rank-local work over rank-local time)
                tp = sp["flop"] * st[0].item() / (pot_ms * 1e-3) / 1e12
                r["roofline"]["potential_launches"] = {
                    "achieved": tp, "frac": tp / peak, "ms_per_launch": pot_ms / len(evs),
                    "basis": "the same FLOPs over the summed durations of the potential launches (whitening "
                             "products + model kernel), HIP events on their stream"}
        else:
            gbs = sp["bytes"] * leap / wall / 1e9
            r["roofline"] = {"bound": "hbm", "achieved": gbs, "peak": MI355X_HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": gbs / MI355X_HBM_PEAK_GBS, "basis": sp["basis"] + " over the sampling wall time"}
            if sp.get("valu_profile"):
                r["roofline"]["valu"] = _valu_roofline(sp["valu_profile"], st[0].item() / wall)
        # end-of-run exchange: cross-chain split R-hat over ranks (+ sample
        # gather for the sharded config); R-hat of the timed draws is the regime check
        torch.cuda.synchronize()
        te = time.perf_counter()
        sm = mcmc.get_samples(group_by_chain=True)
        rh = max(float(shard.split_gelman_rubin(v.reshape(v.shape[0], v.shape[1], -1)).max()) for v in sm.values())
        r["max_split_rhat"] = rh
        if not sp["one_gpu"]:
            # the whole draw set of every site, all_gathered to every rank (SURVEY.md §8e sample gather)
            gathered = {k: shard.gather_chains(v) for k, v in sm.items()}
            torch.cuda.synchronize()
            nbytes = sum(v.numel() * v.element_size() for v in gathered.values())
            r["end_of_run"] = {"ms": (time.perf_counter() - te) * 1e3,
                               "gathered_chains": int(next(iter(gathered.values())).shape[0]),
                               "gathered": f"every site's draws [chains, {sp['steps']}, ...]: {nbytes / 1e6:.0f} MB "
                                           f"on every rank, plus the cross-chain split R-hat",
                               "collective": _collective(world)}
            r["parallelism"] = f"chains sharded {world}-way (no data-path collective)"
            r["scaling"] = "strong"
        if parity_leg:
            k = min(sp["cpu_chains"], eng.C)
            dev_ns = ef["num_steps"][:k].cpu().numpy()
            dev_z = mcmc._samples[:, :, :k].permute(2, 0, 1).to(torch.float64).cpu().numpy()  # model space
            dev_trace = eng.trace_records()
            eng.set_trace(0, 0, 0)
            # resume the CPU chains from the post-warmup state (the timed run moved the engine on)
            from numpyro_amd.infer.hmc import restore_state
            restore_state(eng, mcmc.post_warmup_state)
            cb, par = cpu_baseline_config(sp, eng, key_to_seed(8), dev_ns, dev_z, cpu_seconds, dev_trace)
            r["cpu_baseline"], r["parity"] = cb, par
        out[key] = r
        del mcmc, eng, pot
        torch.cuda.empty_cache()
    return out


def _identity(z):
    return z


def _collective(world):
    if world == 1:
        return "none (1 rank)"
    import torch.distributed as dist

    b = dist.get_backend()
    return "all_reduce + all_gather (" + ("RCCL" if b == "nccl" else b) + ")"


_STREAMS = {}


def _ext_stream(s):
    """torch handle of a raw hipStream_t (the engine's launch streams) for recording events."""
    import torch

    cur = torch.cuda.current_stream()
    if s == cur.cuda_stream:  # (the null stream is 0: an ExternalStream of it records elsewhere)
        return cur
    if s not in _STREAMS:
        _STREAMS[s] = torch.cuda.ExternalStream(s)
    return _STREAMS[s]


def _heartbeat(t_start, period=30.0):
    """A line on stderr every `period` seconds (rank 0): the long untimed phases (adaptation of the
    configs, the CPU baselines) print nothing else for minutes, and runners that watch output take
    a silent process for a hung one.  Daemon thread, stderr only: the JSON line stays alone on stdout."""
    import threading

    def beat():
        while True:
            time.sleep(period)
            print(f"[bench] running, {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    t_start = time.perf_counter()
    args = parse()
    if int(os.environ.get("RANK", "0")) == 0:
        _heartbeat(t_start)
    if args.lib:
        from numpyro_amd import native as _native

        _native.LIB_PATH = os.path.abspath(args.lib)
    import numpy as np
    import torch
    import torch.distributed as dist

    if args.chain_groups is not None:
        from numpyro_amd.engine import Engine

        Engine.chain_groups = args.chain_groups
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # NMX_BENCH_BACKEND=gloo (rehearsal only): run N ranks on fewer GPUs than ranks (rank r on
    # GPU r mod count) with gloo collectives, to exercise the multi-rank bench path on a
    # one-GPU box; the driver's multi-GPU runs use the default, one rank per GPU over RCCL
    backend = os.environ.get("NMX_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    from numpyro_amd import datasets
    from numpyro_amd import potentials as P
    from numpyro_amd.infer import MCMC, NUTS, shard_chains
    from numpyro_amd.random import key_to_seed

    if args.design == "structured":
        X, y = datasets.covtype_structured(n_rows=args.rows, seed=0)
        data_desc = ("synthetic covtype, real-data column structure (10 correlated quantitative + one-hot 4 wilderness "
                     "+ 40 soil types, standardized + intercept; y~Bernoulli(sigmoid(X@ref_coefs)))")
    else:
        X, y = datasets.covtype_synthetic(n_rows=args.rows, seed=0)
        data_desc = "synthetic covtype (581012x54 N(0,1) standardized + intercept, y~Bernoulli(sigmoid(X@ref_coefs)))"
    lo, hi = shard_chains(args.chains, rank, world)
    kernel = NUTS(P.logistic_regression)
    mcmc = MCMC(kernel, num_warmup=args.adapt, num_samples=args.warmup, num_chains=hi - lo,
                chain_offset=lo, chain_method="vectorized", progress_bar=False,
                sync_chains=args.sync_chains)
    Xd = torch.from_numpy(X).to(device)
    yd = torch.from_numpy(y).to(device)
    # untimed: init + adaptation, then the untimed sampling transitions
    mcmc.warmup(args.seed, Xd, yd)
    if args.warmup > 0:
        mcmc.run(args.seed + 1, Xd, yd)
        mcmc.post_warmup_state = mcmc.last_state
    start_state = mcmc.post_warmup_state
    mcmc.num_samples = args.steps
    eng = mcmc._engine
    pot = eng.potential
    # time the potential launches inside the timed region with events on the stream each is
    # launched on (chain groups use one stream each)
    evs = []
    orig_eval = pot.evaluate

    def timed_eval(ev, s, *rest):
        st = _ext_stream(s)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(st)
        orig_eval(ev, s, *rest)
        b.record(st)
        evs.append((a, b))

    pot.evaluate = timed_eval
    parity_leg = not args.no_cpu_baseline and world == 1
    if parity_leg:  # decision trace of the CPU comparator's chains (parity located per leaf)
        eng.set_trace(min(args.cpu_chains, hi - lo), eng.iteration, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mcmc.run(args.seed + 2, Xd, yd, extra_fields=("num_steps", "diverging", "potential_energy"))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pot.evaluate = orig_eval
    elapsed = t1 - t0
    # end-of-run exchange: cross-chain R-hat / ESS by all_reduce of per-chain
    # statistics and the sample gather (RCCL under torch.distributed); reported, not in `value`
    from numpyro_amd import shard

    torch.cuda.synchronize()
    te0 = time.perf_counter()
    site = mcmc.get_samples(group_by_chain=True)["coefs"]
    rhat = shard.split_gelman_rubin(site) if site.shape[1] >= 4 else None
    ess = shard.effective_sample_size(site)
    gathered = shard.gather_chains(site)
    torch.cuda.synchronize()
    end_of_run_ms = (time.perf_counter() - te0) * 1e3
    ef = mcmc.get_extra_fields(group_by_chain=True)
    ns = ef["num_steps"].to(torch.float64)  # [C_local, steps]
    num_steps = ns.sum()
    launches = mcmc.last_run_stats["launches"]
    pot_ms = sum(a.elapsed_time(b) for a, b in evs)
    stats = torch.tensor([num_steps.item(), elapsed, pot_ms, float(len(evs)), float(launches),
                          float(ef["diverging"].sum().item())], dtype=torch.float64, device=device)
    tree_max = ns.max(0).values.to(device)  # per timed transition: the largest tree of the shard
    if world > 1:
        tot = stats.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(tree_max, op=dist.ReduceOp.MAX)
        useful, elapsed, divergent = tot[0].item(), mx[1].item(), tot[5].item()
    else:
        useful, divergent = stats[0].item(), stats[5].item()
    value = useful / elapsed
    # dominant kernel: fused logreg potential (two f32 MFMA GEMMs), algorithmic FLOPs per
    # chain-leapfrog = 4 N D; one launch evaluates every LEAF chain.
    local_useful = stats[0].item()
    flop = 4.0 * args.rows * X.shape[1] * local_useful
    achieved = flop / (pot_ms * 1e-3) / 1e12 if pot_ms > 0 else 0.0
    peak = MI355X_BF16_MFMA_PEAK_TFLOPS / SPLIT_PRODUCTS
    traffic = None
    try:
        with open(args.traffic_json) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        traffic = None
    if rank == 0:
        out = {
            "metric": "leapfrog steps/sec across 4096 NUTS chains (covtype LR)",
            "value": value,
            "unit": "leapfrog/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data_desc,
            "config": {"workload": "covtype logistic regression NUTS, diag mass, max_tree_depth 10",
                       "num_chains": args.chains, "rows": args.rows, "dim": int(X.shape[1]),
                       "adapt_transitions": args.adapt, "design": args.design,
                       "parallelism": f"chains sharded {world}-way (no data-path collective)",
                       "schedule": "lockstep" if args.sync_chains else "per-chain async",
                       "chain_groups": eng._groups()},
            "useful_leapfrogs": useful,
            "mean_tree_size": useful / (args.chains * args.steps),
            "divergent_frac": divergent / (args.chains * args.steps),
            "lockstep_equivalent_leapfrogs": float(tree_max.sum().item()) * args.chains,
            "evaluated_leapfrogs": useful,
            "leapfrog_launches": launches,
            "chain_slot_occupancy": local_useful / max(1, launches * (hi - lo)),
            "potential_ms_per_launch": pot_ms / max(1, len(evs)),
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak,
                         "unit": "TFLOP/s", "frac": achieved / peak, "traffic": traffic,
                         "kernel": "k_logreg_x3 + k_logreg_finalize",
                         "peak_basis": ("bf16 MFMA 2500 TF/s / 6 split products (f32 operands as three bf16 terms, "
                                        "f32 accumulation); achieved = algorithmic 4*N*D f32 FLOP per chain-leapfrog"),
                         "frac_of_f32_mfma_peak": achieved / MI355X_FP32_MFMA_PEAK_TFLOPS},
            "cpu_baseline": None,
            "end_of_run": {"ms": end_of_run_ms, "gathered_chains": int(gathered.shape[0]),
                           "max_split_rhat": float(rhat.max()) if rhat is not None else None,
                           "min_ess": float(ess.min()),
                           "collective": _collective(world)},
        }
        if parity_leg:
            k = min(args.cpu_chains, hi - lo)
            cb = cpu_baseline(X, y, start_state, key_to_seed(args.seed + 2), args.adapt + args.warmup, args.adapt, k,
                              args.cpu_seconds, dev_ns=ns[:k].cpu().numpy(),
                              dev_z=site[:k].to(torch.float64).cpu().numpy(), dev_trace=eng.trace_records())
            out["parity"] = cb.pop("parity")
            out["cpu_baseline"] = cb
    eng.set_trace(0, 0, 0)
    if args.configs != "none":
        del mcmc, eng, pot, start_state
        torch.cuda.empty_cache()
        cfgs = secondary_configs(args.configs, rank, world, device,
                                 0.0 if args.no_cpu_baseline else args.config_cpu_seconds)
        if rank == 0:
            out["configs"] = cfgs
    if rank == 0:
        out["bench_wall_s"] = time.perf_counter() - t_start
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
