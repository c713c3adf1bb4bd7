"""Throughput of the BASELINE.json secondary configs (one GPU), plus kernel microbenchmarks.

    python scripts/bench_configs.py gemm  [D] [C]          # nmx_gemm_chains alone
    python scripts/bench_configs.py chainmv [D] [--chains C]  # per-chain dense matvec (HBM)
    python scripts/bench_configs.py funnel [--dim 10000 --chains 4096 --warmup W --steps K]
    python scripts/bench_configs.py sv     [--chains 1024 ...]
    python scripts/bench_configs.py bnn    [--chains 2048 ...]
    python scripts/bench_configs.py covtype [--chains 1024 ...]

Each model run does `mcmc.warmup` (untimed) then times `mcmc.run` between synchronizes and
prints one JSON line: leapfrogs/s (= sum num_steps / wall), average potential-launch time
(HIP events on the launch stream) and the roofline fraction of the dominant kernel.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import datasets, native  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402

PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def bench_gemm(D, C, reps=10, tri=0, x3=False):
    dev = torch.device("cuda:0")
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    ldc = (C + 63) // 64 * 64
    A = torch.randn(D, D, device=dev)
    A = {0: A, 1: torch.triu(A), 2: torch.tril(A)}[tri]
    At = torch.zeros(lda, lda, device=dev)
    At[:D, :D] = A.t()
    x = torch.randn(D, ldc, device=dev)
    y = torch.empty(D, ldc, device=dev)
    s = native.stream_ptr()
    nws = lib.nmx_gemm_chains_workspace_bytes(D, ldc)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev) if nws else None
    if x3:
        Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=dev)
        sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=dev)
        native.check(lib.nmx_gemm_x3_pack_a(native.ptr(At), lda, native.ptr(Ap), s))

    def run():
        if x3:
            native.check(lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(x), native.ptr(y), None, tri, ldc,
                                                None, None, C, native.ptr(sp), native.ptr(ws), s))
        else:
            native.check(lib.nmx_gemm_chains(native.ptr(At), lda, D, native.ptr(x), native.ptr(y), None, tri, ldc,
                                             None, None, C, native.ptr(ws), s))

    for _ in range(2):
        run()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        run()
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    tf = (2.0 if tri == 0 else 1.0) * D * D * C / (ms * 1e-3) / 1e12  # triangular: D^2 C useful
    ref = (At[:D, :D].t().double() @ x[:, :8].double())
    err = float((y[:, :8].double() - ref).abs().max() / ref.abs().max())
    print(json.dumps({"kernel": "k_gemm_x3" if x3 else "k_gemm_chains", "triangle": tri, "D": D, "C": C, "ms": round(ms, 4),
                      "useful_tflops": round(tf, 2), "frac": round(tf / PEAK_F32_TFLOPS, 3), "max_rel_err": err}),
          flush=True)


def bench_chain_matvec(D, C, reps=10):
    """nmx_chain_matvec_tri (per-chain dense mass, every chain listed): HBM-bound, each chain's
    triangle of T_c (2 D^2 B f32 of the D^2 stored) read once per product, plus the in / out
    vectors; reported against 8 TB/s on that algorithmic basis."""
    dev = torch.device("cuda:0")
    lib = native.lib()
    ldc = (C + 63) // 64 * 64
    M = torch.triu(torch.randn(C, D, D, device=dev)).transpose(1, 2).contiguous()  # T_c^T, T_c upper
    x = torch.randn(D, ldc, device=dev)
    y = torch.empty(D, ldc, device=dev)
    s = native.stream_ptr()
    out = {}
    for tri in (0, 1):
        def run():
            native.check(lib.nmx_chain_matvec_tri(native.ptr(M), D, native.ptr(x), native.ptr(y), ldc, None, None,
                                                  None, C, tri, s))
        for _ in range(2):
            run()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            run()
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / reps
        mbytes = (4.0 * D * D if tri == 0 else 2.0 * D * (D + 1)) * C + 8.0 * D * C
        ref = torch.einsum("cba,bc->ac", M[:4].double(), x[:, :4].double())
        err = float((y[:, :4].double() - ref).abs().max() / ref.abs().max())
        out["full" if tri == 0 else "triangular"] = {"ms": round(ms, 4), "GBs": round(mbytes / (ms * 1e-3) / 1e9, 1),
                                                     "frac": round(mbytes / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 3),
                                                     "max_rel_err": err}
    print(json.dumps({"kernel": "nmx_chain_matvec_tri", "D": D, "C": C, **out}), flush=True)


class Timed:
    """Wraps Potential.evaluate with HIP events on the launch stream."""

    def __init__(self, pot):
        self.pot, self.orig, self.events = pot, pot.evaluate, []
        self.on = False
        self.streams = {}
        pot.evaluate = self

    def __call__(self, ev, s, *rest):
        if not self.on:
            return self.orig(ev, s, *rest)
        st = torch.cuda.current_stream()  # the launch stream (its own for chain groups > 0)
        if s != st.cuda_stream:
            st = self.streams.setdefault(s, torch.cuda.ExternalStream(s))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        self.orig(ev, s, *rest)
        b.record(st)
        self.events.append((a, b))

    def total_ms(self):
        return sum(a.elapsed_time(b) for a, b in self.events)


def run_model(name, model, args, chains, warmup, steps, flops_per_leapfrog=None, bytes_per_leapfrog=None,
              **kernel_kw):
    kernel = NUTS(model, **kernel_kw)
    mcmc = MCMC(kernel, num_warmup=warmup, num_samples=steps, num_chains=chains, progress_bar=False,
                chain_method="vectorized")
    t0 = time.time()
    mcmc._fields_only = True  # warmup transitions' fields (tree sizes, divergences), no draws
    mcmc.warmup(0, *args, collect_warmup=True, extra_fields=("num_steps", "diverging"))
    mcmc._fields_only = False
    torch.cuda.synchronize()
    t_warm = time.time() - t0
    wf = mcmc.get_extra_fields(group_by_chain=True)
    w_ns = wf["num_steps"].to(torch.float64)
    warm = {"warmup_leapfrogs": int(w_ns.sum().item()), "warmup_leapfrog_per_s": round(float(w_ns.sum()) / t_warm, 1),
            "warmup_mean_tree_per_window_third": [round(float(x.mean()), 1) for x in w_ns.chunk(3, dim=1)],
            "warmup_divergent_frac": round(float(wf["diverging"].float().mean()), 4)}
    eng = mcmc._engine
    timer = Timed(eng.potential)
    timer.on = True
    torch.cuda.synchronize()
    t0 = time.time()
    mcmc.run(1, *args, extra_fields=("num_steps", "diverging"))
    torch.cuda.synchronize()
    wall = time.time() - t0
    timer.on = False
    ns = int(mcmc.get_extra_fields()["num_steps"].sum().item())
    from numpyro_amd import shard
    sm = mcmc.get_samples(group_by_chain=True)
    rh = max(float(shard.split_gelman_rubin(v.reshape(v.shape[0], v.shape[1], -1)).max()) for v in sm.values()) \
        if steps >= 4 else None
    warm.update({"divergent_frac": round(float(mcmc.get_extra_fields()["diverging"].float().mean()), 4),
                 "max_split_rhat": rh, "mean_tree": round(ns / (chains * steps), 1)})
    pot_ms = timer.total_ms()
    launches = len(timer.events)
    out = {"config": name, "chains": chains, "dim": eng.D, "warmup": warmup, "steps": steps,
           "leapfrogs": ns, "wall_s": round(wall, 3), "leapfrog_per_s": round(ns / wall, 1),
           "launches": launches, "potential_ms_avg": round(pot_ms / max(launches, 1), 4),
           "potential_share": round(pot_ms / 1e3 / wall, 3), "warmup_wall_s": round(t_warm, 2),
           "dense": bool(eng.dense), **warm}
    if flops_per_leapfrog:
        tf = flops_per_leapfrog * ns / (pot_ms * 1e-3) / 1e12
        peak = PEAK_F32_TFLOPS
        if name == "covtype" or eng.dense:
            peak = 2500.0 / 6  # split-bf16 products: bf16 MFMA peak / 6 (bench.py)
        out["roofline"] = {"bound": "mfma", "achieved_tflops": round(tf, 2), "peak": round(peak, 1),
                           "frac": round(tf / peak, 3)}
    if bytes_per_leapfrog:
        # SURVEY.md §8d (C2 diag / C4): algorithmic bytes per chain-leapfrog 7 D x 4 B (z, r, g
        # read + write, inverse mass read) over the sampling wall time (the whole step loop)
        gbs = 7 * 4 * eng.D * ns / wall / 1e9
        out["roofline"] = {"bound": "hbm", "achieved_GBs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 3),
                           "basis": "7*D*4 B per chain-leapfrog / sampling wall time"}
        if pot_ms > 0:  # launched loop: the potential kernels alone (read z, write grad)
            out["roofline"]["potential_GBs"] = round(bytes_per_leapfrog * ns / (pot_ms * 1e-3) / 1e9, 1)
        out["fused_wide"] = launches == 0
        out["schedule"] = "persistent" if getattr(eng, "crow", False) else ("fused" if launches == 0 else "launched")
    print(json.dumps(out), flush=True)
    return mcmc


def main():
    p = argparse.ArgumentParser()
    p.add_argument("what")
    p.add_argument("rest", nargs="*")
    p.add_argument("--chains", type=int, default=None)
    p.add_argument("--dim", type=int, default=10000)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--max-tree-depth", type=int, default=10)
    p.add_argument("--dense", type=int, default=1)
    p.add_argument("--launched", action="store_true", help="wide models: potential + step loop (A/B)")
    p.add_argument("--fused", action="store_true", help="wide models: the launched fused step, not the persistent one")
    p.add_argument("--slices", action="store_true", help="dense wide models: the D-slice step kernels (A/B)")
    p.add_argument("--lib", default=None, help="A/B: load this build of libnumpyro_amd.so")
    a = p.parse_args()
    if a.lib:
        native.LIB_PATH = os.path.abspath(a.lib)
    if a.slices:
        from numpyro_amd.engine import Engine
        Engine.chain_rows_step = False
    if a.launched or a.fused:
        from numpyro_amd.engine import Engine
        Engine.wide_persistent = False
        Engine.fused_wide = not a.launched
    if a.what == "gemm":
        D = int(a.rest[0]) if a.rest else 10000
        C = int(a.rest[1]) if len(a.rest) > 1 else 4096
        for x3 in (False, True):
            bench_gemm(D, C, x3=x3)
            bench_gemm(D, C, tri=1, x3=x3)
            bench_gemm(D, C, tri=2, x3=x3)
    elif a.what == "chainmv":
        for D in ([int(a.rest[0])] if a.rest else [512, 1024, 2048, 4096]):
            bench_chain_matvec(D, a.chains or (256 if D <= 1024 else 64))
    elif a.what == "funnel":
        D = a.dim
        # dense: two triangular products z = T w, g = T^T g_z (D^2 FLOP each per chain)
        run_model("funnel", P.funnel, (D,), a.chains or 4096, a.warmup, a.steps,
                  flops_per_leapfrog=2.0 * D * D if a.dense else None,
                  bytes_per_leapfrog=None if a.dense else 2 * D * 4,
                  dense_mass="pooled" if a.dense else False, max_tree_depth=a.max_tree_depth)
    elif a.what == "sv":
        r = datasets.sp500_synthetic()
        D = r.size + 2
        run_model("stochastic_volatility", P.stochastic_volatility, (r,), a.chains or 1024, a.warmup, a.steps,
                  bytes_per_leapfrog=2 * D * 4, max_tree_depth=a.max_tree_depth)
    elif a.what == "bnn":
        X, Y = datasets.bnn_data(N=100, D_X=3)
        H = 69
        D = 1 + 3 * H + H * H + H
        model_flops = 6.0 * 100 * H * H + 6.0 * 100 * 3 * H
        run_model("bnn", P.bnn, (X, Y, H), a.chains or 2048, a.warmup, a.steps,
                  flops_per_leapfrog=(2.0 * D * D if a.dense else 0.0) + model_flops,
                  dense_mass="pooled" if a.dense else False, max_tree_depth=a.max_tree_depth)
    elif a.what == "covtype":
        X, y = datasets.covtype_synthetic(seed=0)
        dev = torch.device("cuda:0")
        Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
        run_model("covtype", P.logistic_regression, (Xd, yd), a.chains or 1024, a.warmup, a.steps,
                  flops_per_leapfrog=4.0 * X.shape[0] * X.shape[1], max_tree_depth=a.max_tree_depth)
    else:
        raise SystemExit(f"unknown config {a.what}")


if __name__ == "__main__":
    main()
