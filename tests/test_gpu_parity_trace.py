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
leaf's bound (hmc_util.py:984-1085 _iterative_build_subtree, :1088-1180 build_tree).  The
fixed-step cases of every schedule are tests/test_gpu_nuts.py test_engine_matches_oracle_fixed_step;
the shared machinery is tests/parity_cases.py."""
import numpy as np
import pytest
import torch

from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS
from oracle import parity as PR
from parity_cases import as_trace as _as_trace
from parity_cases import engine_fixed as _engine_fixed
from parity_cases import f32 as _f32
from parity_cases import oracle_runs as _oracle_runs
from parity_cases import report as _report
from parity_cases import second_f32 as _second_f32

pytestmark = pytest.mark.gpu


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
    cal = PR.compare_traced(hist, ctr, cns, cz, atol=2e-3, rtol=2e-3, through_draws=True)
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
    _, hist32, evals, _ = CB.run_chains(f, states, oracles, T, record=True)
    to_model = lambda w: f.to_model(np.asarray(w)[None])[0]  # noqa: E731
    print(f"[bnn pooled dense D=5038] {evals} oracle leapfrogs, device trees {ns.tolist()}")
    # the reference: the oracle in rounded float64 (network and whitening) from the same states;
    # the float32 NumPy batch above is the rounding calibration against it
    f64 = OB.Whitened(OB.BNNBatch(X, Y, Hh, dtype=np.float64), wt.T.cpu().numpy(), wt.mu.cpu().numpy(),
                      dtype=np.float64)
    states, oracles = CB.chains_from_state(st["z"], st["zgrad"], st["pe"], st["step_size"], ones, ones, W,
                                           seed + 1, W)
    _, hist, _, _ = CB.run_chains(f64, states, oracles, T, record=True)
    par = PR.compare_traced(hist, eng.trace_records(), ns, zdev, atol=1e-3, rtol=1e-3, to_model=to_model)
    ctr, cns, cz = _as_trace(hist32)
    cal = PR.compare_traced(hist, ctr, cns, np.stack([[to_model(w) for w in cc] for cc in cz]), atol=1e-3,
                            rtol=1e-3, to_model=to_model, through_draws=True)
    _report(par, "bnn pooled dense D=5038", cal=cal)
