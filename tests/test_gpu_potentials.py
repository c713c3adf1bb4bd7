"""Fused potential kernels vs the oracle (oracle/potentials.py), on the GPU through the C-ABI.

Tolerances (fp32 kernels vs float64 oracle): pe relative 2e-5 (logreg sums up to 1e5 rows),
grad |g - g_ref| <= 1e-4 * (|g_ref| + sum_n |x_n|) -- the f32 MFMA k-ordered fma chains
carry ~1e-7 relative error per term (cdna_hip_programming.md §3 'FP32-input MFMA').
"""
import ctypes

import numpy as np
import pytest

from numpyro_amd import datasets
from oracle import potentials as OP

pytestmark = pytest.mark.gpu


def _eval(pot, Z, device, phase=None):
    import torch

    from numpyro_amd import native

    C, D = Z.shape
    ldc = (C + 63) // 64 * 64
    pot.bind(C, ldc, device)
    z = torch.zeros(D, ldc, device=device)
    z[:, :C] = torch.from_numpy(Z.T.astype(np.float32)).to(device)
    g = torch.full((D, ldc), float("nan"), device=device)
    pe = torch.full((ldc,), float("nan"), device=device)
    ph = None
    if phase is not None:
        ph = torch.zeros(ldc, dtype=torch.int32, device=device)
        ph[:C] = torch.from_numpy(phase.astype(np.int32)).to(device)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), phase=native.ptr(ph),
                          num_chains=C, ldc=ldc)
    pot.evaluate(ev, native.stream_ptr())
    torch.cuda.synchronize()
    return pe[:C].cpu().numpy().astype(np.float64), g[:, :C].cpu().numpy().T.astype(np.float64)


@pytest.mark.parametrize("N,D,C", [(1000, 55, 200), (517, 5, 64), (3000, 33, 130), (64, 2, 1),
                                   (20000, 55, 256)])
def test_logreg_matches_oracle(device, N, D, C):
    from numpyro_amd.potentials import LogisticRegression

    rs = np.random.RandomState(N + D)
    X = rs.randn(N, D).astype(np.float32)
    y = (rs.rand(N) < 0.4).astype(np.float32)
    Z = (rs.randn(C, D) * 0.3).astype(np.float32)
    pe, g = _eval(LogisticRegression(X, y), Z, device)
    ref = OP.LogisticRegression(X.astype(np.float64), y.astype(np.float64))
    pe_r, g_r = ref.pe_grad_batch(Z.astype(np.float64))
    np.testing.assert_allclose(pe, pe_r, rtol=2e-5, atol=1e-3)
    scale = np.abs(g_r) + np.abs(X).sum(0)[None, :]
    assert np.all(np.abs(g - g_r) <= 1e-4 * scale), np.max(np.abs(g - g_r) / scale)


def test_logreg_covtype_shape_at_scale(device):
    """Full covtype row count (581012 x 55), 128 chains: size-independent checks plus a
    float64 reference on the same synthetic data."""
    from numpyro_amd.potentials import LogisticRegression

    X, y = datasets.covtype_synthetic(seed=0)
    rs = np.random.RandomState(5)
    Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.01 * rs.randn(128, 55)).astype(np.float32)
    pe, g = _eval(LogisticRegression(X, y), Z, device)
    ref = OP.LogisticRegression(X, y)
    pe_r, g_r = ref.pe_grad_batch(Z.astype(np.float64))
    np.testing.assert_allclose(pe, pe_r, rtol=2e-6)
    scale = np.abs(g_r) + np.abs(X).sum(0)[None, :]
    assert np.all(np.abs(g - g_r) <= 2e-5 * scale)


def test_logreg_skips_inactive_chains(device):
    from numpyro_amd.potentials import LogisticRegression

    rs = np.random.RandomState(3)
    X = rs.randn(700, 7).astype(np.float32)
    y = (rs.rand(700) < 0.5).astype(np.float32)
    Z = rs.randn(300, 7).astype(np.float32)
    phase = np.full(300, 3)
    phase[:150] = 0  # first 150 chains inactive (whole chain groups skipped)
    pe, g = _eval(LogisticRegression(X, y), Z, device, phase=phase)
    pe_r, g_r = OP.LogisticRegression(X, y).pe_grad_batch(Z)
    assert np.all(np.isnan(pe[:128]))  # a fully inactive workgroup writes nothing
    np.testing.assert_allclose(pe[150:], pe_r[150:], rtol=2e-5)
    np.testing.assert_allclose(g[150:], g_r[150:], rtol=1e-3, atol=1e-2)


def test_logreg_split_invariance(device):
    """A chain's U/dU must not depend on how many chains share the launch (bitwise)."""
    from numpyro_amd.potentials import LogisticRegression

    rs = np.random.RandomState(4)
    X = rs.randn(5000, 55).astype(np.float32)
    y = (rs.rand(5000) < 0.5).astype(np.float32)
    Z = rs.randn(300, 55).astype(np.float32) * 0.1
    pe_a, g_a = _eval(LogisticRegression(X, y), Z, device)
    pe_b, g_b = _eval(LogisticRegression(X, y), Z[200:260], device)
    np.testing.assert_array_equal(pe_a[200:260], pe_b)
    np.testing.assert_array_equal(g_a[200:260], g_b)


@pytest.mark.parametrize("n_rows", [4001, 70001, 581012])
def test_logreg_tail_forms_are_bitwise_the_full_kernel(device, n_rows):
    """Launches over <= 256 chains run the role-split tail form; the chains of a 300-chain
    launch (the full split-bf16 kernel) get bitwise the same U / dU from it: one chain, one
    chain tile, two chain groups; ragged row counts (a short last split, padded tile rows)
    up to the covtype size."""
    from numpyro_amd.potentials import LogisticRegression

    rs = np.random.RandomState(n_rows % 1000)
    X = rs.randn(n_rows, 55).astype(np.float32)
    y = (rs.rand(n_rows) < 0.4).astype(np.float32)
    Z = rs.randn(300, 55).astype(np.float32) * 0.05
    pot = LogisticRegression(X, y)
    pe_a, g_a = _eval(pot, Z, device)
    for lo, hi in ((7, 8), (200, 232), (0, 256)):
        pe_b, g_b = _eval(pot, Z[lo:hi], device)
        np.testing.assert_array_equal(pe_a[lo:hi], pe_b, err_msg=f"chains {lo}:{hi}")
        np.testing.assert_array_equal(g_a[lo:hi], g_b, err_msg=f"chains {lo}:{hi}")
    if n_rows <= 70001:
        pe_r, g_r = OP.LogisticRegression(X, y).pe_grad_batch(Z[:8])
        np.testing.assert_allclose(pe_a[:8], pe_r, rtol=2e-5)
        np.testing.assert_allclose(g_a[:8], g_r, rtol=1e-3, atol=1e-2)


def _eval_list(pot, Z, idx, device):
    """The potential of the chains idx (a compacted active list, count = len(idx)) inside a
    batch of every chain of Z, as the NUTS loop evaluates them: U / dU at the chains' columns."""
    import torch

    from numpyro_amd import native

    C, D = Z.shape
    ldc = (C + 63) // 64 * 64
    pot.bind(C, ldc, device)
    z = torch.zeros(D, ldc, device=device)
    z[:, :C] = torch.from_numpy(Z.T.astype(np.float32)).to(device)
    g = torch.full((D, ldc), float("nan"), device=device)
    pe = torch.full((ldc,), float("nan"), device=device)
    lst = torch.zeros(ldc, dtype=torch.int32, device=device)
    lst[:len(idx)] = torch.as_tensor(np.asarray(idx, np.int32), device=device)
    cnt = torch.tensor([len(idx)], dtype=torch.int32, device=device)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(lst),
                          active_count=native.ptr(cnt), num_chains=len(idx), ldc=ldc)
    pot.evaluate(ev, native.stream_ptr())
    torch.cuda.synchronize()
    return pe[idx].cpu().numpy().astype(np.float64), g[:, idx].cpu().numpy().T.astype(np.float64)


@pytest.mark.parametrize("n_rows", [4001, 70001, 581012])
def test_logreg_listed_tail_forms_are_bitwise_the_full_kernel(device, n_rows):
    """Compacted lists of <= 32 chains (the narrow form: one chain tile on four waves), 33-256
    chains (the role-split form) and a wide list (the full kernel's early-exit groups): every
    listed chain's U / dU bitwise equal to the full kernel's over the whole batch, for scattered
    chain indices and ragged row counts (short last split, odd tile counts)."""
    from numpyro_amd.potentials import LogisticRegression

    rs = np.random.RandomState(n_rows % 997)
    X = rs.randn(n_rows, 55).astype(np.float32)
    y = (rs.rand(n_rows) < 0.4).astype(np.float32)
    Z = rs.randn(300, 55).astype(np.float32) * 0.05
    pot = LogisticRegression(X, y)
    pe_a, g_a = _eval(pot, Z, device)
    perm = rs.permutation(300)
    for n in (1, 7, 32, 33, 200, 300):
        idx = np.sort(perm[:n]) if n % 2 else perm[:n]
        pe_b, g_b = _eval_list(pot, Z, idx, device)
        np.testing.assert_array_equal(pe_a[idx], pe_b, err_msg=f"{n} listed chains")
        np.testing.assert_array_equal(g_a[idx], g_b, err_msg=f"{n} listed chains")


def test_eight_schools_matches_oracle(device):
    from numpyro_amd.potentials import EightSchools

    rs = np.random.RandomState(0)
    Z = rs.uniform(-2, 2, (100, 10)).astype(np.float32)
    pe, g = _eval(EightSchools(8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y), Z, device)
    ref = OP.EightSchools(datasets.EIGHT_SCHOOLS_Y, datasets.EIGHT_SCHOOLS_SIGMA)
    for c in range(100):
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        np.testing.assert_allclose(pe[c], pr, rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(g[c], gr, rtol=1e-4, atol=1e-4)


def test_diag_normal(device):
    from numpyro_amd.potentials import DiagNormal

    mu = np.array([1.0, -2.0, 0.5], np.float32)
    sd = np.array([0.5, 2.0, 1.0], np.float32)
    Z = np.random.RandomState(0).randn(70, 3).astype(np.float32)
    pe, g = _eval(DiagNormal(mu, sd), Z, device)
    ref = OP.IsoNormal(mu, sd)
    for c in range(70):
        pr, gr = ref.pe_grad(Z[c])
        np.testing.assert_allclose(pe[c], pr, rtol=1e-5)
        np.testing.assert_allclose(g[c], gr, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("which", ["logreg", "eight_schools"])
def test_compacted_active_list_is_bitwise_equal_to_dense(device, which):
    """Potentials evaluated through the nuts_step's compacted chain list (arbitrary order)
    give bitwise the dense results for the listed chains and leave the others untouched."""
    import torch

    from numpyro_amd import native
    from numpyro_amd.potentials import EightSchools, LogisticRegression

    rs = np.random.RandomState(9)
    if which == "logreg":
        X = rs.randn(4000, 55).astype(np.float32)
        y = (rs.rand(4000) < 0.5).astype(np.float32)
        pot, D = LogisticRegression(X, y), 55
    else:
        pot, D = EightSchools(8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y), 10
    C = 300
    Z = (0.1 * rs.randn(C, D)).astype(np.float32)
    pe_dense, g_dense = _eval(pot, Z, device)
    ldc = 320
    pot.bind(C, ldc, device)
    z = torch.zeros(D, ldc, device=device)
    z[:, :C] = torch.from_numpy(Z.T.copy()).to(device)
    g = torch.full((D, ldc), float("nan"), device=device)
    pe = torch.full((ldc,), float("nan"), device=device)
    chosen = rs.permutation(C)[:77]
    idx = torch.zeros(ldc, dtype=torch.int32, device=device)
    idx[:77] = torch.from_numpy(chosen.astype(np.int32)).to(device)
    cnt = torch.tensor([77], dtype=torch.int32, device=device)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(idx),
                          active_count=native.ptr(cnt), num_chains=C, ldc=ldc)
    pot.evaluate(ev, native.stream_ptr())
    torch.cuda.synchronize()
    pe_l = pe[:C].cpu().numpy().astype(np.float64)
    g_l = g[:, :C].cpu().numpy().T.astype(np.float64)
    np.testing.assert_array_equal(pe_l[chosen], pe_dense[chosen])
    np.testing.assert_array_equal(g_l[chosen], g_dense[chosen])
    others = np.setdiff1d(np.arange(C), chosen)
    assert np.all(np.isnan(pe_l[others]))


def test_sv_row_exp_is_bitwise_expf(device):
    """The SV row's exp (nmx_expf_unchecked: expf's reduction without its range selects) equals the
    device expf bit for bit over |x| <= 87, the range -2 s of a stochastic-volatility row spans."""
    import torch

    from numpyro_amd import native

    rs = np.random.RandomState(0)
    xs = np.concatenate([np.linspace(-87.0, 87.0, 200001), rs.uniform(-30, 30, 100000),
                         rs.standard_normal(100000) * 1e-3, [0.0, -0.0, 1e-30, -1e-30]]).astype(np.float32)
    x = torch.from_numpy(xs).to(device)
    fast, ref = torch.empty_like(x), torch.empty_like(x)
    native.check(native.lib().nmx_selftest_expf(native.ptr(x), native.ptr(fast), native.ptr(ref), x.numel(),
                                                native.stream_ptr()))
    torch.cuda.synchronize()
    same = (fast.view(torch.int32) == ref.view(torch.int32)).cpu().numpy()
    assert same.all(), f"{(~same).sum()} of {same.size} differ, first at x = {xs[~same][:5]}"


def test_stochastic_volatility_matches_oracle(device):
    """examples/stochastic_volatility.py model at the SP500 length (T = 2517, D = 2519).
    U sums ~3T terms of magnitude up to ~10 with cancellation, so the fp32 tolerance is
    absolute: |dU| <= 2e-2 (~ T * eps_f32 * 10 with margin) plus 1e-6 |U| (the f32 ulp of
    the result itself when sigma is small and U reaches ~3e5)."""
    from numpyro_amd.potentials import StochasticVolatility

    r = datasets.sp500_synthetic()
    rs = np.random.RandomState(0)
    C = 70
    Z = np.empty((C, r.size + 2), np.float32)
    Z[:, 0] = rs.uniform(0.5, 3.5, C)        # log nu
    Z[:, -1] = rs.uniform(-5.0, -2.0, C)     # log sigma
    Z[:, 1:-1] = (np.log(np.abs(r)).mean() + np.cumsum(0.05 * rs.randn(C, r.size), axis=1)).astype(np.float32)
    pe, g = _eval(StochasticVolatility(r), Z, device)
    ref = OP.StochasticVolatility(r)
    for c in range(C):
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        np.testing.assert_allclose(pe[c], pr, rtol=1e-6, atol=2e-2)  # fp32 ulp of |U| ~ 3e5 is 0.03
        np.testing.assert_allclose(g[c], gr, rtol=2e-3, atol=2e-2 + 2e-4 * np.abs(gr).max())


@pytest.mark.parametrize("dim", [10, 10000])
def test_funnel_matches_oracle(device, dim):
    from numpyro_amd.potentials import Funnel

    rs = np.random.RandomState(dim)
    Z = rs.uniform(-2, 2, (65, dim)).astype(np.float32)
    pe, g = _eval(Funnel(dim), Z, device)
    ref = OP.Funnel(dim)
    for c in range(65):
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        np.testing.assert_allclose(pe[c], pr, rtol=2e-5)
        np.testing.assert_allclose(g[c], gr, rtol=1e-4, atol=1e-3 * max(1.0, np.abs(gr).max() * 1e-2))


@pytest.mark.parametrize("dim", [10, 10000])
def test_funnel_noncentered_matches_oracle(device, dim):
    from numpyro_amd.potentials import FunnelNonCentered

    rs = np.random.RandomState(dim + 1)
    Z = rs.uniform(-2, 2, (65, dim)).astype(np.float32)
    pe, g = _eval(FunnelNonCentered(dim), Z, device)
    ref = OP.FunnelNonCentered(dim)
    for c in range(65):
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        np.testing.assert_allclose(pe[c], pr, rtol=2e-5)
        np.testing.assert_allclose(g[c], gr, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("N,H", [(100, 69), (50, 5), (37, 16)])
def test_bnn_matches_oracle(device, N, H):
    """examples/bnn.py model (D_X = 3, D_Y = 1) at the BASELINE width H = 69 (D = 5038) and
    small/ragged shapes.  fp32 vs float64: |dU| <= 1e-4 |U| + 1e-2; grad to 1e-3 of scale."""
    from numpyro_amd.potentials import BNN

    X, Y = datasets.bnn_data(N=N, D_X=3)
    ref = OP.BNN(X.astype(np.float64), Y.astype(np.float64), H)
    rs = np.random.RandomState(H)
    C = 130
    Z = (0.5 * rs.randn(C, ref.dim)).astype(np.float32)
    Z[:, 0] = rs.uniform(-1.0, 2.0, C)
    pe, g = _eval(BNN(X, Y, H), Z, device)
    for c in range(C):
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        np.testing.assert_allclose(pe[c], pr, rtol=1e-4, atol=1e-2)
        scale = np.abs(gr).max()
        np.testing.assert_allclose(g[c], gr, rtol=1e-3, atol=1e-3 * scale)


def test_bnn_skips_inactive_and_list(device):
    """Only listed/LEAF chains are evaluated (grad rows of other chains stay NaN)."""
    from numpyro_amd.potentials import BNN

    X, Y = datasets.bnn_data(N=30, D_X=3)
    pot = BNN(X, Y, 8)
    C = 70
    Z = np.random.RandomState(0).randn(C, pot.dim).astype(np.float32) * 0.3
    phase = np.zeros(C, np.int32)
    phase[::3] = 3
    pe, g = _eval(pot, Z, device, phase=phase)
    assert np.all(np.isnan(pe[phase == 0])) and np.all(np.isfinite(pe[phase == 3]))


def test_logreg_split_bf16_matches_f32_accuracy(device):
    """The split-bf16 kernel (every f32 operand as three bf16 terms, six bf16 MFMA products
    per k-step, f32 accumulation) carries f32-level error: against a float64 evaluation its U
    and gradient errors stay within 3x those of a plain float32 evaluation of the same
    formulas (NumPy, the oracle in float32) and below 3e-6 of max|grad| per chain."""
    from numpyro_amd.potentials import LogisticRegression

    X, y = datasets.covtype_synthetic(seed=0)
    X, y = X[:60000], y[:60000]
    rs = np.random.RandomState(5)
    C, D = 160, X.shape[1]
    Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.05 * rs.randn(C, D)).astype(np.float32)
    pe_r, g_r = OP.LogisticRegression(X.astype(np.float64), y.astype(np.float64)).pe_grad_batch(Z.astype(np.float64))
    f32 = OP.LogisticRegression(X, y, dtype=np.float32)
    o32 = [f32.pe_grad(z) for z in Z]
    pe32 = np.array([o[0] for o in o32], np.float64)
    g32 = np.stack([o[1] for o in o32]).astype(np.float64)
    pe, g = _eval(LogisticRegression(X, y), Z, device)
    gscale = np.abs(g_r).max(1)
    e_pe, e_g = np.abs(pe - pe_r) / np.abs(pe_r), np.abs(g - g_r).max(1) / gscale
    r_pe, r_g = np.abs(pe32 - pe_r) / np.abs(pe_r), np.abs(g32 - g_r).max(1) / gscale
    print(f"split-bf16 vs fp64: U {e_pe.max():.2e} grad {e_g.max():.2e} (median {np.median(e_g):.2e}); "
          f"NumPy float32: U {r_pe.max():.2e} grad {r_g.max():.2e} (median {np.median(r_g):.2e})")
    assert e_pe.max() <= max(3 * r_pe.max(), 2e-7)
    assert e_g.max() <= 3e-6
    assert np.median(e_g) <= 3 * max(np.median(r_g), 1e-7)


def _bf16_rne(v):
    """float32 -> its round-to-nearest-even bf16 value as float32 (finite inputs)."""
    u = np.ascontiguousarray(v, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def test_logreg_packed_split_is_bitwise_the_numpy_split(device):
    """nmx_logreg_pack's tiles hold each X value as three bf16 terms v1 = bf16(v),
    v2 = bf16(v - v1), v3 = bf16(v - v1 - v2), round to nearest even (potential_logreg.hip
    split3, converted in value pairs): bit-exact against a NumPy restatement of that split,
    in both operand layouts (GEMM1 A pieces: X[32 t + r][16 kb + 8 h + j]; GEMM2 B pieces:
    X[16 s + 8 (j >> 2) + 4 h + (j & 3)][32 dt + r]) and in the combined last-k-block pieces
    of D % 16 <= 8 (every lane X[32 t + r][48 + j], terms (1 | 2) and (3 | 1) by lane half),
    padded rows and columns zero."""
    import torch

    from numpyro_amd.potentials import LogisticRegression

    rs = np.random.RandomState(11)
    N, D = 77, 55
    X = (rs.randn(N, D) * np.exp(rs.randn(N, D) * 3)).astype(np.float32)  # wide exponent range
    X[3, :7] = [0.0, -0.0, 1e-30, -3e-30, 65504.0, 1.0 + 2 ** -23, -(1.0 + 2 ** -9)]
    y = (rs.rand(N) < 0.5).astype(np.float32)
    pot = LogisticRegression(X, y)
    pot.bind(64, 64, device)
    raw = pot.packed.view(torch.uint8).cpu().numpy()
    KB, DT = (D + 15) // 16, (D + 31) // 32
    H = 1  # D = 55: combined last k-block (potential_logreg.hip x3_h)
    NP = 3 * KB + 2 * H + 6 * DT + 1
    nt = (N + 31) // 32
    tiles = raw[512:512 + nt * NP * 1024].view(np.uint16).reshape(nt, NP, 64, 8)
    got = (tiles.astype(np.uint32) << 16).view(np.float32)  # bf16 bits -> float32 values

    Xp = np.zeros((nt * 32, 64), np.float32)
    Xp[:N, :D] = X
    t1 = _bf16_rne(Xp)
    e1 = Xp - t1
    t2 = _bf16_rne(e1)
    t3 = _bf16_rne(e1 - t2)
    planes = [t1, t2, t3]
    lane = np.arange(64)
    r, h = lane & 31, lane >> 5
    j = np.arange(8)
    for t in range(nt):
        for p in range(3):
            for kb in range(KB):
                rows = 32 * t + r[:, None]
                cols = 16 * kb + 8 * h[:, None] + j[None, :]
                want = planes[p][rows, cols]
                np.testing.assert_array_equal(got[t, p * KB + kb].view(np.uint32), want.view(np.uint32))
            for dt in range(DT):
                for s in range(2):
                    rows = 32 * t + 16 * s + 8 * (j[None, :] >> 2) + 4 * h[:, None] + (j[None, :] & 3)
                    cols = 32 * dt + r[:, None] + 0 * j[None, :]
                    want = planes[p][rows, cols]
                    piece = 3 * KB + 2 * H + p * 2 * DT + 2 * dt + s
                    np.testing.assert_array_equal(got[t, piece].view(np.uint32), want.view(np.uint32))
    rows = 32 * np.arange(nt)[:, None, None] + r[None, :, None]
    cols = 16 * (KB - 1) + j[None, None, :] + 0 * rows
    for cp, (ph0, ph1) in enumerate([(0, 1), (2, 0)]):
        want = np.where((h == 0)[None, :, None], planes[ph0][rows, cols], planes[ph1][rows, cols])
        np.testing.assert_array_equal(got[:, 3 * KB + cp].view(np.uint32), want.view(np.uint32))
    # the three terms represent every value to within 2^-24 relative (f32 rounding unit)
    assert np.all(np.abs((t1.astype(np.float64) + t2 + t3) - Xp) <= 2.0 ** -24 * np.abs(Xp) + 1e-45)
