"""Dense mass matrix (whitening around the potential, numpyro_amd/dense.py) on the GPU.

* `nmx_gemm_chains` (f32 MFMA) vs a float64 product; inactive chain tiles untouched.
  Tolerance |out - ref| <= 2e-6 * (|A| |In|) + 1e-6 (k-ordered f32 fma chain).
* MVN and whitened potentials vs the float64 oracle.
* Fixed dense mass, fixed step: device paths vs the oracle's dense-mass sample kernel
  (oracle/hmc_ref.py, which follows hmc.py:92-110 / hmc_util.py:1183-1220 directly, i.e.
  without whitening): >= 90% of chains take the identical discrete path, draws to 1e-3.
* Pooled adaptation: ports of test/infer/test_mcmc.py:75-100 (test_correlated_mvn) and
  :313-343 (test_dense_mass) with the reference's tolerances, at fewer iterations (the
  pooled estimate uses every chain's window samples).
"""
import numpy as np
import pytest
import torch

from numpyro_amd import native
from numpyro_amd import potentials as P
from numpyro_amd.dense import Whitening, WhitenedPotential
from numpyro_amd.infer import HMC, MCMC, NUTS
import parity_cases as PC
from oracle import hmc_ref as H
from oracle import parity as PR
from oracle import philox
from oracle import potentials as OP

pytestmark = pytest.mark.gpu


def _eval(pot, Z, device, phase=None, bind=True):
    C, D = Z.shape
    ldc = (C + 63) // 64 * 64
    if bind:
        pot.bind(C, ldc, device)
    z = torch.zeros(D, ldc, device=device)
    z[:, :C] = torch.from_numpy(Z.T.astype(np.float32)).to(device)
    g = torch.full((D, ldc), float("nan"), device=device)
    pe = torch.full((ldc,), float("nan"), device=device)
    ph = torch.zeros(ldc, dtype=torch.int32, device=device)
    ph[:C] = native.PH_LEAF if phase is None else torch.from_numpy(phase.astype(np.int32)).to(device)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), phase=native.ptr(ph),
                          num_chains=C, ldc=ldc)
    pot.evaluate(ev, native.stream_ptr())
    torch.cuda.synchronize()
    return pe[:C].cpu().numpy().astype(np.float64), g[:, :C].cpu().numpy().T.astype(np.float64)


@pytest.mark.parametrize("tri", [0, 1, 2])
@pytest.mark.parametrize("D,C,split", [(3, 64, False), (55, 200, False), (130, 130, False), (300, 256, False),
                                       (1000, 70, False), (3000, 130, True), (5038, 64, True)])
def test_gemm_chains_matches_fp64(device, D, C, tri, split):
    """Default (128 x 64) kernel; the opt-in wide kernel runs in a subprocess below."""
    rs = np.random.RandomState(D)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    ldc = (C + 63) // 64 * 64
    A = rs.randn(D, D)
    A = {0: A, 1: np.triu(A), 2: np.tril(A)}[tri]
    At = np.zeros((lda, lda), np.float32)
    At[:D, :D] = A.T
    In = rs.randn(D, ldc).astype(np.float32)
    bias = rs.randn(D).astype(np.float32)
    phase = np.full(ldc, native.PH_DONE, np.int32)
    act = rs.rand(C) < 0.5
    act[64:128] = False  # a fully idle tile (when present) must be left untouched
    phase[:C][act] = native.PH_LEAF
    dAt, dIn, db = (torch.from_numpy(x).to(device) for x in (At, In, bias))
    dph = torch.from_numpy(phase).to(device)
    out = torch.full((D, ldc), float("nan"), device=device)
    nws = lib.nmx_gemm_chains_workspace_bytes(D, ldc)
    ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=device) if split else None
    native.check(lib.nmx_gemm_chains(native.ptr(dAt), lda, D, native.ptr(dIn), native.ptr(out), native.ptr(db),
                                     tri, ldc, native.ptr(dph), None, C, native.ptr(ws) if nws else None,
                                     native.stream_ptr()))
    torch.cuda.synchronize()
    o = out.cpu().numpy().astype(np.float64)
    A32 = At[:D, :D].T.astype(np.float64)
    ref = A32 @ In.astype(np.float64) + bias[:, None]
    bound = 2e-6 * (np.abs(A32) @ np.abs(In.astype(np.float64)) + np.abs(bias)[:, None]) + 1e-6
    for t in range(ldc // 64):
        cols = slice(64 * t, 64 * t + 64)
        tile_active = bool((phase[cols] >= native.PH_LEAF).any())
        if tile_active:
            assert np.all(np.abs(o[:, cols] - ref[:, cols]) <= bound[:, cols])
        else:
            assert np.all(np.isnan(o[:, cols]))
    # error paths
    assert lib.nmx_gemm_chains(native.ptr(dAt), lda - 1, D, native.ptr(dIn), native.ptr(out), None, 0, ldc, None,
                               None, C, None, None) != 0
    assert lib.nmx_gemm_chains(native.ptr(dAt), lda, D, native.ptr(dIn), native.ptr(dIn), None, 0, ldc, None, None,
                               C, None, None) != 0
    assert lib.nmx_gemm_chains(native.ptr(dAt), lda, D, native.ptr(dIn), native.ptr(out), None, 3, ldc, None, None,
                               C, None, None) != 0


@pytest.mark.parametrize("tri", [0, 1, 2])
@pytest.mark.parametrize("D,C,split", [(3, 64, False), (55, 200, False), (300, 256, False), (1000, 70, False),
                                       (3000, 130, True), (5038, 64, True), (10000, 256, False),
                                       (10000, 2048, False)])
def test_gemm_chains_x3_matches_fp64(device, D, C, tri, split):
    """Split-bf16 products (nmx_gemm_chains_x3): f32-level error against float64 -- the same
    bound as the f32-MFMA kernel -- and inactive 64-chain tiles untouched.  D = 10000 is
    BASELINE config 2 (funnel-10k dense mass) on the default path: no split-K workspace (the
    x3 kernel splits K only above D = 16384), XCD-aware block order."""
    rs = np.random.RandomState(D + 7)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    ldc = (C + 63) // 64 * 64
    A = rs.randn(D, D)
    A = {0: A, 1: np.triu(A), 2: np.tril(A)}[tri]
    At = np.zeros((lda, lda), np.float32)
    At[:D, :D] = A.T
    In = rs.randn(D, ldc).astype(np.float32)
    bias = rs.randn(D).astype(np.float32)
    phase = np.full(ldc, native.PH_DONE, np.int32)
    act = rs.rand(C) < 0.5
    act[64:128] = False
    phase[:C][act] = native.PH_LEAF
    dAt, dIn, db = (torch.from_numpy(x).to(device) for x in (At, In, bias))
    dph = torch.from_numpy(phase).to(device)
    out = torch.full((D, ldc), float("nan"), device=device)
    nws = lib.nmx_gemm_chains_workspace_bytes(D, ldc)
    ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=device) if split else None
    Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=device)
    sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=device)
    s = native.stream_ptr()
    native.check(lib.nmx_gemm_x3_pack_a(native.ptr(dAt), lda, native.ptr(Ap), s))
    native.check(lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(dIn), native.ptr(out), native.ptr(db),
                                        tri, ldc, native.ptr(dph), None, C, native.ptr(sp),
                                        native.ptr(ws) if (split and nws) else None, s))
    torch.cuda.synchronize()
    o = out.cpu().numpy().astype(np.float64)
    # float64 reference (on the device for the large case: 2.6e10 multiply-adds)
    A64 = dAt[:D, :D].t().to(torch.float64)
    In64 = dIn.to(torch.float64)
    ref = (A64 @ In64 + db.to(torch.float64)[:, None]).cpu().numpy()
    bound = (2e-6 * (A64.abs() @ In64.abs() + db.to(torch.float64).abs()[:, None]) + 1e-6).cpu().numpy()
    for t in range(ldc // 64):
        cols = slice(64 * t, 64 * t + 64)
        if bool((phase[cols] >= native.PH_LEAF).any()):
            err = np.abs(o[:, cols] - ref[:, cols])
            assert np.all(err <= bound[:, cols]), (err / bound[:, cols]).max()
        else:
            assert np.all(np.isnan(o[:, cols]))
    assert lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(dIn), native.ptr(out), None, 0, ldc, None,
                                  None, C, None, None, None) != 0  # no split buffer


def test_gemm_chains_x3_error_is_a_float32_gemms(device):
    """The split-bf16 product's rounding is that of a float32 GEMM (BLAS sgemm in NumPy) on the
    same float32 operands, both against float64: at D = 5038 (BASELINE config 3's whitening) the
    median over chains of the largest relative error is within 1.25x sgemm's.  History: 4x when
    the five correction products shared the main accumulator (round 5's c3 draw drift), 1.7x
    with one main accumulator over all of K (the MFMA rounds its running sum every few products),
    ~0.4x modelled with the 256-deep block sums of round 6."""
    D, C, tri = 5038, 128, 1
    rs = np.random.RandomState(11)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    A32 = np.triu(rs.randn(D, D) / np.sqrt(D)).astype(np.float32)
    x32 = rs.randn(D, C).astype(np.float32)
    At = torch.zeros(lda, lda, device=device)
    At[:D, :D] = torch.from_numpy(A32.T.copy()).to(device)
    xd = torch.from_numpy(x32).to(device)
    out = torch.empty(D, C, device=device)
    Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=device)
    sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, C), dtype=torch.uint8, device=device)
    s = native.stream_ptr()
    native.check(lib.nmx_gemm_x3_pack_a(native.ptr(At), lda, native.ptr(Ap), s))
    native.check(lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(xd), native.ptr(out), None, tri, C, None,
                                        None, C, native.ptr(sp), None, s))
    torch.cuda.synchronize()
    y64 = A32.astype(np.float64) @ x32.astype(np.float64)
    sc = np.abs(y64).max(0)
    dev = np.median(np.abs(out.cpu().numpy().astype(np.float64) - y64).max(0) / sc)
    ref = np.median(np.abs((A32 @ x32).astype(np.float64) - y64).max(0) / sc)
    print(f"[x3 accuracy D={D}] device {dev:.3g} vs sgemm {ref:.3g} ({dev / ref:.2f}x)")
    assert dev <= 1.25 * ref, (dev, ref)


@pytest.mark.parametrize("tri", [0, 1, 2])
def test_gemm_chains_x3_tiles_agree(device, tri):
    """nmx_gemm_chains_x3 picks its workgroup tile from the grid size (256 x 128 when the launch
    still fills the chip twice over, else 128 x 64); the products must not depend on it: the
    same active columns computed under a chain bound that selects each tile are equal."""
    D, ldc = 10000, 2048
    rs = np.random.RandomState(tri)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    A = rs.randn(D, D)
    A = {0: A, 1: np.triu(A), 2: np.tril(A)}[tri]
    At = np.zeros((lda, lda), np.float32)
    At[:D, :D] = A.T
    In = rs.randn(D, ldc).astype(np.float32)
    bias = rs.randn(D).astype(np.float32)
    phase = np.full(ldc, native.PH_DONE, np.int32)
    phase[:1024][rs.rand(1024) < 0.7] = native.PH_LEAF
    dAt, dIn, db, dph = (torch.from_numpy(x).to(device) for x in (At, In, bias, phase))
    Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=device)
    sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=device)
    s = native.stream_ptr()
    native.check(lib.nmx_gemm_x3_pack_a(native.ptr(dAt), lda, native.ptr(Ap), s))
    outs = []
    for bound in (2048, 1024):  # 40 x 16 = 640 big-tile workgroups, then 40 x 8 = 320: small tiles
        out = torch.full((D, ldc), float("nan"), device=device)
        native.check(lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(dIn), native.ptr(out), native.ptr(db),
                                            tri, ldc, native.ptr(dph), None, bound, native.ptr(sp), None, s))
        outs.append(out[:, :1024].cpu().numpy())
    torch.cuda.synchronize()
    act = phase[:1024] >= native.PH_LEAF
    tiles = act.reshape(16, 64).any(axis=1).repeat(64)
    assert np.array_equal(outs[0][:, tiles], outs[1][:, tiles])
    assert np.all(np.isnan(outs[0][:, ~tiles])) and np.all(np.isnan(outs[1][:, ~tiles]))


@pytest.mark.parametrize("D,ldc,n", [(5, 64, 3), (150, 256, 77), (200, 128, 100), (1001, 512, 300), (10000, 4096, 4000)])
def test_gemm_chains_x3_rows_matches_pack_then_product(device, D, ldc, n):
    """nmx_gemm_chains_x3_rows (the listed chains' rows gathered inside the operand split) gives
    bitwise the product columns of nmx_pack_rows + nmx_gemm_chains_x3 for positions < count
    (D = 10000 x 4000 listed: config 2's shape, the 256 x 128 tile)."""
    rs = np.random.RandomState(D)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    At = np.zeros((lda, lda), np.float32)
    At[:D, :D] = np.triu(rs.randn(D, D)).T
    dAt = torch.from_numpy(At).to(device)
    rows = torch.from_numpy(rs.randn(ldc, D).astype(np.float32)).to(device)
    lst = torch.zeros(ldc, dtype=torch.int32, device=device)
    lst[:n] = torch.from_numpy(rs.permutation(ldc)[:n].astype(np.int32)).to(device)
    cnt = torch.tensor([n], dtype=torch.int32, device=device)
    db = torch.from_numpy(rs.randn(D).astype(np.float32)).to(device)
    Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=device)
    sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=device)
    s = native.stream_ptr()
    P_ = native.ptr
    native.check(lib.nmx_gemm_x3_pack_a(P_(dAt), lda, P_(Ap), s))
    packed = torch.full((D, ldc), 7.0, device=device)  # stale values past the count
    native.check(lib.nmx_pack_rows(P_(rows), ldc, D, P_(lst), P_(cnt), P_(packed), ldc, s))
    ref = torch.full((D, ldc), float("nan"), device=device)
    native.check(lib.nmx_gemm_chains_x3(P_(Ap), lda, D, P_(packed), P_(ref), P_(db), 1, ldc, None, P_(cnt), ldc,
                                        P_(sp), None, s))
    out = torch.full((D, ldc), float("nan"), device=device)
    native.check(lib.nmx_gemm_chains_x3_rows(P_(Ap), lda, D, P_(rows), P_(lst), P_(out), P_(db), 1, ldc, P_(cnt),
                                             ldc, P_(sp), None, s))
    torch.cuda.synchronize()
    assert torch.equal(out[:, :n], ref[:, :n])
    assert not torch.isnan(out[:, :n]).any()
    assert lib.nmx_gemm_chains_x3_rows(P_(Ap), lda, D, P_(rows), None, P_(out), None, 0, ldc, P_(cnt), ldc,
                                       P_(sp), None, s) != 0  # a list is required


@pytest.mark.parametrize("D,ldc,n", [(5, 64, 3), (150, 256, 77), (200, 128, 100), (1001, 512, 300),
                                     (10000, 4096, 4000)])
def test_gemm_chains_x3_to_rows_matches_product_then_unpack(device, D, ldc, n):
    """nmx_gemm_chains_x3_to_rows (the product stored to the listed chains' rows by its epilogue)
    gives bitwise the rows and pe of nmx_gemm_chains_x3 + nmx_unpack_rows, and leaves the rows of
    unlisted chains untouched."""
    rs = np.random.RandomState(D + 1)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    At = np.zeros((lda, lda), np.float32)
    At[:D, :D] = np.tril(rs.randn(D, D)).T
    dAt = torch.from_numpy(At).to(device)
    cols = torch.from_numpy(rs.randn(D, ldc).astype(np.float32)).to(device)
    lst = torch.zeros(ldc, dtype=torch.int32, device=device)
    chosen = rs.permutation(ldc)[:n].astype(np.int32)
    lst[:n] = torch.from_numpy(chosen).to(device)
    cnt = torch.tensor([n], dtype=torch.int32, device=device)
    pe_in = torch.from_numpy(rs.randn(ldc).astype(np.float32)).to(device)
    Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=device)
    sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=device)
    s = native.stream_ptr()
    P_ = native.ptr
    native.check(lib.nmx_gemm_x3_pack_a(P_(dAt), lda, P_(Ap), s))
    prod = torch.full((D, ldc), float("nan"), device=device)
    native.check(lib.nmx_gemm_chains_x3(P_(Ap), lda, D, P_(cols), P_(prod), None, 2, ldc, None, P_(cnt), ldc,
                                        P_(sp), None, s))
    ref = torch.full((ldc, D), float("nan"), device=device)
    pe_ref = torch.full((ldc,), float("nan"), device=device)
    native.check(lib.nmx_unpack_rows(P_(prod), ldc, D, P_(lst), P_(cnt), P_(ref), ldc, P_(pe_in), P_(pe_ref), s))
    out = torch.full((ldc, D), float("nan"), device=device)
    pe = torch.full((ldc,), float("nan"), device=device)
    native.check(lib.nmx_gemm_chains_x3_to_rows(P_(Ap), lda, D, P_(cols), P_(lst), P_(out), None, 2, ldc, P_(cnt),
                                                ldc, P_(sp), P_(pe_in), P_(pe), s))
    torch.cuda.synchronize()
    others = torch.from_numpy(np.setdiff1d(np.arange(ldc), chosen)).to(device)
    sel = torch.from_numpy(chosen.astype(np.int64)).to(device)
    assert torch.equal(out[sel], ref[sel]) and torch.equal(pe[sel], pe_ref[sel])
    assert not torch.isnan(out[sel]).any()
    assert torch.isnan(out[others]).all() and torch.isnan(pe[others]).all()


def _corr_cov(D, seed=0):
    rs = np.random.RandomState(seed)
    a = np.tril(0.5 * np.fliplr(np.eye(D)) + 0.1 * np.exp(rs.randn(D, D)))
    return a @ a.T


@pytest.mark.parametrize("D", [2, 5, 40, 200])
def test_mvn_potential_matches_oracle(device, D):
    cov = _corr_cov(D, D) + 0.1 * np.eye(D)
    mu = np.linspace(-1, 1, D)
    rs = np.random.RandomState(1)
    Z = rs.randn(100, D).astype(np.float32)
    pe, g = _eval(P.MultivariateNormal(mu, cov), Z, device)
    ref = OP.MVN(np.linalg.inv(cov), mu)
    prec = np.linalg.inv(cov)
    for c in range(Z.shape[0]):
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        scale = np.abs(prec) @ (np.abs(Z[c]) + np.abs(mu))
        assert np.all(np.abs(g[c] - gr) <= 1e-5 * scale + 1e-5)
        np.testing.assert_allclose(pe[c], pr, rtol=1e-4, atol=1e-4)


def test_mvn_potential_compacted_list_high_indices(device):
    """A compacted list whose count bound (num_chains = C - finished, as in a run's tail) is
    below the listed chains' indices: every listed chain is still evaluated."""
    D, C, ldc = 7, 200, 256
    cov = _corr_cov(D, 4) + 0.1 * np.eye(D)
    pot = P.MultivariateNormal(np.zeros(D), cov)
    pot.bind(C, ldc, device)
    rs = np.random.RandomState(2)
    Z = rs.randn(C, D).astype(np.float32)
    z = torch.zeros(D, ldc, device=device)
    z[:, :C] = torch.from_numpy(Z.T.copy()).to(device)
    g = torch.full((D, ldc), float("nan"), device=device)
    pe = torch.full((ldc,), float("nan"), device=device)
    chosen = np.array([199, 180, 150, 3], np.int32)
    ph = torch.zeros(ldc, dtype=torch.int32, device=device)
    ph[torch.from_numpy(chosen.astype(np.int64)).to(device)] = native.PH_LEAF
    idx = torch.zeros(ldc, dtype=torch.int32, device=device)
    idx[:4] = torch.from_numpy(chosen).to(device)
    cnt = torch.tensor([4], dtype=torch.int32, device=device)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), phase=native.ptr(ph),
                          active_idx=native.ptr(idx), active_count=native.ptr(cnt), num_chains=8, ldc=ldc)
    pot.evaluate(ev, native.stream_ptr())
    torch.cuda.synchronize()
    ref = OP.MVN(np.linalg.inv(cov))
    for c in chosen:
        pr, gr = ref.pe_grad(Z[c].astype(np.float64))
        np.testing.assert_allclose(pe[c].item(), pr, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(g[:, c].cpu().numpy(), gr, rtol=1e-4, atol=1e-4)


def test_whitened_potential_matches_oracle(device):
    D = 12
    cov = _corr_cov(D, 3) + 0.05 * np.eye(D)
    target = P.MultivariateNormal(np.ones(D), cov)
    wp = WhitenedPotential(target)
    C = 96
    wp.bind(C, 128, device)
    imm = _corr_cov(D, 4) + 0.2 * np.eye(D)
    mu = np.linspace(0, 2, D)
    wp.whitening.set(torch.from_numpy(imm), torch.from_numpy(mu))
    rs = np.random.RandomState(2)
    W = rs.randn(C, D).astype(np.float32)
    pe, gw = _eval(wp, W, device, bind=False)
    T = wp.whitening.T.cpu().numpy()
    np.testing.assert_allclose(T @ T.T, imm, rtol=1e-10, atol=1e-12)
    assert np.allclose(np.tril(T, -1), 0)  # T = tril_inv^T is upper triangular
    ref = OP.MVN(np.linalg.inv(cov), np.ones(D))
    for c in range(C):
        z = mu + T @ W[c].astype(np.float64)
        pr, gz = ref.pe_grad(z)
        np.testing.assert_allclose(pe[c], pr, rtol=2e-4, atol=2e-4)
        np.testing.assert_allclose(gw[c], T.T @ gz, rtol=1e-3, atol=1e-3)


def _oracle_chain(pe_grad, dim, seed, chain, num_iters, algo, **kw):
    o = H.NUTSOracle(lambda z: tuple(np.asarray(v, np.float32) if np.ndim(v) else np.float32(v)
                                     for v in pe_grad(z)), dim, 0, algo=algo, **kw)
    s = o.init(philox.init_uniform(seed, chain, 0, dim), seed, chain)
    out = []
    for _ in range(num_iters):
        s = o.sample(s)
        out.append(s)
    return out


@pytest.mark.parametrize("algo", ["NUTS", "HMC"])
@pytest.mark.parametrize("model", ["logreg", "mvn"])
def test_dense_fixed_mass_matches_oracle(device, algo, model):
    seed, C, T, D = 31, 64, 3, 6
    rs = np.random.RandomState(7)
    imm = _corr_cov(D, 11) * 0.05 + 0.01 * np.eye(D)
    if model == "logreg":
        X = rs.randn(400, D).astype(np.float32)
        beta = rs.randn(D) * 0.3
        y = (rs.rand(400) < 1 / (1 + np.exp(-X @ beta))).astype(np.float32)
        args, fm = (X, y), P.logistic_regression
        ref = OP.LogisticRegression(X, y, dtype=np.float32)
        site, step = "coefs", 0.1
    else:
        cov = _corr_cov(D, 12) + 0.1 * np.eye(D)
        args, fm = (None, cov), P.multivariate_normal
        ref = OP.MVN(np.linalg.inv(cov))
        site, step = "x", 0.2
    kw = dict(step_size=step, adapt_step_size=False, adapt_mass_matrix=False, dense_mass=True,
              inverse_mass_matrix=imm)
    if algo == "HMC":
        kw["trajectory_length"] = 10 * step
    kcls = NUTS if algo == "NUTS" else HMC
    mcmc = MCMC(kcls(fm, **kw), num_warmup=0, num_samples=T, num_chains=C, progress_bar=False)
    mcmc.run(seed, *args, extra_fields=("num_steps",))
    ns_dev = mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()
    zs = mcmc.get_samples(True)[site].cpu().numpy()
    okw = dict(step_size=step, adapt_step_size=False, adapt_mass_matrix=False, dense_mass=True,
               inverse_mass_matrix=imm.astype(np.float32))
    if algo == "HMC":
        okw["trajectory_length"] = 10 * step
    match = 0
    for c in range(C):
        states = _oracle_chain(ref.pe_grad, D, seed, c, T, algo, **okw)
        ns = np.array([s.num_steps for s in states])
        if np.array_equal(ns, ns_dev[c]):
            match += 1
            np.testing.assert_allclose(zs[c], np.stack([s.z for s in states]), rtol=1e-3, atol=1e-3)
    assert match >= int(0.9 * C), f"only {match}/{C} chains reproduced the oracle path"
    # HMCAdaptState carries the reference's matrices
    st = mcmc.last_state.adapt_state
    np.testing.assert_allclose(st.inverse_mass_matrix.cpu().numpy(), imm, rtol=1e-5, atol=1e-7)
    msq = st.mass_matrix_sqrt.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(msq @ msq.T, np.linalg.inv(imm), rtol=1e-3, atol=1e-3)


def _kernel(cls, *args, dense_mass, **kw):
    if dense_mass == "pooled":
        with pytest.warns(UserWarning, match="pooled"):
            return cls(*args, dense_mass=dense_mass, **kw)
    return cls(*args, dense_mass=dense_mass, **kw)


@pytest.mark.parametrize("mode", [True, "pooled"])
@pytest.mark.parametrize("kernel_cls", [NUTS, HMC])
@pytest.mark.parametrize("rho", [-0.7, 0.8])
def test_dense_mass_adaptation(device, kernel_cls, rho, mode):
    """test/infer/test_mcmc.py:313-343 (2-d MVN, trajectory_length=2): the adapted dense
    mass recovers the target covariance (rtol 0.10; per-chain matrices: their mean) and the
    sample moments match.  dense_mass=True adapts one matrix per chain (the reference's
    semantics), 'pooled' one matrix from every chain's draws."""
    true_cov = np.array([[10.0, rho], [rho, 0.1]])
    kernel = _kernel(kernel_cls, P.multivariate_normal, trajectory_length=2.0, dense_mass=mode)
    mcmc = MCMC(kernel, num_warmup=1000, num_samples=1000, num_chains=64, progress_bar=False)
    mcmc.run(0, None, true_cov)
    msq = mcmc.last_state.adapt_state.mass_matrix_sqrt.cpu().numpy().astype(np.float64)
    assert msq.shape == ((64, 2, 2) if mode is True else (2, 2))
    est_cov = np.linalg.inv(msq @ np.swapaxes(msq, -1, -2))
    if mode is True:
        est_cov = est_cov.mean(0)
    np.testing.assert_allclose(est_cov, true_cov, rtol=0.10)
    x = mcmc.get_samples()["x"].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(x[:, 0].mean(), 0.0, atol=0.50)
    np.testing.assert_allclose(x[:, 1].mean(), 0.0, atol=0.05)
    np.testing.assert_allclose((x[:, 0] * x[:, 1]).mean(), rho, atol=0.20)
    np.testing.assert_allclose(x.var(0), [10.0, 0.1], rtol=0.20)


@pytest.mark.parametrize("mode", [True, "pooled"])
@pytest.mark.parametrize("regularize", [True, False])
def test_correlated_mvn(device, regularize, mode):
    """test/infer/test_mcmc.py:75-100 (D = 5, dense NUTS from zeros)."""
    D = 5
    true_cov = _corr_cov(D, 0)
    kernel = _kernel(NUTS, P.multivariate_normal, dense_mass=mode, regularize_mass_matrix=regularize)
    C = 64
    mcmc = MCMC(kernel, num_warmup=1000, num_samples=1000, num_chains=C, progress_bar=False)
    mcmc.run(0, None, None, np.linalg.inv(true_cov), init_params=torch.zeros(C, D))
    x = mcmc.get_samples()["x"].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(x.mean(), 0.0, atol=0.02)
    assert np.sum(np.abs(np.cov(x.T) - true_cov)) / D ** 2 < 0.02


@pytest.mark.parametrize("mode", [True, "pooled"])
def test_dense_resume_from_post_warmup_state(device, mode):
    cov = _corr_cov(4, 5) + 0.1 * np.eye(4)
    mcmc = MCMC(_kernel(NUTS, P.multivariate_normal, dense_mass=mode), num_warmup=200, num_samples=50,
                num_chains=64)
    mcmc.warmup(1, None, cov)
    st = mcmc.post_warmup_state
    mcmc.run(2, None, cov)
    a = mcmc.get_samples()["x"].cpu().numpy()
    mcmc.post_warmup_state = st
    mcmc.run(2, None, cov)
    np.testing.assert_array_equal(a, mcmc.get_samples()["x"].cpu().numpy())
    assert st.adapt_state.inverse_mass_matrix.shape == ((64, 4, 4) if mode is True else (4, 4))


def test_whitening_roundtrip(device):
    D = 9
    wt = Whitening(D, device)
    imm = _corr_cov(D, 9) + 0.3 * np.eye(D)
    wt.set(torch.from_numpy(imm), torch.arange(D, dtype=torch.float32))
    z = torch.randn(D, 64, device=device)
    w = wt.to_whitened(z)
    wpad = torch.zeros(D, 64, device=device)
    wpad[:] = w
    zb = torch.empty(D, 64, device=device)
    wt.to_model(wpad, zb, stream=native.stream_ptr())
    torch.cuda.synchronize()
    np.testing.assert_allclose(zb.cpu().numpy(), z.cpu().numpy(), rtol=1e-4, atol=1e-4)


def test_whitened_packed_list_matches_dense_batch(device):
    """The compacted-list path (pack -> products on packed columns -> unpack) gives bitwise
    the dense-batch results for the listed chains and leaves the others untouched."""
    D, C = 150, 200
    ldc = 256
    cov = _corr_cov(D, 8) + 0.1 * np.eye(D)
    wp = WhitenedPotential(P.MultivariateNormal(np.zeros(D), cov))
    wp.bind(C, ldc, device)
    imm = _corr_cov(D, 9) + 0.3 * np.eye(D)
    wp.whitening.set(torch.from_numpy(imm), torch.from_numpy(np.linspace(-1, 1, D)))
    rs = np.random.RandomState(5)
    W = torch.zeros(D, ldc, device=device)
    W[:, :C] = torch.from_numpy(rs.randn(D, C).astype(np.float32)).to(device)
    s = native.stream_ptr()

    def run(active_idx=None, count=None):
        g = torch.full((D, ldc), float("nan"), device=device)
        pe = torch.full((ldc,), float("nan"), device=device)
        ph = torch.zeros(ldc, dtype=torch.int32, device=device)
        ph[:C] = native.PH_LEAF
        ev = native.EvalBatch(z=native.ptr(W), grad=native.ptr(g), pe=native.ptr(pe), phase=native.ptr(ph),
                              active_idx=native.ptr(active_idx), active_count=native.ptr(count), num_chains=C,
                              ldc=ldc)
        wp.evaluate(ev, s)
        torch.cuda.synchronize()
        return pe.cpu().numpy(), g.cpu().numpy()

    pe_d, g_d = run()
    chosen = rs.permutation(C)[:77].astype(np.int32)
    idx = torch.zeros(ldc, dtype=torch.int32, device=device)
    idx[:77] = torch.from_numpy(chosen).to(device)
    cnt = torch.tensor([77], dtype=torch.int32, device=device)
    pe_l, g_l = run(idx, cnt)
    np.testing.assert_array_equal(pe_l[chosen], pe_d[chosen])
    np.testing.assert_array_equal(g_l[:, chosen], g_d[:, chosen])
    others = np.setdiff1d(np.arange(ldc), chosen)
    assert np.all(np.isnan(pe_l[others])) and np.all(np.isnan(g_l[:, others]))


def test_whitened_bnn_rows_path_matches_packed_columns(device):
    """On a chain-row arena the whitened BNN runs its products from and to rows around
    nmx_pe_bnn_rows (no transposes); the packed-column path (NMX_DENSE_PACK_ROWS=1: pack, column
    products, transposes in nmx_pe_bnn, unpack) gives bitwise the same pe and gradient rows for
    the listed chains, and neither touches the others."""
    rs = np.random.RandomState(11)
    N, Dx, H = 40, 5, 7
    X = rs.randn(N, Dx).astype(np.float32)
    Y = rs.randn(N).astype(np.float32)
    base = P.BNN(X, Y, H)
    D = base.dim
    C, ldc, n = 150, 192, 61
    wp = WhitenedPotential(base)
    wp.bind(C, ldc, device)
    wp.rows = True
    a = rs.randn(D, D) * 0.05
    wp.whitening.set(torch.from_numpy(a @ a.T + np.eye(D)), torch.from_numpy(rs.randn(D) * 0.1))
    Z = torch.from_numpy(rs.randn(ldc, D).astype(np.float32)).to(device)
    chosen = rs.permutation(C)[:n].astype(np.int32)
    idx = torch.zeros(ldc, dtype=torch.int32, device=device)
    idx[:n] = torch.from_numpy(chosen).to(device)
    cnt = torch.tensor([n], dtype=torch.int32, device=device)
    s = native.stream_ptr()
    res = []
    for fused in (True, False):
        wp.fused_rows = fused
        g = torch.full((ldc, D), float("nan"), device=device)
        pe = torch.full((ldc,), float("nan"), device=device)
        ev = native.EvalBatch(z=native.ptr(Z), grad=native.ptr(g), pe=native.ptr(pe), phase=None,
                              active_idx=native.ptr(idx), active_count=native.ptr(cnt), num_chains=C, ldc=ldc)
        wp.evaluate(ev, s)
        torch.cuda.synchronize()
        res.append((pe.cpu().numpy(), g.cpu().numpy()))
    (pe_f, g_f), (pe_p, g_p) = res
    np.testing.assert_array_equal(pe_f[chosen], pe_p[chosen])
    np.testing.assert_array_equal(g_f[chosen], g_p[chosen])
    assert np.all(np.isfinite(pe_f[chosen])) and np.all(np.isfinite(g_f[chosen]))
    others = np.setdiff1d(np.arange(ldc), chosen)
    assert np.all(np.isnan(pe_f[others])) and np.all(np.isnan(g_f[others]))


def test_funnel_10k_dense_nuts_runs(device):
    """BASELINE config 2 shape (examples/funnel.py at dim 10000, dense mass) end to end at
    reduced chains and iterations: W = 20 (windows [0-2], [3-17], [18-19]: one pooled
    dense-mass update and re-expression at D = 10000), S = 2.  Every leaf consumes exactly
    one potential evaluation (the whitened potential's listed-chain count) and the draws are
    finite."""
    C = 256
    mcmc = MCMC(_kernel(NUTS, P.funnel, dense_mass="pooled", max_tree_depth=8), num_warmup=20, num_samples=2,
                num_chains=C)
    mcmc.warmup(0, 10000)
    eng = mcmc._engine
    assert eng.D == 10000 and eng.dense
    cnt = eng.view("counters")
    logged = torch.zeros(200000, dtype=torch.int32, device=eng.device)
    n = [0]
    orig = eng.potential.evaluate

    def counting(ev, s):
        p = 0 if ev is eng.eval_lists[0] else 1
        logged[n[0]] = cnt[2 + p]
        n[0] += 1
        orig(ev, s)

    eng.potential.evaluate = counting
    mcmc.run(1, 10000, extra_fields=("num_steps", "diverging"))
    eng.potential.evaluate = orig
    ef = mcmc.get_extra_fields()
    assert int(logged[:n[0]].sum().item()) == int(ef["num_steps"].sum().item())
    s = mcmc.get_samples()
    assert s["x"].shape == (C * 2, 9999) and s["y"].shape == (C * 2,)
    assert torch.isfinite(s["x"]).all() and torch.isfinite(s["y"]).all()
    imm = mcmc.post_warmup_state.adapt_state.inverse_mass_matrix
    assert imm.shape == (10000, 10000) and torch.isfinite(imm).all()
    assert not torch.equal(imm.cpu(), torch.eye(10000, dtype=imm.dtype))  # the window update happened


def test_per_chain_dense_needs_pooled_when_too_large(device):
    """Per-chain dense matrices at D = 10000 (C2) do not fit: the error names dense_mass='pooled'."""
    mcmc = MCMC(NUTS(P.funnel, dense_mass=True), num_warmup=10, num_samples=1, num_chains=64)
    with pytest.raises(ValueError, match="pooled"):
        mcmc.run(0, 10000)


@pytest.mark.parametrize("D,C", [(3, 64), (55, 130), (256, 70), (257, 40), (1100, 33)])
def test_chain_matvec_matches_fp64(device, D, C):
    """nmx_chain_matvec: out[a][c] = sum_b M[c][b][a] in[b][c] for listed chains (others
    untouched) and for the phase-selected dense batch; f32 fma-chain error bound."""
    lib = native.lib()
    rs = np.random.RandomState(D)
    ldc = (C + 63) // 64 * 64
    M = rs.randn(C, D, D).astype(np.float32)
    x = rs.randn(D, ldc).astype(np.float32)
    dM, dx = torch.from_numpy(M).to(device), torch.from_numpy(x).to(device)
    ref = np.einsum("cba,bc->ac", M.astype(np.float64), x[:, :C].astype(np.float64))
    bound = 1e-6 * np.einsum("cba,bc->ac", np.abs(M).astype(np.float64), np.abs(x[:, :C]).astype(np.float64)) + 1e-6
    chosen = np.sort(rs.choice(C, C // 3, replace=False)).astype(np.int32)[::-1].copy()
    idx = torch.zeros(ldc, dtype=torch.int32, device=device)
    idx[:len(chosen)] = torch.from_numpy(chosen).to(device)
    cnt = torch.tensor([len(chosen)], dtype=torch.int32, device=device)
    out = torch.full((D, ldc), float("nan"), device=device)
    native.check(lib.nmx_chain_matvec(native.ptr(dM), D, native.ptr(dx), native.ptr(out), ldc, native.ptr(idx),
                                      native.ptr(cnt), None, C, native.stream_ptr()))
    o = out.cpu().numpy().astype(np.float64)
    assert np.all(np.abs(o[:, chosen] - ref[:, chosen]) <= bound[:, chosen])
    others = np.setdiff1d(np.arange(ldc), chosen)
    assert np.all(np.isnan(o[:, others]))
    phase = torch.full((ldc,), native.PH_DONE, dtype=torch.int32, device=device)
    phase[:C:2] = native.PH_LEAF
    out.fill_(float("nan"))
    native.check(lib.nmx_chain_matvec(native.ptr(dM), D, native.ptr(dx), native.ptr(out), ldc, None, None,
                                      native.ptr(phase), C, native.stream_ptr()))
    o = out.cpu().numpy().astype(np.float64)
    assert np.all(np.abs(o[:, :C:2] - ref[:, ::2]) <= bound[:, ::2]) and np.all(np.isnan(o[:, 1:C:2]))


@pytest.mark.parametrize("D,C", [(300, 37), (1030, 20)])
def test_chain_matvec_triangular_skips_zero_rows(device, D, C):
    """nmx_chain_matvec_tri (dim > 256: one workgroup per chain and 256 outputs): with T_c upper
    triangular the forward product (M = T_c^T) skips rows b < a and the backward (M = T_c) rows
    b > a -- bitwise the full products (the skipped terms are exact zeros), and within the f32
    fma-chain bound of float64."""
    lib = native.lib()
    rs = np.random.RandomState(D)
    ldc = (C + 63) // 64 * 64
    T = np.triu(rs.randn(C, D, D)).astype(np.float32)
    x = rs.randn(D, ldc).astype(np.float32)
    dx = torch.from_numpy(x).to(device)
    for tri, M in ((1, np.ascontiguousarray(T.transpose(0, 2, 1))), (2, T)):
        dM = torch.from_numpy(M).to(device)
        outs = []
        for t in (0, tri):
            out = torch.full((D, ldc), float("nan"), device=device)
            native.check(lib.nmx_chain_matvec_tri(native.ptr(dM), D, native.ptr(dx), native.ptr(out), ldc, None, None,
                                                  None, C, t, native.stream_ptr()))
            outs.append(out.cpu().numpy())
        assert np.array_equal(outs[0][:, :C], outs[1][:, :C]), tri
        ref = np.einsum("cba,bc->ac", M.astype(np.float64), x[:, :C].astype(np.float64))
        bound = 1e-6 * np.einsum("cba,bc->ac", np.abs(M).astype(np.float64), np.abs(x[:, :C]).astype(np.float64))
        assert np.all(np.abs(outs[1][:, :C] - ref) <= bound + 1e-6), tri


@pytest.mark.parametrize("D,C", [(300, 9), (700, 5)])
def test_chain_welford_large_dim_matches_oracle(device, D, C):
    """nmx_chain_welford_ws above dim 256 (the two-launch form): every chain's mean and m2 after
    a few draws equal the oracle's f32 welford_covariance(diagonal=False) update_fn
    (hmc_util.py:172-196) to f32 rounding."""
    rs = np.random.RandomState(D)
    ldc = 64
    W = native.lib().nmx_chain_welford_work_bytes(D, C)
    assert W == C * 2 * D * 4
    from numpyro_amd.dense import ChainWelford
    cw = ChainWelford(D, C, device)
    _, upd, _ = H.welford_covariance(diagonal=False)
    st = [(np.zeros(D, np.float32), np.zeros((D, D), np.float32), 0) for _ in range(C)]
    for _ in range(4):
        z = rs.randn(D, ldc).astype(np.float32)
        cw.add(torch.from_numpy(z).to(device), stream=native.stream_ptr())
        st = [upd(z[:, c], st[c]) for c in range(C)]
    mean, m2 = cw.mean.cpu().numpy(), cw.m2.cpu().numpy()
    for c in range(C):
        np.testing.assert_allclose(mean[c], st[c][0], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(m2[c], st[c][1], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("D,C,K", [(512, 256, 24), (1024, 256, 12)])
def test_per_chain_dense_large_dim_matches_oracle(device, D, C, K):
    """Per-chain dense mass above dim 256 (the reference's vmapped init_kernel, hmc.py:790-798:
    every chain adapts its own matrix; no pooled deviation): MVN targets of dim 512 and 1024 with
    256 chains, W = 150 (one middle window), max_tree_depth 6.  (1) teacher-forced: the oracle's
    dense Welford + final_fn over each checked chain's device draws of the window reproduces its
    adapted inverse mass matrix; (2) from the post-warmup state the oracle's dense-mass NUTS takes
    the device's next three trees, every parting located at a rounding-level decision (the first
    K chains are traced and checked)."""
    seed, W = 23, 150
    cov = _corr_cov(D, 5) / D * 8 + 0.1 * np.eye(D)
    ref = OP.MVN(np.linalg.inv(cov))
    mcmc = MCMC(NUTS(P.multivariate_normal, dense_mass=True, max_tree_depth=6), num_warmup=W, num_samples=3,
                num_chains=C, progress_bar=False)
    mcmc.warmup(seed, None, cov, collect_warmup=True)
    eng = mcmc._engine
    assert eng.chain_dense and not eng.crow and eng.D == D
    draws = mcmc.get_samples(group_by_chain=True)["x"][:K].cpu().numpy().reshape(K, W, D)
    st = mcmc.post_warmup_state
    imm = st.adapt_state.inverse_mass_matrix[:K].cpu().numpy().astype(np.float64)
    _, upd, fin = H.welford_covariance(diagonal=False)
    for c in range(K):
        wst = (np.zeros(D, np.float32), np.zeros((D, D), np.float32), 0)
        for t in range(75, 100):
            wst = upd(draws[c, t], wst)
        np.testing.assert_allclose(imm[c], fin(wst, regularize=True)[0], rtol=1e-4, atol=1e-7, err_msg=f"chain {c}")
    eng.set_trace(K, W, 3)
    mcmc.run(seed, None, cov, extra_fields=("num_steps",))
    tr = eng.trace_records()
    ns_dev = mcmc.get_extra_fields(True)["num_steps"][:K].cpu().numpy()
    zs = mcmc.get_samples(True)["x"][:K].cpu().numpy()
    z0, g0 = st.z["x"][:K].cpu().numpy(), st.z_grad[:K].cpu().numpy()
    pe0, ss = st.potential_energy[:K].cpu().numpy(), st.adapt_state.step_size[:K].cpu().numpy()
    hist = []
    for c in range(K):
        o = H.NUTSOracle(PC.f32(ref.pe_grad), D, W, step_size=float(ss[c]), adapt_step_size=False,
                         adapt_mass_matrix=False, dense_mass=True, inverse_mass_matrix=imm[c].astype(np.float32),
                         max_tree_depth=6)
        wa = o.wa_init((z0[c],), None, np.float32(ss[c]), inverse_mass_matrix=imm[c].astype(np.float32),
                       mass_matrix_size=D)
        s0 = H.HMCState(W, z0[c].astype(np.float32), g0[c].astype(np.float32), np.float32(pe0[c]), None, None, None,
                        0, np.float32(0), np.float32(0), False, wa, (seed, c))
        hist.append(PC.traced(o, s0, 3))
    par = PR.compare_traced(hist, tr, ns_dev, zs, atol=1e-3, rtol=1e-3)
    print(f"[per-chain dense D={D}] device trees {ns_dev.tolist()}")
    PC.report(par, f"per-chain dense mvn D={D}", frac=0.9)


@pytest.mark.parametrize("model", ["mvn", "logreg"])
def test_per_chain_dense_adaptation_matches_oracle(device, model):
    """Per-chain dense adaptation (hmc.py:790-798: each chain its own welford_covariance
    (diagonal=False), hmc_util.py:133-239) over W = 150 (one middle window, [75-99]):
    (1) teacher-forced -- the oracle's dense Welford + final_fn fed each chain's device draws of
    the window reproduces the chain's adapted inverse mass matrix (rtol 1e-4: the same f32
    updates; the device's Cholesky is float64); (2) from each chain's post-warmup state the
    oracle's dense-mass NUTS (mass_matrix_sqrt @ eps momentum, M^-1 r in the leapfrog and the
    U-turn dots, hmc_util.py:1183-1220) takes the device's next three trees and draws (>= 95%
    of chains, every mismatch at a rounding-level decision tie)."""

    seed, C, W, D = 17, 64, 150, 6
    rs = np.random.RandomState(3)
    if model == "mvn":
        cov = _corr_cov(D, 21) + 0.1 * np.eye(D)
        args, fm, site = (None, cov), P.multivariate_normal, "x"
        ref = OP.MVN(np.linalg.inv(cov))
    else:
        X = rs.randn(500, D).astype(np.float32)
        X[:, 1] = X[:, 0] + 0.3 * X[:, 1]  # correlated posterior
        beta = rs.randn(D) * 0.3
        y = (rs.rand(500) < 1 / (1 + np.exp(-X @ beta))).astype(np.float32)
        args, fm, site = (X, y), P.logistic_regression, "coefs"
        ref = OP.LogisticRegression(X, y, dtype=np.float32)
    mcmc = MCMC(NUTS(fm, dense_mass=True), num_warmup=W, num_samples=3, num_chains=C)
    mcmc.warmup(seed, *args, collect_warmup=True)
    draws = mcmc.get_samples(group_by_chain=True)[site].cpu().numpy().reshape(C, W, D)
    st = mcmc.post_warmup_state
    imm = st.adapt_state.inverse_mass_matrix.cpu().numpy().astype(np.float64)
    assert imm.shape == (C, D, D)
    _, upd, fin = H.welford_covariance(diagonal=False)
    for c in range(C):
        wst = (np.zeros(D, np.float32), np.zeros((D, D), np.float32), 0)
        for t in range(75, 100):
            wst = upd(draws[c, t], wst)
        cov_o = fin(wst, regularize=True)[0]
        np.testing.assert_allclose(imm[c], cov_o, rtol=1e-4, atol=1e-7, err_msg=f"chain {c}")
    # (2) sampling transitions from the post-warmup state (decision trace on)
    mcmc._engine.set_trace(C, W, 3)
    mcmc.run(seed, *args, extra_fields=("num_steps",))
    tr = mcmc._engine.trace_records()
    ns_dev = mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()
    zs = mcmc.get_samples(True)[site].cpu().numpy()
    z0 = st.z[site].cpu().numpy()
    g0 = st.z_grad.cpu().numpy()
    pe0 = st.potential_energy.cpu().numpy()
    ss = st.adapt_state.step_size.cpu().numpy()
    hist = []
    for c in range(C):
        o = H.NUTSOracle(PC.f32(ref.pe_grad), D, W, step_size=float(ss[c]), adapt_step_size=False,
                         adapt_mass_matrix=False, dense_mass=True, inverse_mass_matrix=imm[c].astype(np.float32))
        wa = o.wa_init((z0[c],), None, np.float32(ss[c]), inverse_mass_matrix=imm[c].astype(np.float32),
                       mass_matrix_size=D)
        s = H.HMCState(W, z0[c].astype(np.float32), g0[c].astype(np.float32), np.float32(pe0[c]), None, None, None,
                       0, np.float32(0), np.float32(0), False, wa, (seed, c))
        hist.append(PC.traced(o, s, 3))
    par = PR.compare_traced(hist, tr, ns_dev, zs, atol=1e-3, rtol=1e-3)
    PC.report(par, f"per-chain dense {model}", frac=0.95)


def test_structured_dense_mass_matches_oracle(device):
    """Structured mass (dense_mass=[("theta", "mu")], hmc.py:239-252) on eight schools: a dense
    block over (theta, mu) in that order and a diagonal block over tau, adapted per chain over
    W = 150 (middle window [75-99]).  (1) teacher-forced: the oracle's Welford + final_fn of
    each block (hmc_util.py:439-515 builds the blocks, :133-239 adapts them) over the chain's
    device draws reproduces the chain's adapted blocks; the state holds them as a dict keyed by
    site group.  (2) from each chain's post-warmup state the oracle's dense-mass NUTS with the
    block matrices scattered into full ones (M^-1 and mass_matrix_sqrt block by block, so the
    momentum and kinetic energy are the reference's per-block ones) takes the device's next three
    trees and draws for >= 90% of chains, every mismatch at a rounding-level tie."""
    from numpyro_amd import datasets

    seed, C, W, D = 23, 64, 150, 10
    args = (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y)
    groups = [("theta", "mu")]
    # postprocess_fn = identity: the draws stay unconstrained (tau on the log scale)
    mcmc = MCMC(NUTS(P.eight_schools, dense_mass=groups), num_warmup=W, num_samples=3, num_chains=C,
                postprocess_fn=lambda z: z)
    mcmc.warmup(seed, *args, collect_warmup=True)
    eng = mcmc._engine
    assert eng.chain_dense and eng.blocks is not None
    ws = mcmc.get_samples(group_by_chain=True)
    flat = lambda d: np.concatenate([d["mu"].cpu().numpy()[..., None], d["tau"].cpu().numpy()[..., None],  # noqa
                                     d["theta"].cpu().numpy()], axis=-1)
    draws = flat(ws).astype(np.float32)  # ravel order (mu, log tau, theta)
    st = mcmc.post_warmup_state
    imm = st.adapt_state.inverse_mass_matrix
    assert set(imm) == {("theta", "mu"), ("tau",)}
    dense_b = imm[("theta", "mu")].cpu().numpy().astype(np.float64)
    diag_b = imm[("tau",)].cpu().numpy().astype(np.float64)
    assert dense_b.shape == (C, 9, 9) and diag_b.shape == (C, 1)
    order = list(range(2, 10)) + [0]  # (theta, mu) in ravel coordinates
    _, upd_d, fin_d = H.welford_covariance(diagonal=False)
    _, upd_g, fin_g = H.welford_covariance(diagonal=True)
    for c in range(C):
        sd = (np.zeros(9, np.float32), np.zeros((9, 9), np.float32), 0)
        sg = (np.zeros(1, np.float32), np.zeros(1, np.float32), 0)
        for t in range(75, 100):
            sd = upd_d(draws[c, t, order], sd)
            sg = upd_g(draws[c, t, [1]], sg)
        np.testing.assert_allclose(dense_b[c], fin_d(sd, regularize=True)[0], rtol=1e-4, atol=1e-7,
                                   err_msg=f"chain {c} dense block")
        np.testing.assert_allclose(diag_b[c], fin_g(sg, regularize=True)[0], rtol=1e-5, err_msg=f"chain {c} tau")
    # (2) sampling transitions from the post-warmup state (decision trace on)
    eng.set_trace(C, W, 3)
    mcmc.run(seed, *args, extra_fields=("num_steps",))
    tr = eng.trace_records()
    ns_dev = mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()
    zs = flat(mcmc.get_samples(True))
    z0 = torch.cat([st.z["mu"][:, None], st.z["tau"][:, None], st.z["theta"]], 1).cpu().numpy()
    g0, pe0 = st.z_grad.cpu().numpy(), st.potential_energy.cpu().numpy()
    ss = st.adapt_state.step_size.cpu().numpy()
    ref = OP.EightSchools(datasets.EIGHT_SCHOOLS_Y, datasets.EIGHT_SCHOOLS_SIGMA)
    hist = []
    for c in range(C):
        imm_f = np.zeros((D, D), np.float32)
        msq_f = np.zeros((D, D), np.float32)
        i_b, sq_b, _ = H._initialize_mass_matrix(9, dense_b[c].astype(np.float32), True)
        imm_f[np.ix_(order, order)] = i_b
        msq_f[np.ix_(order, order)] = sq_b
        i_t, sq_t, _ = H._initialize_mass_matrix(1, diag_b[c].astype(np.float32), False)
        imm_f[1, 1], msq_f[1, 1] = i_t[0], sq_t[0]
        o = H.NUTSOracle(PC.f32(ref.pe_grad), D, W, step_size=float(ss[c]), adapt_step_size=False,
                         adapt_mass_matrix=False, dense_mass=True, inverse_mass_matrix=np.eye(D, dtype=np.float32))
        wa = o.wa_init((z0[c],), None, np.float32(ss[c]), inverse_mass_matrix=np.eye(D, dtype=np.float32),
                       mass_matrix_size=D)._replace(inverse_mass_matrix=imm_f, mass_matrix_sqrt=msq_f)
        s = H.HMCState(W, z0[c].astype(np.float32), g0[c].astype(np.float32), np.float32(pe0[c]), None, None, None,
                       0, np.float32(0), np.float32(0), False, wa, (seed, c))
        hist.append(PC.traced(o, s, 3))
    par = PR.compare_traced(hist, tr, ns_dev, zs, atol=1e-3, rtol=1e-3)
    PC.report(par, "structured dense eight schools", frac=0.9)


def _dense_wide_run(monkeypatch, rows_step, C=96, sync=False, chain_offset=None, W=20, S=4, seed=5, fixed=False):
    from numpyro_amd.engine import Engine

    monkeypatch.setattr(Engine, "chain_rows_step", rows_step)
    if fixed:  # one given dense matrix for every chain (no pooled adaptation: shards independent)
        rs = np.random.RandomState(1)
        a = rs.randn(600, 600) / 60.0
        kern = NUTS(P.funnel, dense_mass=True, adapt_mass_matrix=False, inverse_mass_matrix=a @ a.T + np.eye(600),
                    max_tree_depth=7, **({"step_size": 0.02, "adapt_step_size": False} if W == 0 else {}))
    else:
        kern = _kernel(NUTS, P.funnel, dense_mass="pooled", max_tree_depth=7)
    mcmc = MCMC(kern, num_warmup=W, num_samples=S, num_chains=C, sync_chains=sync, chain_offset=chain_offset)
    mcmc.run(seed, 600, extra_fields=("num_steps",))
    assert mcmc._engine.crow == rows_step
    return (mcmc.get_samples(True)["x"].cpu().numpy(), mcmc.get_extra_fields(True)["num_steps"].cpu().numpy())


def test_dense_wide_chain_row_step_matches_slices(device, monkeypatch):
    """Dense mass at D >= 257: the launched loop with the per-chain step on a chain-row arena
    (k_chain_step; the whitening packs the listed chains' rows) against the D-slice kernels
    (V1 / R / S / V2) on the chain-minor arena.  Same per-coordinate arithmetic, dot products
    summed in another fixed order: tree sizes and draws agree to rounding for >= 90% of chains
    (funnel D = 600, a given dense matrix and a fixed step size: with pooled adaptation one
    chain's rounding moves every chain's matrix, and dual averaging amplifies rounding)."""
    x0, n0 = _dense_wide_run(monkeypatch, False, fixed=True, W=0)
    x1, n1 = _dense_wide_run(monkeypatch, True, fixed=True, W=0)
    same = np.all(n0 == n1, axis=1) & np.all(np.isclose(x0, x1, rtol=1e-3, atol=1e-3).reshape(96, -1), axis=1)
    print(f"[dense wide chain rows] {int(same.sum())}/96 chains: same tree sizes and draws as the D-slice step")
    assert same.sum() >= 86


def test_dense_wide_chain_row_step_invariances(device, monkeypatch):
    """The chain-row step keeps the engine's invariances bitwise: lockstep == async (pooled
    adaptation), and two chain shards reproduce the unsharded run (a given dense matrix: the
    pooled one would be adapted per shard here, all_reduced across ranks in a real run)."""
    a = _dense_wide_run(monkeypatch, True)
    b = _dense_wide_run(monkeypatch, True, sync=True)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)
    f = _dense_wide_run(monkeypatch, True, fixed=True)
    lo = _dense_wide_run(monkeypatch, True, C=40, chain_offset=0, fixed=True)
    hi = _dense_wide_run(monkeypatch, True, C=56, chain_offset=40, fixed=True)
    np.testing.assert_array_equal(f[0][:40], lo[0])
    np.testing.assert_array_equal(f[0][40:], hi[0])


def test_inverse_mass_matrix_dict_of_blocks_matches_oracle(device):
    """inverse_mass_matrix as a dict {site group: block} (hmc_util.py:439-487, hmc.py:223-234)
    with a structured dense_mass and no adaptation: the dense block over (theta, mu) in the group's
    order and the diagonal block of tau come from the dict; the state holds them back keyed by
    group; the oracle's dense-mass NUTS with the blocks scattered into full matrices (momentum from
    each block's own factor) takes the device's trees and draws at a fixed step size."""
    from numpyro_amd import datasets

    seed, C, T, D = 29, 32, 3, 10
    args = (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y)
    rs = np.random.RandomState(3)
    a = rs.randn(9, 9) * 0.3
    blk = (a @ a.T + np.eye(9)).astype(np.float32)
    imm = {("theta", "mu"): blk, ("tau",): np.array([0.5], np.float32)}
    mcmc = MCMC(NUTS(P.eight_schools, dense_mass=[("theta", "mu")], inverse_mass_matrix=imm, adapt_mass_matrix=False,
                     step_size=0.1, adapt_step_size=False), num_warmup=0, num_samples=T, num_chains=C,
                postprocess_fn=lambda z: z)
    eng = mcmc._get_engine(args, {})
    eng.set_trace(C, 0, T)
    mcmc.run(seed, *args, extra_fields=("num_steps",))
    assert mcmc._engine is eng
    tr = eng.trace_records()
    st = mcmc.last_state.adapt_state.inverse_mass_matrix
    np.testing.assert_allclose(st[("theta", "mu")][0].cpu().numpy(), blk, rtol=1e-6)
    np.testing.assert_allclose(st[("tau",)][0].cpu().numpy(), [0.5], rtol=1e-6)
    ns_dev = mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()
    sm = mcmc.get_samples(True)
    zs = np.concatenate([sm["mu"].cpu().numpy()[..., None], sm["tau"].cpu().numpy()[..., None],
                         sm["theta"].cpu().numpy()], axis=-1)
    order = list(range(2, 10)) + [0]
    imm_f = np.zeros((D, D), np.float32)
    msq_f = np.zeros((D, D), np.float32)
    i_b, sq_b, _ = H._initialize_mass_matrix(9, blk, True)
    imm_f[np.ix_(order, order)], msq_f[np.ix_(order, order)] = i_b, sq_b
    i_t, sq_t, _ = H._initialize_mass_matrix(1, np.array([0.5], np.float32), False)
    imm_f[1, 1], msq_f[1, 1] = i_t[0], sq_t[0]
    ref = OP.EightSchools(datasets.EIGHT_SCHOOLS_Y, datasets.EIGHT_SCHOOLS_SIGMA)
    hist = []
    for c in range(C):
        o = H.NUTSOracle(PC.f32(ref.pe_grad), D, 0, step_size=0.1, adapt_step_size=False, adapt_mass_matrix=False,
                         dense_mass=True, inverse_mass_matrix=np.eye(D, dtype=np.float32))
        s = o.init(philox.init_uniform(seed, c, 0, D), seed, c)
        s = s._replace(adapt_state=s.adapt_state._replace(inverse_mass_matrix=imm_f, mass_matrix_sqrt=msq_f))
        hist.append(PC.traced(o, s, T))
    par = PR.compare_traced(hist, tr, ns_dev, zs, atol=1e-3, rtol=1e-3)
    PC.report(par, "inverse_mass_matrix dict", frac=0.9)


def test_pooled_structured_mass_matches_oracle(device):
    """dense_mass=pooled([("w3", "prec_obs")]) on the BNN at H = 16 (D = 321: the chain-row dense
    step): one structured mass for all chains -- a dense block over (w3, prec_obs) in that group's
    order, a diagonal block over w1 and w2 (hmc.py:239-252, hmc_util.py:439-515) -- adapted from the
    pooled draws of the middle window.  (1) teacher-forced: the window's draws of every chain, pooled
    (mean and covariance over chains and draws), regularized as welford_covariance's final_fn
    (hmc_util.py:212-226) and cut to the blocks, reproduce the state's {group: block} matrices; the
    group order makes T non-triangular in ravel order, so the whitening runs the full products.
    (2) from the post-warmup state the oracle's dense-mass NUTS with the block matrices scattered into
    full ones (each block's own flipped Cholesky: mass_matrix_sqrt block by block) takes the device's
    trees and draws, leaf-located against the device's decision trace."""
    import warnings

    from numpyro_amd import datasets
    from numpyro_amd.infer import pooled

    Hh, C, W, T, seed = 16, 64, 150, 3, 41
    X, Y = datasets.bnn_data(N=30, D_X=3)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        kern = NUTS(P.bnn, dense_mass=pooled([("w3", "prec_obs")]), max_tree_depth=6)
    mcmc = MCMC(kern, num_warmup=W, num_samples=T, num_chains=C, postprocess_fn=lambda z: z)
    mcmc.warmup(seed, X, Y, Hh, collect_warmup=True)
    eng = mcmc._engine
    assert eng.dense and not eng.chain_dense and eng.blocks is not None and eng.crow
    wt = eng.potential.whitening
    assert not wt.upper  # (w3, prec_obs) is not in ravel order
    ws = mcmc.get_samples(group_by_chain=True)
    D = eng.D
    flat = lambda d: np.concatenate([d["prec_obs"].cpu().numpy()[..., None],  # noqa: E731
                                     d["w1"].cpu().numpy().reshape(*d["w1"].shape[:2], -1),
                                     d["w2"].cpu().numpy().reshape(*d["w2"].shape[:2], -1),
                                     d["w3"].cpu().numpy().reshape(*d["w3"].shape[:2], -1)], axis=-1)
    draws = flat(ws).astype(np.float64)  # [C, W, D] ravel order
    assert draws.shape == (C, W, D)
    win = draws[:, 75:100].reshape(-1, D)  # the middle window [75, 99], all chains pooled
    n = win.shape[0]
    cov = np.cov(win.T) * n / (n + 5.0) + 1e-3 * 5.0 / (n + 5.0) * np.eye(D)
    o = 1 + 3 * Hh + Hh * Hh
    grp = list(range(o, o + Hh)) + [0]
    rest = list(range(1, o))
    st = mcmc.post_warmup_state
    imm = st.adapt_state.inverse_mass_matrix
    assert set(imm) == {("w3", "prec_obs"), ("w1", "w2")}
    np.testing.assert_allclose(imm[("w3", "prec_obs")].cpu().numpy(), cov[np.ix_(grp, grp)], rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(imm[("w1", "w2")].cpu().numpy(), cov[rest, rest], rtol=2e-4, atol=1e-6)
    # (2) sampling from the post-warmup state, traced
    eng.set_trace(C, W, T)
    mcmc.run(seed + 1, X, Y, Hh, extra_fields=("num_steps",))
    tr = eng.trace_records()
    ns_dev = mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()
    zs = flat(mcmc.get_samples(True))
    z0 = flat({k: v[:, None] for k, v in st.z.items()})[:, 0]
    g0, pe0 = st.z_grad.cpu().numpy(), st.potential_energy.cpu().numpy()
    ss = st.adapt_state.step_size.cpu().numpy()
    dense_b = imm[("w3", "prec_obs")].cpu().numpy().astype(np.float32)
    diag_b = imm[("w1", "w2")].cpu().numpy().astype(np.float32)
    imm_f = np.zeros((D, D), np.float32)
    msq_f = np.zeros((D, D), np.float32)
    i_b, sq_b, _ = H._initialize_mass_matrix(len(grp), dense_b, True)
    imm_f[np.ix_(grp, grp)], msq_f[np.ix_(grp, grp)] = i_b, sq_b
    i_d, sq_d, _ = H._initialize_mass_matrix(len(rest), diag_b, False)
    imm_f[rest, rest], msq_f[rest, rest] = i_d, sq_d
    ref = OP.BNN(X, Y, Hh, dtype=np.float32)
    hist = []
    for c in range(C):
        o_ = H.NUTSOracle(PC.f32(ref.pe_grad), D, W, step_size=float(ss[c]), adapt_step_size=False,
                          adapt_mass_matrix=False, dense_mass=True, inverse_mass_matrix=np.eye(D, dtype=np.float32),
                          max_tree_depth=6)
        wa = o_.wa_init((z0[c].astype(np.float32),), None, np.float32(ss[c]),
                        inverse_mass_matrix=np.eye(D, dtype=np.float32), mass_matrix_size=D)._replace(
            inverse_mass_matrix=imm_f, mass_matrix_sqrt=msq_f)
        s0 = H.HMCState(W, z0[c].astype(np.float32), g0[c].astype(np.float32), np.float32(pe0[c]), None, None, None,
                        0, np.float32(0), np.float32(0), False, wa, (seed + 1, c))
        hist.append(PC.traced(o_, s0, T))
    par = PR.compare_traced(hist, tr, ns_dev, zs, atol=1e-3, rtol=1e-3)
    PC.report(par, "pooled structured mass BNN D=321", frac=0.8)
