"""Dense mass matrix by whitening (hmc.py:92-110 momentum, hmc_util.py:1183-1220 kinetic
energy, hmc_util.py:198-237 dense Welford finalize, hmc_util.py:488-515 initialisation).

The reference's dense-mass NUTS draws r = mass_matrix_sqrt @ eps, moves z by
dt * M^-1 r and tests U-turns with (M^-1 r) . r_sum.  With T = tril_inv^T (upper
triangular, T T^T = M^-1 = cov) and the change of variables z = mu + T w, p_w = T^T r:

* p_w = tril_inv @ mass_matrix_sqrt @ eps = eps          (identity-mass momentum)
* 0.5 r^T M^-1 r = 0.5 |p_w|^2                           (kinetic energy)
* (M^-1 r_a) . r_b = p_w,a . p_w,b                        (U-turn criterion)
* the leapfrog on (z, r) with M^-1 is the leapfrog on (w, p_w) with identity mass
  and U_w(w) = U(mu + T w), grad_w = T^T grad_z.

So the device state machine runs unchanged with identity mass on w, and the model's
potential is wrapped by two chain-batched MFMA products per leapfrog (`nmx_gemm_chains`):
z = mu + T w before, g_w = T^T g_z after.  Results equal the reference's in exact
arithmetic; in f32 they differ by rounding (the parity test follows the oracle's dense
path at fixed step size).

Adaptation is per chain, as the reference's vmapped init_kernel does (hmc.py:790-798), when
the per-chain matrices fit (dim <= CHAIN_DENSE_MAX_D): ChainWhitenedPotential / ChainWelford.
Otherwise dense_mass="pooled" is the explicit, warned opt-in: at the end of
every middle adaptation window the covariance of every chain's samples in that window (all
ranks, reduced over RCCL) replaces M^-1 for every chain, regularised as in the reference with
n = the pooled sample count (PooledCovariance).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import native
from .native import EvalBatch, check, lib, ptr
from .potentials import REAL, Potential

DENSE, UPPER, LOWER = 0, 1, 2  # nmx_gemm_chains `triangle` (shape of A in Out = A In)


class Whitening:
    """z = mu + T w, T T^T = M^-1.  Holds the two padded At operands of nmx_gemm_chains."""

    def __init__(self, dim: int, device, x3: bool = True, blocks=None):
        """x3: split-bf16 products (nmx_gemm_chains_x3, the default) or the f32-MFMA kernel
        (nmx_gemm_chains, kept for comparison in tests).  blocks (MassBlocks): a structured mass
        (dense_mass=pooled([...])): M^-1 masked to the blocks, T factored block by block in each
        block's own coordinate order -- triangular only when every block's coordinates are
        contiguous and in ravel order, else the products run on the full matrix."""
        self.D = int(dim)
        self.blocks = blocks
        self.upper = True
        self.device = torch.device(device)
        self.lda = int(lib().nmx_dense_padded_dim(self.D))
        self.fwd_t = torch.zeros(self.lda, self.lda, dtype=torch.float32, device=self.device)  # T^T
        self.bwd_t = torch.zeros(self.lda, self.lda, dtype=torch.float32, device=self.device)  # T
        self.mu = torch.zeros(self.D, dtype=torch.float32, device=self.device)
        self._ws = {}
        self._split = {}
        self.version = 0  # bumped by set(): cached views of the matrices are keyed by it
        self.x3 = bool(x3)
        if self.x3:  # MFMA-fragment packs of T^T and T (nmx_gemm_x3_pack_a)
            nb = lib().nmx_gemm_x3_packed_a_bytes(self.lda)
            self.fwd_p = torch.empty(nb, dtype=torch.uint8, device=self.device)
            self.bwd_p = torch.empty(nb, dtype=torch.uint8, device=self.device)
        self.set(torch.eye(self.D, dtype=torch.float64, device=self.device), None)

    def workspace(self, ldc):
        """Split-K workspace of nmx_gemm_chains for [D][ldc] operands (None if no split)."""
        if ldc not in self._ws:
            nb = lib().nmx_gemm_chains_workspace_bytes(self.D, ldc)
            self._ws[ldc] = torch.empty(nb, dtype=torch.uint8, device=self.device) if nb else None
        return self._ws[ldc]

    def split_buffer(self, ldc):
        """Per-call split of the chain operand (nmx_gemm_x3_split_bytes)."""
        if ldc not in self._split:
            self._split[ldc] = torch.empty(lib().nmx_gemm_x3_split_bytes(self.lda, ldc), dtype=torch.uint8,
                                           device=self.device)
        return self._split[ldc]

    def product(self, forward, x, out, bias, phase, count, num_chains, ldc, stream):
        """Out = T In (+ bias) if forward else T^T In, on raw device pointers (x, out, bias,
        phase, count: ints or None): the nmx_gemm_chains(_x3) call of every dense product."""
        at, ap, tri = (self.fwd_t, getattr(self, "fwd_p", None), self._tri(True)) if forward else \
            (self.bwd_t, getattr(self, "bwd_p", None), self._tri(False))
        ws = ptr(self.workspace(ldc))
        if self.x3:
            check(lib().nmx_gemm_chains_x3(ptr(ap), self.lda, self.D, x, out, bias, tri, ldc, phase, count,
                                           int(num_chains), ptr(self.split_buffer(ldc)), ws, stream),
                  "nmx_gemm_chains_x3")
        else:
            check(lib().nmx_gemm_chains(ptr(at), self.lda, self.D, x, out, bias, tri, ldc, phase, count,
                                        int(num_chains), ws, stream), "nmx_gemm_chains")

    def product_rows(self, rows, list_, count, out, num_chains, ldc, stream):
        """Out = T In + mu on the listed chains' rows gathered in place (In column p = rows[list[p]]):
        nmx_gemm_chains_x3_rows, the pack + forward product in one call (x3 only)."""
        check(lib().nmx_gemm_chains_x3_rows(ptr(self.fwd_p), self.lda, self.D, rows, list_, out, ptr(self.mu),
                                            self._tri(True),
                                            ldc, count, int(num_chains), ptr(self.split_buffer(ldc)),
                                            ptr(self.workspace(ldc)), stream), "nmx_gemm_chains_x3_rows")

    def product_to_rows(self, x, list_, count, rows, pe_in, pe_out, num_chains, ldc, stream):
        """rows[list[p]] = (T^T In)[:, p] for p < count, pe_out[list[p]] = pe_in[p]:
        nmx_gemm_chains_x3_to_rows, the backward product + unpack in one call (x3 only)."""
        check(lib().nmx_gemm_chains_x3_to_rows(ptr(self.bwd_p), self.lda, self.D, x, list_, rows, None,
                                               self._tri(False), ldc,
                                               count, int(num_chains), ptr(self.split_buffer(ldc)), pe_in, pe_out,
                                               stream), "nmx_gemm_chains_x3_to_rows")

    def product_lists(self, forward, x, in_list, out, out_list, bias, count, num_chains, ldc, stream, pe_in=None,
                      pe_out=None):
        """nmx_gemm_chains_x3_lists: In gathered from rows through in_list (or columns), Out stored to
        rows through out_list (or columns), positions < count (x3 only)."""
        ap, tri = (self.fwd_p, self._tri(True)) if forward else (self.bwd_p, self._tri(False))
        check(lib().nmx_gemm_chains_x3_lists(ptr(ap), self.lda, self.D, x, in_list, out, out_list, bias, tri, ldc,
                                             count, int(num_chains), ptr(self.split_buffer(ldc)), pe_in, pe_out,
                                             stream), "nmx_gemm_chains_x3_lists")

    def _tri(self, forward):
        """The products' triangle flag: T upper (T^T lower) triangular, or the full matrix (0)."""
        return (UPPER if forward else LOWER) if self.upper else 0

    def set(self, inverse_mass_matrix, mu=None):
        """inverse_mass_matrix [D, D] (or diagonal [D]); mu [D] or None (keep)."""
        imm = torch.as_tensor(inverse_mass_matrix, dtype=torch.float64).to(self.device)
        if imm.dim() == 1:
            imm = torch.diag(imm)
        if imm.shape != (self.D, self.D):
            raise ValueError(f"inverse_mass_matrix must be [{self.D}, {self.D}]")
        if self.blocks is not None:
            # per block the flipped Cholesky in the block's order (hmc_util.py:224-231 per
            # welford_covariance block, :439-515 structure), the diagonal block's square roots
            imm = self.blocks.mask(imm[None])[0]
            T = self.blocks.factor(imm[None])[0]
            self.upper = bool(torch.equal(torch.triu(T), T))
        else:
            # tril_inv = swap(chol(cov[::-1, ::-1])[::-1, ::-1])  (hmc_util.py:228-231); T = tril_inv^T
            T = torch.linalg.cholesky(imm.flip(0, 1)).flip(0, 1)
        self.inverse_mass_matrix = imm.clone()  # never the caller's tensor: snapshots share it
        self.version += 1
        self.T = T
        self._tinv = None
        self.fwd_t[:self.D, :self.D] = T.t().to(torch.float32)
        self.bwd_t[:self.D, :self.D] = T.to(torch.float32)
        if self.x3:
            s = native.stream_ptr()
            check(lib().nmx_gemm_x3_pack_a(ptr(self.fwd_t), self.lda, ptr(self.fwd_p), s), "nmx_gemm_x3_pack_a")
            check(lib().nmx_gemm_x3_pack_a(ptr(self.bwd_t), self.lda, ptr(self.bwd_p), s), "nmx_gemm_x3_pack_a")
        if mu is not None:
            self.mu.copy_(torch.as_tensor(mu, dtype=torch.float32))

    # reference-named views (HMCAdaptState fields)
    def mass_matrix_sqrt_inv(self):
        return self.T.t()  # tril_inv

    def tinv(self):
        """T^-1 (upper triangular, float64), by column chunks: hipBLAS trsm refuses very large
        right-hand sides (D = 10000 x 4096 fails to allocate its workspace)."""
        if self._tinv is None:
            if self.blocks is not None:  # block by block: T is block-diagonal up to the blocks' order
                inv = torch.zeros_like(self.T)
                for _, idx, dense in self.blocks.blocks:
                    idx = idx.to(self.device)
                    if dense:
                        inv[idx[:, None], idx[None, :]] = torch.linalg.inv(self.T[idx[:, None], idx[None, :]])
                    else:
                        inv[idx, idx] = 1.0 / self.T[idx, idx]
                self._tinv = inv
                return inv
            eye = torch.eye(self.D, dtype=torch.float64, device=self.device)
            cols = [torch.linalg.solve_triangular(self.T, eye[:, a:a + 1024], upper=True)
                    for a in range(0, self.D, 1024)]
            self._tinv = torch.cat(cols, dim=1)
        return self._tinv

    def mass_matrix_sqrt(self):
        # mass_matrix_sqrt = tril_inv^-1 = (T^T)^-1 = (T^-1)^T
        return self.tinv().t()

    def to_model(self, w, out, phase=None, num_chains=None, stream=0):
        """out[:, c] = mu + T w[:, c] for [D, ldc] buffers."""
        ldc = w.shape[-1]
        self.product(True, ptr(w), ptr(out), ptr(self.mu), ptr(phase), None, num_chains or ldc, ldc, stream)

    def grad_to_w(self, g, out, phase=None, num_chains=None, stream=0):
        """out[:, c] = T^T g[:, c]."""
        ldc = g.shape[-1]
        self.product(False, ptr(g), ptr(out), None, ptr(phase), None, num_chains or ldc, ldc, stream)

    def to_whitened(self, z):
        """w = T^-1 (z - mu) for z [D, n] (host-side re-expression at window ends)."""
        zz = z.to(torch.float64) - self.mu.to(torch.float64)[:, None]
        return (self.tinv() @ zz).to(torch.float32)

    def grad_to_model(self, g_w):
        """g_z = T^-T g_w for g_w [D, n]."""
        return (self.tinv().t() @ g_w.to(torch.float64)).to(torch.float32)


class WhitenedPotential(Potential):
    """U_w(w) = U(mu + T w), grad_w = T^T grad U (see module docstring); with `blocks` the T of a
    pooled structured mass (Whitening)."""

    def __init__(self, base: Potential, blocks=None):
        self.base = base
        self.blocks = blocks
        self.dim = base.dim
        self.sites = [(n, s, REAL) for n, s, _ in base.sites]
        self.whitening = None
        # the engine's arena is in chain rows ([ldc][D], k_chain_step): listed chains are
        # gathered from / scattered to rows (nmx_pack_rows / nmx_unpack_rows)
        self.rows = False
        # (NMX_DENSE_PACK_ROWS=1, experiments: the separate nmx_pack_rows pass, for A/B runs)
        self.fused_rows = os.environ.get("NMX_DENSE_PACK_ROWS", "0") != "1"

    def _bind(self, C, ldc, device):
        self.base.bind(C, ldc, device)
        if self.whitening is None or self.whitening.device != device:
            self.whitening = Whitening(self.dim, device, blocks=getattr(self, "blocks", None))
        self._rows_zg = None
        self.zb = torch.zeros(self.dim, ldc, dtype=torch.float32, device=device)
        self.gb = torch.zeros(self.dim, ldc, dtype=torch.float32, device=device)
        self.wp = torch.zeros(self.dim, ldc, dtype=torch.float32, device=device)   # packed w / g_w
        self.pe_p = torch.zeros(ldc, dtype=torch.float32, device=device)
        self.ident = torch.arange(ldc, dtype=torch.int32, device=device)
        self._batches = {}

    def _base_batch(self, ev):
        """Model-space batch: dense (phase-selected) or, for a compacted list, the packed
        positions [0, *active_count) through an identity list."""
        key = (ev.active_idx, ev.active_count, ev.pe, ev.phase)
        b = self._batches.get(key)
        if b is None:
            if ev.active_idx:
                b = EvalBatch(z=ptr(self.zb), grad=ptr(self.gb), pe=ptr(self.pe_p), phase=None,
                              active_idx=ptr(self.ident), active_count=ev.active_count, num_chains=ev.num_chains,
                              ldc=ev.ldc)
            else:
                b = EvalBatch(z=ptr(self.zb), grad=ptr(self.gb), pe=ev.pe, phase=ev.phase, active_idx=None,
                              active_count=None, num_chains=ev.num_chains, ldc=ev.ldc)
            self._batches[key] = b
        return b

    def _row_buffers(self, ldc):
        """Model-space z and gradient of the packed positions in rows ([ldc][D]), allocated on
        first use (the base potentials with evaluate_rows)."""
        if getattr(self, "_rows_zg", None) is None or self._rows_zg[0].shape[0] != ldc:
            self._rows_zg = tuple(torch.zeros(ldc, self.dim, dtype=torch.float32, device=self.zb.device)
                                  for _ in range(2))
        return self._rows_zg

    def evaluate(self, ev, stream):
        wt = self.whitening
        L = lib()
        C, ldc, D = ev.num_chains, ev.ldc, self.dim
        if ev.active_idx and self.rows and wt.x3 and self.fused_rows and hasattr(self.base, "evaluate_rows"):
            # a base potential that reads and writes rows (BNN): both products gather from and
            # store to rows -- the chain rows through the list, the model-space rows through the
            # identity -- and no transpose runs on either side of the base kernel
            zr, gr = self._row_buffers(ldc)
            wt.product_lists(True, ev.z, ev.active_idx, ptr(zr), ptr(self.ident), ptr(wt.mu), ev.active_count, C,
                             ldc, stream)
            self.base.evaluate_rows(self._base_batch(ev), ptr(zr), ptr(gr), stream)
            wt.product_lists(False, ptr(gr), ptr(self.ident), ev.grad, ev.active_idx, None, ev.active_count, C, ldc,
                             stream, ptr(self.pe_p), ev.pe)
            return
        if ev.active_idx:
            # compacted list: the products run on packed columns of the listed chains only
            if self.rows and wt.x3 and self.fused_rows:
                # gathered from the rows inside the operand split (no packed copy)
                wt.product_rows(ev.z, ev.active_idx, ev.active_count, ptr(self.zb), C, ldc, stream)
            else:
                if self.rows:
                    check(L.nmx_pack_rows(ev.z, ldc, D, ev.active_idx, ev.active_count, ptr(self.wp), ldc, stream),
                          "nmx_pack_rows")
                else:
                    check(L.nmx_pack_columns(ev.z, ldc, D, ev.active_idx, ev.active_count, ptr(self.wp), ldc,
                                             stream), "nmx_pack_columns")
                wt.product(True, ptr(self.wp), ptr(self.zb), ptr(wt.mu), None, ev.active_count, C, ldc, stream)
            self.base.evaluate(self._base_batch(ev), stream)
            if self.rows and wt.x3 and self.fused_rows:
                # stored to the chain rows by the product's epilogue (no packed copy)
                wt.product_to_rows(ptr(self.gb), ev.active_idx, ev.active_count, ev.grad, ptr(self.pe_p), ev.pe, C,
                                   ldc, stream)
                return
            wt.product(False, ptr(self.gb), ptr(self.wp), None, None, ev.active_count, C, ldc, stream)
            if self.rows:
                check(L.nmx_unpack_rows(ptr(self.wp), ldc, D, ev.active_idx, ev.active_count, ev.grad, ldc,
                                        ptr(self.pe_p), ev.pe, stream), "nmx_unpack_rows")
            else:
                check(L.nmx_unpack_columns(ptr(self.wp), ldc, D, ev.active_idx, ev.active_count, ev.grad, ldc,
                                           ptr(self.pe_p), ev.pe, stream), "nmx_unpack_columns")
            return
        # (a batch without a list is [D][ldc] in either layout: a chain-row engine passes
        # transposed copies, Engine._evaluate_all)
        wt.product(True, ev.z, ptr(self.zb), ptr(wt.mu), ev.phase, None, C, ldc, stream)
        self.base.evaluate(self._base_batch(ev), stream)
        wt.product(False, ptr(self.gb), ev.grad, None, ev.phase, None, C, ldc, stream)

    def flops_per_eval(self, num_chains):
        """Algorithmic FLOPs of the two triangular products (D^2 each per chain) -- the
        dense-matrix count 4 D^2 of SURVEY.md §8d halves because T is triangular (a structured
        T in a non-triangular coordinate order runs the full products)."""
        full = self.whitening is not None and not self.whitening.upper
        return (4.0 if full else 2.0) * self.dim * self.dim * num_chains


class PooledCovariance:
    """Sum / outer-product accumulators of model-space samples for one window (float64),
    shifted by a reference point to avoid cancellation; reduced over ranks on finalize."""

    def __init__(self, dim, device, shift):
        self.D = dim
        self.shift = shift.to(torch.float64).to(device)
        self.n = 0
        self.s1 = torch.zeros(dim, dtype=torch.float64, device=device)
        self.s2 = torch.zeros(dim, dim, dtype=torch.float64, device=device)

    def add(self, z):
        """z: [D, m] samples (columns)."""
        y = z.to(torch.float64) - self.shift[:, None]
        self.n += y.shape[1]
        self.s1 += y.sum(1)
        self.s2 += y @ y.t()

    def all_reduce(self, group=None):
        """Sum the moments over ranks: torch.distributed ranks, or the devices of one process
        (group = (shard.DeviceGroup, rank))."""
        if group is not None:
            g, rank = group
            n = torch.tensor([float(self.n)], dtype=torch.float64, device=self.s1.device)
            n, self.s1, self.s2 = g.all_reduce_sum(rank, [n, self.s1, self.s2])
            self.n = int(round(float(n.item())))
            return
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            n = torch.tensor([float(self.n)], dtype=torch.float64, device=self.s1.device)
            for t in (n, self.s1, self.s2):
                dist.all_reduce(t)
            self.n = int(round(float(n.item())))

    def finalize(self, regularize=True):
        """(cov, mean) as welford_covariance.final_fn (hmc_util.py:212-226) over the pool."""
        n = self.n
        if n < 2:
            raise RuntimeError("pooled dense adaptation needs at least 2 samples per window")
        mean_y = self.s1 / n
        cov = (self.s2 - n * torch.outer(mean_y, mean_y)) / (n - 1)
        cov = 0.5 * (cov + cov.t())
        if regularize:
            cov = (n / (n + 5.0)) * cov + 1e-3 * (5.0 / (n + 5.0)) * torch.eye(self.D, dtype=cov.dtype,
                                                                              device=cov.device)
        return cov, mean_y + self.shift


# ------------------------------------------------------------------ initial matrix as site blocks
def assemble_inverse_mass_matrix(sites, dense_mass, inverse_mass_matrix):
    """The initial inverse mass matrix in ravel coordinates from the reference's structural
    forms (hmc_util.py:439-487 _initialize_mass_matrix, dict branch; hmc.py:759-769 turns a model's
    dense_mass=True / False into [tuple(sorted(z))] / []): a dict {site group: block} or, with a
    structured dense_mass, an array (converted to {tuple(sorted(z)): array}).  Dense groups take
    their block from the dict (in the group's coordinate order) or the identity; the dict's other
    groups are diagonal blocks (a vector, or the diagonal of a matrix); the remaining sites get
    ones.  Returns a [D] diagonal when no group is dense, else a [D, D] float64 matrix.  A site in
    two groups raises the reference's assertion."""
    import numpy as np

    pos, o = {}, 0
    for name, shape, _ in sites:
        n = int(np.prod(shape, dtype=np.int64))
        pos[name] = (o, n)
        o += n
    D = o
    names = tuple(sorted(pos))
    if isinstance(dense_mass, bool):
        dense_mass = [names] if dense_mass else []
    dense_mass = [tuple(g) for g in dense_mass]
    imm = inverse_mass_matrix
    if not isinstance(imm, dict):
        imm = {names: imm}
    imm = {tuple(k): v for k, v in imm.items()}
    groups = list(dense_mass) + [k for k in imm if k not in dense_mass]
    got = sorted(n for g in groups for n in g)
    rest = tuple(sorted(set(pos) - set(got)))
    if sorted(got + list(rest)) != sorted(pos) or len(set(got)) != len(got):
        raise AssertionError("There seems to be a conflict of sites names specified in the initial "
                             "`inverse_mass_matrix` and in `dense_mass` argument.")
    idx = lambda g: np.concatenate([np.arange(pos[n][0], pos[n][0] + pos[n][1]) for n in g])  # noqa: E731
    full = np.zeros((D, D))
    for g in groups:
        ii = idx(g)
        v = imm.get(g)
        v = None if v is None else np.asarray(v.cpu() if hasattr(v, "cpu") else v, np.float64)
        if g in dense_mass:
            if v is None:
                v = np.eye(len(ii))
            elif v.ndim == 1:
                v = np.diag(v)
            if v.shape != (len(ii), len(ii)):
                raise ValueError(f"inverse_mass_matrix block {g} must be [{len(ii)}, {len(ii)}], got {v.shape}")
            full[np.ix_(ii, ii)] = v
        else:
            d = np.ones(len(ii)) if v is None else (np.diag(v) if v.ndim == 2 else v.reshape(-1))
            if d.shape != (len(ii),):
                raise ValueError(f"inverse_mass_matrix block {g} must have {len(ii)} diagonal entries")
            full[ii, ii] = d
    for n in rest:
        ii = idx((n,))
        full[ii, ii] = 1.0
    if not dense_mass:
        return torch.from_numpy(np.diag(full).copy())
    return torch.from_numpy(full)


# --------------------------------------------------------------------------------------- per chain
CHAIN_DENSE_MAX_D = 4096  # nmx_chain_matvec_tri / nmx_chain_welford_ws (dense_chain.hip)


class MassBlocks:
    """Structured mass matrix (dense_mass=[("x", "y"), ...], hmc.py:239-252; blocks as
    hmc_util.py:439-515 _initialize_mass_matrix builds them): one dense block per listed site
    group, its coordinates in the group's order (the reference's z_block = tuple(z[k] for k in
    site_names)), and one diagonal block over the remaining sites in sorted order.  Every block
    adapts by its own Welford covariance; here the per-chain dense Welford of all coordinates is
    masked to the blocks (its diagonal entries are the diagonal Welford's, bitwise: the same
    product delta_pre * delta_post), and each dense block is factored in its own order, so the
    whitening T_c is block-diagonal up to that ordering."""

    def __init__(self, sites, groups):
        import numpy as np

        pos, o = {}, 0
        for name, shape, _ in sites:
            n = int(np.prod(shape, dtype=np.int64))
            pos[name] = (o, n)
            o += n
        self.D = o
        used, self.blocks = set(), []
        for g in groups:
            for n in g:
                if n not in pos:
                    raise ValueError(f"dense_mass names {n!r}, which is not a latent site ({sorted(pos)})")
                if n in used:
                    raise ValueError(f"site {n!r} appears in two dense_mass groups")
                used.add(n)
            self.blocks.append((tuple(g), self._idx(pos, g), True))
        rest = tuple(sorted(set(pos) - used))
        if rest:
            self.blocks.append((rest, self._idx(pos, rest), False))

    @staticmethod
    def _idx(pos, names):
        return torch.cat([torch.arange(pos[n][0], pos[n][0] + pos[n][1]) for n in names])

    def mask(self, m):
        """[C, D, D]: keep each dense block's entries and the diagonal block's diagonal."""
        out = torch.zeros_like(m)
        for _, idx, dense in self.blocks:
            idx = idx.to(m.device)
            if dense:
                out[:, idx[:, None], idx[None, :]] = m[:, idx[:, None], idx[None, :]]
            else:
                out[:, idx, idx] = m[:, idx, idx]
        return out

    def factor(self, imm):
        """T [C, D, D] with T T^T = imm for a block-structured imm: per dense block the upper
        factor of the flipped Cholesky (hmc_util.py:224-231) in the block's order, per diagonal
        entry the square root."""
        T = torch.zeros_like(imm)
        for _, idx, dense in self.blocks:
            idx = idx.to(imm.device)
            if dense:
                sub = imm[:, idx[:, None], idx[None, :]]
                T[:, idx[:, None], idx[None, :]] = torch.linalg.cholesky(sub.flip(-2, -1)).flip(-2, -1)
            else:
                T[:, idx, idx] = torch.sqrt(imm[:, idx, idx])
        return T

    def split(self, m):
        """{site group: [C, n, n] (dense block, group order) or [C, n] (diagonal block)}."""
        out = {}
        for names, idx, dense in self.blocks:
            idx = idx.to(m.device)
            out[names] = m[:, idx[:, None], idx[None, :]] if dense else m[:, idx, idx]
        return out


def chain_dense_bytes(dim, num_chains):
    """Device bytes of per-chain dense mass state: T^T and T (f32), Welford m2 (f32), the
    float64 matrices held for HMCAdaptState / re-expression (inverse mass, T)."""
    return int(num_chains) * int(dim) * int(dim) * (3 * 4 + 2 * 8)


class ChainWhitening:
    """Per-chain z_c = T_c w_c with T_c T_c^T = M_c^-1 (T_c = tril_inv_c^T, hmc_util.py:224-231),
    every chain its own matrix as in the reference's vmapped adaptation (hmc.py:790-798).
    Holds T_c^T and T_c row-major for nmx_chain_matvec (forward / backward)."""

    def __init__(self, dim: int, num_chains: int, device, blocks=None):
        self.D, self.C = int(dim), int(num_chains)
        self.device = torch.device(device)
        self.blocks = blocks  # MassBlocks (structured mass) or None (one dense block)
        self.fwd = torch.zeros(self.C, self.D, self.D, dtype=torch.float32, device=self.device)  # T^T
        self.bwd = torch.zeros(self.C, self.D, self.D, dtype=torch.float32, device=self.device)  # T
        self.version = 0
        eye = torch.eye(self.D, dtype=torch.float64, device=self.device)
        self.set(eye.expand(self.C, self.D, self.D))

    def set(self, inverse_mass_matrix, mu=None):
        """inverse_mass_matrix [C, D, D] or a shared [D, D] / diagonal [D]; mu must be None
        (per-chain whitening is linear, z = T w)."""
        imm = torch.as_tensor(inverse_mass_matrix, dtype=torch.float64).to(self.device)
        if imm.dim() == 1:
            imm = torch.diag(imm)
        if imm.dim() == 2:
            imm = imm.expand(self.C, self.D, self.D)
        if imm.shape != (self.C, self.D, self.D):
            raise ValueError(f"inverse_mass_matrix must be [{self.C}, {self.D}, {self.D}]")
        if self.blocks is not None:
            imm = self.blocks.mask(imm)
            T = self.blocks.factor(imm)
        else:
            T = torch.linalg.cholesky(imm.flip(-2, -1)).flip(-2, -1)  # upper, T T^T = imm
        self.inverse_mass_matrix = imm.contiguous().clone()
        self.version += 1
        self.T = T
        self.fwd.copy_(T.transpose(-1, -2))
        self.bwd.copy_(T)

    def mass_matrix_sqrt_inv(self):
        return self.T.transpose(-1, -2)  # tril_inv

    def mass_matrix_sqrt(self):
        # tril_inv^-1 per chain (hmc_util.py:226-231 cov_inv_sqrt), in chunks of chains: batched
        # hipBLAS trsm fails to allocate its workspace for large right-hand sides (256 chains of
        # dim 512 x 512 identities), as for the pooled matrix's column chunks (Whitening.tinv)
        out = torch.empty(self.C, self.D, self.D, dtype=torch.float64, device=self.device)
        eye = torch.eye(self.D, dtype=torch.float64, device=self.device)
        step = max(1, (1 << 22) // (self.D * self.D))
        for a in range(0, self.C, step):
            Lt = self.T[a:a + step].transpose(-1, -2)
            rhs = eye.expand(Lt.shape[0], self.D, self.D)
            if self.blocks is not None:  # block-triangular up to the blocks' coordinate order
                out[a:a + step] = torch.linalg.solve(Lt, rhs)
            else:
                out[a:a + step] = torch.linalg.solve_triangular(Lt, rhs, upper=False)
        return out

    def tri(self, forward):
        """nmx_chain_matvec_tri's triangle flag: T_c upper triangular (one dense block) lets the
        large-dim products skip the zero rows of T_c^T (forward) / T_c (backward)."""
        return 0 if self.blocks is not None else (1 if forward else 2)

    def matvec(self, forward, x, out, list_, count, phase, num_chains, ldc, stream):
        """out[:, c] = T_c x[:, c] (forward) or T_c^T x[:, c] on raw pointers (nmx_chain_matvec_tri)."""
        check(lib().nmx_chain_matvec_tri(ptr(self.fwd if forward else self.bwd), self.D, x, out, ldc, list_, count,
                                         phase, int(num_chains), self.tri(forward), stream), "nmx_chain_matvec_tri")

    def to_model(self, w, out, phase=None, num_chains=None, stream=0):
        """out[:, c] = T_c w[:, c] for [D, ldc] buffers (chains < C)."""
        self.matvec(True, ptr(w), ptr(out), None, None, ptr(phase), num_chains or self.C, w.shape[-1], stream)

    def to_whitened(self, z):
        """w_c = T_c^-1 z_c for z [D, C]."""
        zc = z.to(torch.float64).t().unsqueeze(-1)  # [C, D, 1]
        if self.blocks is not None:
            return torch.linalg.solve(self.T, zc).squeeze(-1).t().to(torch.float32)
        return torch.linalg.solve_triangular(self.T, zc, upper=True).squeeze(-1).t().to(torch.float32)

    def grad_to_model(self, g_w):
        """g_z = T_c^-T g_w for g_w [D, C]."""
        gc = g_w.to(torch.float64).t().unsqueeze(-1)
        if self.blocks is not None:
            return torch.linalg.solve(self.T.transpose(-1, -2), gc).squeeze(-1).t().to(torch.float32)
        return torch.linalg.solve_triangular(self.T.transpose(-1, -2), gc, upper=False).squeeze(-1).t().to(
            torch.float32)


class ChainWhitenedPotential(Potential):
    """U_w(w) = U(T_c w), grad_w = T_c^T grad U, per chain (nmx_chain_matvec around the model)."""

    def __init__(self, base: Potential, blocks=None):
        self.base = base
        self.dim = base.dim
        self.sites = [(n, s, REAL) for n, s, _ in base.sites]
        self.whitening = None
        self.blocks = blocks

    def _bind(self, C, ldc, device):
        self.base.bind(C, ldc, device)
        if self.whitening is None or self.whitening.device != device or self.whitening.C != C:
            self.whitening = ChainWhitening(self.dim, C, device, self.blocks)
        self.zb = torch.zeros(self.dim, ldc, dtype=torch.float32, device=device)
        self.gb = torch.zeros(self.dim, ldc, dtype=torch.float32, device=device)
        self._batches = {}

    def evaluate(self, ev, stream):
        wt = self.whitening
        key = (ev.active_idx, ev.active_count, ev.pe, ev.phase, ev.num_chains)
        b = self._batches.get(key)
        if b is None:
            b = EvalBatch(z=ptr(self.zb), grad=ptr(self.gb), pe=ev.pe, phase=ev.phase, active_idx=ev.active_idx,
                          active_count=ev.active_count, num_chains=ev.num_chains, ldc=ev.ldc)
            self._batches[key] = b
        b.num_chains = ev.num_chains
        wt.matvec(True, ev.z, ptr(self.zb), ev.active_idx, ev.active_count, ev.phase, ev.num_chains, ev.ldc, stream)
        self.base.evaluate(b, stream)
        wt.matvec(False, ptr(self.gb), ev.grad, ev.active_idx, ev.active_count, ev.phase, ev.num_chains, ev.ldc, stream)


class ChainWelford:
    """welford_covariance(diagonal=False) of every chain (hmc_util.py:133-239), f32 on the
    device (nmx_chain_welford); final_fn per chain with the reference's regulariser."""

    def __init__(self, dim, num_chains, device):
        self.D, self.C = int(dim), int(num_chains)
        self.mean = torch.zeros(self.C, self.D, dtype=torch.float32, device=device)
        self.m2 = torch.zeros(self.C, self.D, self.D, dtype=torch.float32, device=device)
        nb = lib().nmx_chain_welford_work_bytes(self.D, self.C)  # dim > 256: delta vectors [C][2][D]
        self.work = torch.empty(nb, dtype=torch.uint8, device=device) if nb else None
        self.n = 0

    def add(self, z, stream=0):
        """z: [D, ldc] model-space draws of every chain."""
        self.n += 1
        check(lib().nmx_chain_welford_ws(ptr(z), self.D, z.shape[-1], self.C, self.n, ptr(self.mean), ptr(self.m2),
                                         ptr(self.work), stream), "nmx_chain_welford_ws")

    def finalize(self, regularize=True, blocks=None):
        """final_fn (hmc_util.py:198-237) per chain: cov [C, D, D] float64 (masked to the
        blocks of a structured mass matrix: each block's own final_fn)."""
        n = self.n
        if n < 2:
            raise RuntimeError("dense adaptation needs at least 2 draws per window")
        cov = self.m2.to(torch.float64) / (n - 1)
        if blocks is not None:
            cov = blocks.mask(cov)
        if regularize:
            cov = (n / (n + 5.0)) * cov + 1e-3 * (5.0 / (n + 5.0)) * torch.eye(self.D, dtype=cov.dtype,
                                                                              device=cov.device)
        # jnp.linalg.cholesky symmetrizes its input (symmetrize_input=True)
        return 0.5 * (cov + cov.transpose(-1, -2))
