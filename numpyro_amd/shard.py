"""Chains across GPUs: one process per GPU, each owning a contiguous block of
global chain ids; no collective during sampling.  At the end of a run the only exchanges are

* cross-chain diagnostics -- split Gelman-Rubin (numpyro/diagnostics.py:64-80) and the
  Geyer initial-monotone ESS (:101-203) -- computed from per-chain sufficient statistics
  that are summed over ranks with one all_reduce each (O(draws x D) bytes, independent of
  the number of chains), and
* the quantiles of the summary (median, HPDI): each coordinate chunk's draws gathered to rank 0
  only, in their own precision, the small results broadcast (`summary`), and
* the sample gather (all_gather of [C_local, S, ...] blocks) when a caller wants every
  chain's draws on every rank (`gather_chains`).

`torch.distributed` with backend "nccl" is RCCL over xGMI on the GPU box; the same code
runs on "gloo" with CPU tensors (tests).  With one process every function reduces to the
single-process result (checked against numpyro_amd.diagnostics).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch


def shard_chains(num_chains, rank, world_size):
    """Contiguous chain shard [lo, hi) of `rank`."""
    per = num_chains // world_size
    rem = num_chains % world_size
    lo = rank * per + min(rank, rem)
    hi = lo + per + (1 if rank < rem else 0)
    return lo, hi


class DeviceGroup:
    """Chains of ONE process sharded over several devices, one host thread per device (MCMC
    chain_method="parallel" without torch.distributed; the reference pmaps over local devices,
    mcmc.py:700-715): the in-process counterpart of the torch.distributed ranks.  Shards are
    contiguous in global chain id (shard_chains), so every chain's draws equal the one-device
    and the torchrun runs bitwise; the only exchange while sampling is the pooled dense-mass
    moment sum at window ends (all_reduce_sum, ranks summed in rank order: for two devices
    the same single addition an all_reduce makes)."""

    def __init__(self, size):
        import threading

        self.size = int(size)
        self.barrier = threading.Barrier(self.size)
        self.slots = [None] * self.size
        # the window-end factorizations of the ranks' threads run one at a time: the linear
        # algebra libraries behind torch.linalg keep per-device state that concurrent host
        # threads on one device must not share (a rank's factorization then equals the torchrun
        # rank's, which has a process of its own)
        self.linalg_lock = threading.Lock()

    def all_reduce_sum(self, rank, tensors):
        """Every rank passes the same list of tensors; each gets back their sums over ranks (in
        rank order), on its own tensors' devices."""
        self.slots[rank] = list(tensors)
        self.barrier.wait()
        out = []
        for i, t in enumerate(tensors):
            acc = self.slots[0][i].to(t.device).clone()
            for r in range(1, self.size):
                acc += self.slots[r][i].to(t.device)
            out.append(acc)
        self.barrier.wait()  # every rank has read the slots before they are reused
        return out

    def abort(self):
        self.barrier.abort()


def dist_info():
    d = torch.distributed
    if d.is_available() and d.is_initialized():
        return d.get_rank(), d.get_world_size()
    return 0, 1


def _all_reduce(t):
    if dist_info()[1] > 1:
        torch.distributed.all_reduce(t)
    return t


def _next_fast_len(n):
    if n <= 2:
        return n
    while True:
        m = n
        for p in (2, 3, 5):
            while m % p == 0:
                m //= p
        if m == 1:
            return n
        n += 1


def _autocovariance(x):
    """Biased autocovariance along dim 1 of x [C, N, ...] (float64), FFT based
    (numpyro/diagnostics.py:101-147)."""
    n = x.shape[1]
    m2 = 2 * _next_fast_len(n)
    y = (x - x.mean(dim=1, keepdim=True)).movedim(1, -1)
    f = torch.fft.rfft(y, n=m2, dim=-1)
    ac = torch.fft.irfft(f * f.conj(), n=m2, dim=-1)[..., :n] / n
    return ac.movedim(-1, 1)


def split_gelman_rubin(x):
    """Split R-hat over all ranks' chains; x [C_local, N, ...] on this rank."""
    x = torch.as_tensor(x).to(torch.float64)
    half = x.shape[1] // 2
    xs = torch.cat([x[:, :half], x[:, -half:]], dim=0)
    m = xs.mean(dim=1)
    s2 = xs.var(dim=1, unbiased=True)
    k = torch.full_like(m[:1], float(xs.shape[0]))
    stats = _all_reduce(torch.cat([k, m.sum(0, keepdim=True), (m * m).sum(0, keepdim=True),
                                   s2.sum(0, keepdim=True)], dim=0))
    K, sm, smm, ss2 = stats[0], stats[1], stats[2], stats[3]
    w = ss2 / K
    var_m = (smm - sm * sm / K) / (K - 1)
    est = w * (half - 1) / half + var_m
    return torch.sqrt(est / w)


def effective_sample_size(x):
    """ESS over all ranks' chains (numpyro/diagnostics.py:150-203); x [C_local, N, ...]."""
    x = torch.as_tensor(x).to(torch.float64)
    N = x.shape[1]
    gamma = _autocovariance(x)  # [C, N, ...]
    mean_c = x.mean(dim=1)
    var_c = x.var(dim=1, unbiased=True)
    k = torch.full_like(mean_c[:1], float(x.shape[0]))
    head = torch.cat([k, mean_c.sum(0, keepdim=True), (mean_c * mean_c).sum(0, keepdim=True),
                      var_c.sum(0, keepdim=True)], dim=0)
    stats = _all_reduce(torch.cat([head, gamma.sum(0)], dim=0))
    C, sm, smm, svar = stats[0], stats[1], stats[2], stats[3]
    gamma_mean = stats[4:] / C
    w = svar / C
    est = w * (N - 1) / N
    if float(C.flatten()[0]) > 1:
        est = est + (smm - sm * sm / C) / (C - 1)
    else:
        w = est
    rho = 1.0 - (w - gamma_mean) / est
    rho[0] = 1.0
    pairs = rho[:-1:2] + rho[1::2]
    tail = torch.clamp(pairs[1:], min=0.0)
    mono = torch.cat([pairs[:1], torch.cummin(tail, dim=0).values], dim=0) if tail.shape[0] else pairs[:1]
    tau = -1.0 + 2.0 * mono.sum(dim=0)
    return C * N / tau


def gather_chains(x):
    """all_gather of per-rank chain blocks x [C_local, ...] -> [C_total, ...] on every rank
    (uneven shards are padded to the largest and trimmed)."""
    rank, world = dist_info()
    x = torch.as_tensor(x)
    if world == 1:
        return x
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    torch.distributed.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    mx = max(ns)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)]
    torch.distributed.all_gather(parts, pad.contiguous())
    return torch.cat([p[:k] for p, k in zip(parts, ns)], dim=0)


def _all_reduce_max(v):
    t = torch.tensor([float(v)], dtype=torch.float64)
    if dist_info()[1] > 1:
        if torch.distributed.get_backend() == "nccl":
            t = t.cuda()
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def _gather_to_root(x):
    """Chain blocks x [C_local, ...] of every rank concatenated in rank order on rank 0 (None on
    the others): torch.distributed.gather, uneven shards padded to the largest and trimmed."""
    rank, world = dist_info()
    if world == 1:
        return x
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    torch.distributed.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    pad = torch.zeros((max(ns),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    torch.distributed.gather(pad.contiguous(), parts, dst=0)
    if rank != 0:
        return None
    return torch.cat([p[:k] for p, k in zip(parts, ns)], dim=0)


def _broadcast(t):
    if dist_info()[1] > 1:
        torch.distributed.broadcast(t, src=0)
    return t


def _quantiles(xc, prob):
    """Median and the HPDI (numpyro/diagnostics.py:206-231 hpdi) of every column of xc
    [C_local, S, k] over all ranks' chains: the draws are gathered in their own precision to rank
    0 only (never float64 copies of every draw on every rank), sorted there on their device, and
    the [3, k] float64 result is broadcast back."""
    rank, world = dist_info()
    allx = _gather_to_root(xc)
    out = torch.empty((3, xc.shape[2]), dtype=torch.float64, device=xc.device)
    if rank == 0:
        flat = allx.reshape(-1, xc.shape[2])
        srt = torch.sort(flat, dim=0).values
        m = srt.shape[0]
        mid = srt[(m - 1) // 2].to(torch.float64), srt[m // 2].to(torch.float64)
        out[0] = 0.5 * (mid[0] + mid[1])  # np.median: the mean of the two middle draws
        w = int(np.floor(prob * m))
        lo, hi = srt[:m - w], srt[w:]
        i = torch.argmin((hi.to(torch.float64) - lo.to(torch.float64)), dim=0, keepdim=True)
        out[1] = torch.take_along_dim(lo, i, dim=0)[0].to(torch.float64)
        out[2] = torch.take_along_dim(hi, i, dim=0)[0].to(torch.float64)
        del allx, flat, srt
    return _broadcast(out)


def summary(samples, prob=0.90, quantiles=True, max_chunk_bytes=1 << 30):
    """Per-site mean / std / median / HPDI / n_eff / r_hat over every rank's chains
    (numpyro/diagnostics.py:234-294).  samples: {site: [C_local, S, ...]}.

    Scales to BASELINE config 4 (8192 chains x 1000 draws x 2519 coordinates = 82 GB of float32
    draws over the ranks): each site is processed in chunks of its flattened coordinates sized so
    that a chunk's float64 copy and FFT workspace (moments, split R-hat, ESS: reductions only, one
    all_reduce each) stay under `max_chunk_bytes` per rank, and the quantiles' chunk -- all
    ranks' draws of those coordinates in their own precision -- under it on rank 0, the only rank
    that receives them; the results are broadcast.  Chunk sizes come from the largest shard, so
    every rank runs the same collectives."""
    out = OrderedDict()
    for name, v in samples.items():
        x = torch.as_tensor(v)
        C, S = int(x.shape[0]), int(x.shape[1])
        ev = tuple(x.shape[2:])
        flat = x.reshape(C, S, -1)
        K = int(flat.shape[2])
        c_max = int(_all_reduce_max(C))
        c_tot = int(round(_all_reduce_sum_scalar(C)))
        # float64 chunk + centred copy + complex FFT of length 2 S (x2 for the product)
        per_col = c_max * S * 8 * 2 + c_max * (2 * _next_fast_len(S) + 2) * 16 * 2
        step = max(1, min(K, int(max_chunk_bytes // max(per_col, 1))))
        qstep = max(1, min(K, int(max_chunk_bytes // max(c_tot * S * (flat.element_size() * 2 + 8), 1))))
        cols = {k: [] for k in ("mean", "std", "median", "lo", "hi", "n_eff", "r_hat")}
        for k0 in range(0, K, step):
            xc = flat[:, :, k0:k0 + step].to(torch.float64)
            stats = _all_reduce(torch.cat([torch.full_like(xc[0, :1], float(C * S)),
                                           xc.sum(dim=(0, 1)).unsqueeze(0),
                                           (xc * xc).sum(dim=(0, 1)).unsqueeze(0)], dim=0))
            n, s1, s2 = stats[0], stats[1], stats[2]
            mean = s1 / n
            cols["mean"].append(mean)
            cols["std"].append(torch.sqrt(torch.clamp((s2 - n * mean * mean) / (n - 1), min=0.0)))
            cols["n_eff"].append(effective_sample_size(xc))
            cols["r_hat"].append(split_gelman_rubin(xc) if S >= 4 else torch.full_like(mean, float("nan")))
            del xc
        if quantiles:
            for k0 in range(0, K, qstep):
                q = _quantiles(flat[:, :, k0:k0 + qstep], prob)
                cols["median"].append(q[0])
                cols["lo"].append(q[1])
                cols["hi"].append(q[2])
        cat = {k: torch.cat(v).reshape(ev) for k, v in cols.items() if v}
        site = OrderedDict(mean=cat["mean"], std=cat["std"])
        if quantiles:
            site["median"] = cat["median"]
            site[f"{50 * (1 - prob):.1f}%"] = cat["lo"]
            site[f"{50 * (1 + prob):.1f}%"] = cat["hi"]
        site["n_eff"] = cat["n_eff"]
        site["r_hat"] = cat["r_hat"]
        out[name] = site
    return out


def _all_reduce_sum_scalar(v):
    t = torch.tensor([float(v)], dtype=torch.float64)
    if dist_info()[1] > 1:
        if torch.distributed.get_backend() == "nccl":
            t = t.cuda()
        torch.distributed.all_reduce(t)
    return float(t.item())
