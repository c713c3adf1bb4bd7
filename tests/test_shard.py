"""Multi-GPU end-of-run exchange (numpyro_amd/shard.py) on CPU: single-process parity with
the host diagnostics (numpy restatement of numpyro/diagnostics.py), and world_size-2 gloo
runs (uneven chain shards) that must reproduce the single-process values -- the same code
path RCCL runs on the GPU box."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from numpyro_amd import diagnostics, shard
from numpyro_amd.dense import PooledCovariance


def _ar1(C, N, D, seed=0, phi=0.7):
    rs = np.random.RandomState(seed)
    x = np.zeros((C, N, D))
    x[:, 0] = rs.randn(C, D)
    for t in range(1, N):
        x[:, t] = phi * x[:, t - 1] + rs.randn(C, D)
    return x + rs.randn(C, 1, D) * 0.1


def test_single_process_matches_host_diagnostics():
    x = _ar1(6, 200, 3)
    np.testing.assert_allclose(shard.split_gelman_rubin(torch.from_numpy(x)).numpy(),
                               diagnostics.split_gelman_rubin(x), rtol=1e-10)
    np.testing.assert_allclose(shard.effective_sample_size(torch.from_numpy(x)).numpy(),
                               diagnostics.effective_sample_size(x), rtol=1e-8)
    s = shard.summary({"a": torch.from_numpy(x)})["a"]
    ref = diagnostics.summary({"a": x})["a"]
    for k in ("mean", "std", "median", "5.0%", "95.0%", "n_eff", "r_hat"):
        np.testing.assert_allclose(np.asarray(s[k]), np.asarray(ref[k]), rtol=1e-8, err_msg=k)


def test_shard_chains_partition():
    for C in (1, 7, 4096):
        for w in (1, 2, 3, 8):
            parts = [shard.shard_chains(C, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == C
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def _worker(rank, world, port, path, x, samples_z, x3d):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.shard_chains(x.shape[0], rank, world)
        xl = torch.from_numpy(x[lo:hi])
        out = {
            "rhat": shard.split_gelman_rubin(xl).numpy(),
            "ess": shard.effective_sample_size(xl).numpy(),
            "gather": shard.gather_chains(xl).numpy(),
        }
        s = shard.summary({"a": xl})["a"]
        out.update({f"sum_{k}": np.asarray(v) for k, v in s.items()})
        # config-4 scale path: chunks of a few coordinates, quantiles gathered to rank 0 in float32
        w = torch.from_numpy(x3d[lo:hi]).to(torch.float32)
        s3 = shard.summary({"w": w}, max_chunk_bytes=20000)["w"]
        out.update({f"chk_{k}": np.asarray(v) for k, v in s3.items()})
        # pooled dense-mass covariance over ranks (dense.PooledCovariance.all_reduce)
        lo2, hi2 = shard.shard_chains(samples_z.shape[1], rank, world)
        pool = PooledCovariance(samples_z.shape[0], "cpu", torch.zeros(samples_z.shape[0]))
        pool.add(torch.from_numpy(samples_z[:, lo2:hi2]))
        pool.all_reduce()
        cov, mean = pool.finalize(regularize=True)
        out["cov"], out["mean"], out["n"] = cov.numpy(), mean.numpy(), pool.n
        if rank == 0:
            np.savez(path, **out)
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_reproduce_single_process():
    x = _ar1(7, 120, 2, seed=3)  # 7 chains: uneven 4 / 3 shards
    zs = np.random.RandomState(1).randn(5, 301)
    x3d = _ar1(7, 60, 12, seed=5).reshape(7, 60, 3, 4).astype(np.float32)  # a [3, 4] site
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.npz")
        port = 29500 + (os.getpid() % 1000)
        mp.spawn(_worker, args=(2, port, path, x, zs, x3d), nprocs=2, join=True)
        r = np.load(path)
        # the chunked summary over uneven shards vs the host diagnostics (numpyro/diagnostics.py
        # restated) of all chains in one process
        ref3 = diagnostics.summary({"w": x3d.astype(np.float64)})["w"]
        for k in ("mean", "std", "median", "5.0%", "95.0%", "n_eff", "r_hat"):
            assert r[f"chk_{k}"].shape == (3, 4), k
            np.testing.assert_allclose(r[f"chk_{k}"], np.asarray(ref3[k]), rtol=1e-6, err_msg=k)
        xt = torch.from_numpy(x)
        np.testing.assert_allclose(r["rhat"], shard.split_gelman_rubin(xt).numpy(), rtol=1e-10)
        np.testing.assert_allclose(r["ess"], shard.effective_sample_size(xt).numpy(), rtol=1e-10)
        np.testing.assert_array_equal(r["gather"], x)
        ref = shard.summary({"a": xt})["a"]
        for k, v in ref.items():
            np.testing.assert_allclose(r[f"sum_{k}"], np.asarray(v), rtol=1e-10, err_msg=k)
        pool = PooledCovariance(5, "cpu", torch.zeros(5))
        pool.add(torch.from_numpy(zs))
        cov, mean = pool.finalize(regularize=True)
        assert int(r["n"]) == 301
        np.testing.assert_allclose(r["cov"], cov.numpy(), rtol=1e-10)
        np.testing.assert_allclose(r["mean"], mean.numpy(), rtol=1e-10)
        n = 301
        ref_cov = np.cov(zs) * n / (n + 5.0) + 1e-3 * 5.0 / (n + 5.0) * np.eye(5)
        np.testing.assert_allclose(r["cov"], ref_cov, rtol=1e-9)


def test_device_group_all_reduce_sum_in_rank_order():
    """shard.DeviceGroup (MCMC chain_method='parallel' in one process): every thread gets the
    rank-ordered sum; two ranks give exactly a + b, as an all_reduce does."""
    import threading

    from numpyro_amd.shard import DeviceGroup

    g = DeviceGroup(3)
    vals = [torch.tensor([0.1, 1e16], dtype=torch.float64) * (r + 1) for r in range(3)]
    out = [None] * 3

    def work(r):
        out[r] = g.all_reduce_sum(r, [vals[r], torch.tensor([float(r)])])

    ts = [threading.Thread(target=work, args=(r,)) for r in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ref = (vals[0] + vals[1]) + vals[2]
    for r in range(3):
        assert torch.equal(out[r][0], ref) and float(out[r][1]) == 3.0


def test_device_group_serializes_window_end_factorizations():
    """MCMC(devices=...) runs one host thread per device; their window-end factorizations
    (torch.linalg) take DeviceGroup.linalg_lock one at a time (Engine._reexpress)."""
    import threading
    import time

    g = shard.DeviceGroup(2)
    inside, peak = [0], [0]

    def work():
        with g.linalg_lock:
            inside[0] += 1
            peak[0] = max(peak[0], inside[0])
            time.sleep(0.02)
            inside[0] -= 1

    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert peak[0] == 1
