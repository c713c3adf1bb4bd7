"""Stage hashes of the pooled dense-mass window ends (test and diagnostic helper).

Wraps shard.DeviceGroup.all_reduce_sum, PooledCovariance.all_reduce and Engine._reexpress so
that every rank records, per window end, sha1 prefixes of the reduced moments (n, s1, s2), the
finalized (cov, mean), the factor T, T^-1 and the re-expressed positions.  Two runs that should
be bitwise equal (in-process two-device vs torchrun ranks) can then be compared stage by stage:
the first stage that differs locates a divergence."""
import contextlib
import hashlib

import torch

from numpyro_amd import shard
from numpyro_amd.dense import PooledCovariance
from numpyro_amd.engine import Engine


def h(t):
    return hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


@contextlib.contextmanager
def recording(rank_of=None, unlocked=False):
    """Yields the list the records are appended to: {"rank", "stage", ...hashes}."""
    rec = []
    orig_reduce, orig_pool_reduce = shard.DeviceGroup.all_reduce_sum, PooledCovariance.all_reduce
    orig_reexpress, orig_init = Engine._reexpress, shard.DeviceGroup.__init__

    def rank(eng=None):
        if eng is not None and eng.device_group is not None:
            return eng.device_group[1]
        d = torch.distributed
        return d.get_rank() if d.is_available() and d.is_initialized() else 0

    def init(self, size):
        orig_init(self, size)
        if unlocked:
            self.linalg_lock = contextlib.nullcontext()

    def pool_reduce(self, group=None):
        orig_pool_reduce(self, group)
        rec.append({"rank": group[1] if group is not None else rank(), "stage": "moments", "n": self.n,
                    "s1": h(self.s1), "s2": h(self.s2)})

    def reexpress(self, imm, mu, s):
        e = {"rank": rank(self), "stage": "window_end", "cov": h(imm), "mean": h(mu) if mu is not None else None}
        orig_reexpress(self, imm, mu, s)
        torch.cuda.synchronize()
        wt = self.potential.whitening
        e.update(T=h(wt.T), tinv=h(wt.tinv()), fwd_t=h(wt.fwd_t), w=h(self.view("z")[:, :self.C]))
        rec.append(e)

    shard.DeviceGroup.__init__ = init
    PooledCovariance.all_reduce = pool_reduce
    Engine._reexpress = reexpress
    try:
        yield rec
    finally:
        shard.DeviceGroup.__init__ = orig_init
        PooledCovariance.all_reduce = orig_pool_reduce
        Engine._reexpress = orig_reexpress
        shard.DeviceGroup.all_reduce_sum = orig_reduce


def by_rank(rec, r):
    return [{k: v for k, v in e.items() if k != "rank"} for e in rec if e["rank"] == r]


def first_difference(a, b, skip=()):
    """(index, stage, [keys]) of the first record of a that differs from b's, or None."""
    for i, (x, y) in enumerate(zip(a, b)):
        keys = [k for k in x if k not in skip and x.get(k) != y.get(k)]
        if keys:
            return i, x["stage"], keys
    if len(a) != len(b):
        return min(len(a), len(b)), "count", [len(a), len(b)]
    return None
