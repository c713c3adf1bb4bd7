"""torch.distributed worker of tests/test_gpu_multi_device.py: one rank of a 2-rank run (gloo,
both ranks on cuda:0) of dense_mass='pooled' NUTS, the reference point the in-process
multi-device run must reproduce bitwise.  usage: torchrun ... dist_pooled_worker.py OUT"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import pooled_stages as PS  # noqa: E402
from test_gpu_multi_device import pooled_run  # noqa: E402

dist.init_process_group("gloo")
torch.cuda.set_device(0)
with PS.recording() as rec:
    x, ns = pooled_run(None)
recs = [None] * dist.get_world_size()
dist.all_gather_object(recs, list(rec))
x, ns = x.cpu().contiguous(), ns.cpu().contiguous()
xs = [torch.zeros_like(x) for _ in range(dist.get_world_size())]
nss = [torch.zeros_like(ns) for _ in range(dist.get_world_size())]
dist.all_gather(xs, x)
dist.all_gather(nss, ns)
if dist.get_rank() == 0:
    torch.save({"x": torch.cat(xs), "ns": torch.cat(nss), "stages": [e for r in recs for e in r]}, sys.argv[1])
dist.destroy_process_group()
