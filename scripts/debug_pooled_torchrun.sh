#!/bin/bash
# debugging aid: is the torchrun pooled-dense reference deterministic?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call29
mkdir -p $O
export PYTHONPATH=$PWD
for i in 1 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + i)) tests/dist_pooled_worker.py $O/ref$i.pt > $O/tr$i.log 2>&1 || exit 1
done
timeout -k 10 300 python - <<'PY' > $O/cmp.txt 2>&1 || exit 1
import sys, torch
sys.path.insert(0, "tests")
from test_gpu_multi_device import TWO, pooled_run
refs = [torch.load(f"gpurun_out/r05/call29/ref{i}.pt", weights_only=True) for i in (1, 2, 3)]
x2, n2 = pooled_run(TWO)
for i, r in enumerate(refs):
    d = (r["x"] - x2.cpu()).abs().reshape(r["x"].shape[0], -1).amax(1)
    d0 = (r["x"] - refs[0]["x"]).abs().max()
    print(f"torchrun {i}: vs in-process chains differing {torch.nonzero(d > 0).flatten().tolist()}; vs torchrun 0 max {float(d0):.3g}; ns eq {bool(torch.equal(r['ns'], n2.cpu()))}")
PY
cat $O/cmp.txt
