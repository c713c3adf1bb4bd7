"""Is the in-process two-engine pooled-dense run deterministic?  Runs it three times and
compares the draws (debugging aid for test_parallel_pooled_dense_equals_torchrun)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from test_gpu_multi_device import TWO, pooled_run  # noqa: E402

runs = [pooled_run(TWO) for _ in range(3)]
for i in (1, 2):
    dx = (runs[i][0] - runs[0][0]).abs()
    per_chain = dx.reshape(dx.shape[0], -1).amax(1)
    print(f"run {i} vs 0: max |dx| {float(dx.max()):.3g}; chains differing: "
          f"{torch.nonzero(per_chain > 0).flatten().tolist()}; ns equal {bool(torch.equal(runs[i][1], runs[0][1]))}")
one = [pooled_run(None) for _ in range(2)]
print("one engine repeat max |dx|", float((one[1][0] - one[0][0]).abs().max()))
