"""Duration of the launched fused step with every chain DONE (the launch floor of k_nuts_step
itself) vs an empty kernel: covtype engine after a short run, 2000 back-to-back nmx_nuts_step
calls timed with HIP events.  usage: python scripts/step_floor.py [chains] [lib]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from numpyro_amd import native  # noqa: E402

if len(sys.argv) > 2:
    native.LIB_PATH = os.path.abspath(sys.argv[2])
from numpyro_amd import datasets  # noqa: E402
from numpyro_amd import potentials as P  # noqa: E402
from numpyro_amd.infer import MCMC, NUTS  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda:0")
X, y = datasets.covtype_synthetic(seed=0)
Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
mcmc = MCMC(NUTS(P.logistic_regression), num_warmup=5, num_samples=2, num_chains=C, progress_bar=False)
mcmc.run(0, Xd, yd)
eng = mcmc._engine
L = native.lib()
s = native.stream_ptr()
cfgp = ctypes.byref(eng.cfg)
arena = native.ptr(eng.arena)
fields = torch.zeros(1, len(native.COLLECT), eng.ldc, device=dev)
tr = eng._collect_codes()
eng.cfg.collection_size = 0


def step():
    native.check(L.nmx_nuts_step(cfgp, arena, None, native.ptr(fields), native.ptr(tr), s))


for _ in range(50):
    step()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(2000):
    step()
b.record()
b.synchronize()
print(f"{C} chains, all DONE: {a.elapsed_time(b) * 1e3 / 2000:.2f} us per nmx_nuts_step", flush=True)
