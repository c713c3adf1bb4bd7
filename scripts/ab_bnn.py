"""A/B timing of the BNN potential between libraries (each in its own process).
usage: python scripts/ab_bnn.py lib1.so lib2.so ..."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, json
sys.path.insert(0, @ROOT@)
import numpy as np, torch
from numpyro_amd import datasets, native
native.LIB_PATH = @LIB@
from numpyro_amd.potentials import BNN
X, Y = datasets.bnn_data(N=100, D_X=3)
H = 69
dev = torch.device("cuda:0")
out = {}
for C in (1, 64, 512, 2048):
    ldc = (C + 63) // 64 * 64
    pot = BNN(X, Y, H); pot.bind(C, ldc, dev)
    D = pot.dim
    torch.manual_seed(0)
    z = (0.3 * torch.randn(D, ldc, device=dev)).contiguous()
    g = torch.zeros(D, ldc, device=dev); pe = torch.zeros(ldc, device=dev)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=C, ldc=ldc)
    s = native.stream_ptr()
    for _ in range(3): pot.evaluate(ev, s)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): pot.evaluate(ev, s)
    b.record(); b.synchronize()
    ms = a.elapsed_time(b) / 20
    out[C] = (ms, 6.0 * 100 * H * H * C / ms / 1e9)
    if C == 2048: np.save(@OUT@, np.concatenate([pe.cpu().numpy()[None, :64], g[:, :64].cpu().numpy()]))
print("RESULT", json.dumps(out))
"""
import numpy as np
res = {}
for i, lib in enumerate(sys.argv[1:]):
    out = os.path.join(ROOT, "gpurun_out", f"abbnn_{i}.npy")
    code = CHILD.replace("@ROOT@", repr(ROOT)).replace("@LIB@", repr(os.path.abspath(lib))).replace("@OUT@", repr(out))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT")]
    if p.returncode or not line:
        sys.exit(p.stdout[-2000:] + p.stderr[-3000:])
    res[lib] = (line[0], out)
base = np.load(res[sys.argv[1]][1])
for lib, (line, out) in res.items():
    o = np.load(out)
    print(lib, line, "max rel diff vs first:", float(np.max(np.abs(o - base)) / np.max(np.abs(base))))
