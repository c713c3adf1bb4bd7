"""A/B timing of covtype potential libraries (scripts/ab_build.py): full batch (4096 chains)
and compacted-list launches of 16..2048 listed chains, each library in its own process,
outputs compared bitwise with the first library's.
usage: python scripts/ab_logreg.py build/ab/a/libnumpyro_amd.so build/ab/b/libnumpyro_amd.so ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, numpy as np, torch
sys.path.insert(0, @ROOT@)
from numpyro_amd import native, datasets
native.LIB_PATH = @LIB@
from numpyro_amd.potentials import LogisticRegression
X, y = datasets.covtype_synthetic(seed=0)
N, D = X.shape
dev = torch.device("cuda:0")
LDC = 4096
pot = LogisticRegression(torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev))
pot.bind(LDC, LDC, dev)
rs = np.random.RandomState(0)
Z = (datasets.COVTYPE_REF_COEFS[None, :] + 0.05 * rs.randn(LDC, D)).astype(np.float32)
z = torch.from_numpy(Z.T.copy()).to(dev)
g = torch.zeros(D, LDC, device=dev); pe = torch.zeros(LDC, device=dev)
s = native.stream_ptr()
res = {}
def timeit(ev, n=@REPS@):
    for _ in range(3): pot.evaluate(ev, s)
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): pot.evaluate(ev, s)
    b.record(); b.synchronize()
    return a.elapsed_time(b) / n
ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=LDC, ldc=LDC)
res["full"] = timeit(ev)
np.savez(@OUT@, pe=pe.cpu().numpy(), g=g.cpu().numpy())
idx = torch.arange(LDC, dtype=torch.int32, device=dev)
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
for n in (16, 128, 512, 1024, 2048):
    cnt.fill_(n)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), active_idx=native.ptr(idx),
                          active_count=native.ptr(cnt), num_chains=n, ldc=LDC)
    res[str(n)] = timeit(ev)
print("RESULT " + json.dumps(res))
"""

libs = sys.argv[1:]
reps = int(os.environ.get("AB_REPS", "20"))
rounds = int(os.environ.get("AB_ROUNDS", "2"))
outs = {}
table = {lib: [] for lib in libs}
for r in range(rounds):
    for i, lib in enumerate(libs):
        out = os.path.join(ROOT, "gpurun_out", f"ab_{i}.npz")
        code = CHILD.replace("@ROOT@", repr(ROOT)).replace("@LIB@", repr(os.path.abspath(lib))).replace(
            "@OUT@", repr(out)).replace("@REPS@", str(reps))
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        if p.returncode or not line:
            sys.exit(f"{lib} failed:\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}")
        table[lib].append(json.loads(line[0][7:]))
        outs[lib] = out
import numpy as np  # noqa: E402
base = np.load(outs[libs[0]])
for lib in libs:
    o = np.load(outs[lib])
    same = bool(np.array_equal(o["pe"], base["pe"]) and np.array_equal(o["g"], base["g"]))
    rel = float(np.max(np.abs(o["g"] - base["g"])) / np.max(np.abs(base["g"])))
    best = {k: min(t[k] for t in table[lib]) for k in table[lib][0]}
    tf = 4.0 * 581012 * 55 * 4096 / (best["full"] * 1e-3) / 1e12
    print(f"{lib}: full {best['full']:.3f} ms ({tf:.1f} TF/s) | " +
          " ".join(f"{k}:{v:.3f}" for k, v in best.items() if k != "full") +
          f" | bitwise {'==' if same else '!='} first (max rel grad diff {rel:.1e})", flush=True)
