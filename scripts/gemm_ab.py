"""A/B of the whitening product k_gemm_x3 between library builds (each in its own process): the
upper / lower triangular split-bf16 products of BASELINE configs 2 (D = 10000, 4096 chains) and
3 (D = 5038, 2048 chains), timed with events, and the output of one product for a bitwise check.
usage: python scripts/gemm_ab.py lib1.so lib2.so ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, json
sys.path.insert(0, @ROOT@)
import numpy as np, torch
from numpyro_amd import native
native.LIB_PATH = @LIB@
lib = native.lib()
dev = torch.device("cuda:0")
out = {}
for D, C in ((10000, 4096), (5038, 2048)):
    lda = lib.nmx_dense_padded_dim(D); ldc = (C + 63) // 64 * 64
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randn(D, D, generator=g).to(dev)
    x = torch.randn(D, ldc, generator=g).to(dev)
    s = native.stream_ptr()
    for tri in (1, 2):
        At = torch.zeros(lda, lda, device=dev)
        At[:D, :D] = (torch.triu(A) if tri == 1 else torch.tril(A)).t()
        Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=dev)
        sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=dev)
        nws = lib.nmx_gemm_chains_workspace_bytes(D, ldc)
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)
        y = torch.empty(D, ldc, device=dev)
        native.check(lib.nmx_gemm_x3_pack_a(native.ptr(At), lda, native.ptr(Ap), s))
        run = lambda: native.check(lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(x), native.ptr(y), None,
                                                          tri, ldc, None, None, C, native.ptr(sp), native.ptr(ws), s))
        for _ in range(3): run()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20): run()
        b.record(); b.synchronize()
        ms = a.elapsed_time(b) / 20
        out[f"D{D}_C{C}_tri{tri}"] = (round(ms, 4), round(2.0 * D * D / 2 * C / ms / 1e9, 1))
        if D == 5038 and tri == 1:
            np.save(@OUT@, y[:, :64].cpu().numpy())
print("RESULT", json.dumps(out))
"""
import numpy as np  # noqa: E402

res = {}
for i, lib in enumerate(sys.argv[1:]):
    out = os.path.join(ROOT, "gpurun_out", f"abgemm_{i}.npy")
    code = CHILD.replace("@ROOT@", repr(ROOT)).replace("@LIB@", repr(os.path.abspath(lib))).replace("@OUT@", repr(out))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT")]
    if p.returncode or not line:
        sys.exit(p.stdout[-2000:] + p.stderr[-3000:])
    res[lib] = (line[0], out)
base = np.load(res[sys.argv[1]][1])
for lib, (line, out) in res.items():
    o = np.load(out)
    print(lib, line, "max rel diff vs first:", float(np.max(np.abs(o - base)) / np.max(np.abs(base))))
