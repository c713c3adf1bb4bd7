"""Per-evaluation accuracy of config 3's pieces: the device against the float64 reference, next to
the NumPy float32 calibration against the same reference (the c3 parity leg's draw drift is ~2x
the calibration's; which piece carries it?).

  * BNN potential (H = 69, D = 5038) at C chain states: |pe - pe64| and max |g - g64| / max |g64|
  * the whitening product y = A x at D = 5038 with a triangular A (split-bf16 k_gemm_x3) vs
    float32 NumPy matmul: max |y - y64| / max |y64| per column

usage: python scripts/bnn_accuracy.py [C]  (GPU)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from numpyro_amd import datasets, native  # noqa: E402
from numpyro_amd.potentials import BNN  # noqa: E402
from oracle import batched as OB  # noqa: E402
from oracle import potentials as OP  # noqa: E402


def device_eval(pot, Z, dev):
    C, D = Z.shape
    ldc = (C + 63) // 64 * 64
    pot.bind(C, ldc, dev)
    z = torch.zeros(D, ldc, device=dev)
    z[:, :C] = torch.from_numpy(Z.T.astype(np.float32)).to(dev)
    g = torch.full((D, ldc), float("nan"), device=dev)
    pe = torch.full((ldc,), float("nan"), device=dev)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), phase=None, num_chains=C, ldc=ldc)
    pot.evaluate(ev, native.stream_ptr())
    torch.cuda.synchronize()
    return pe[:C].cpu().numpy().astype(np.float64), g[:, :C].cpu().numpy().T.astype(np.float64)


def stats(pe, g, pe64, g64):
    de = np.abs(pe - pe64)
    dg = np.abs(g - g64).max(1) / np.abs(g64).max(1)
    dgm = np.median(np.abs(g - g64) / (np.abs(g64).max(1, keepdims=True)), axis=1)
    return {"pe_abs_err_median": float(np.median(de)), "pe_abs_err_max": float(de.max()),
            "grad_maxrel_median": float(np.median(dg)), "grad_maxrel_max": float(dg.max()),
            "grad_medrel_median": float(np.median(dgm))}


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda:0")
    X, Y = datasets.bnn_data(N=100, D_X=3)
    H = 69
    ref = OP.BNN(X.astype(np.float64), Y.astype(np.float64), H)
    D = ref.dim
    rs = np.random.RandomState(5)
    # states of the posterior's scale: weights ~0.5, log precision ~1
    Z = (0.5 * rs.randn(C, D)).astype(np.float32)
    Z[:, 0] = rs.uniform(0.0, 2.0, C)
    out = {"C": C, "D": D}
    pe64 = np.empty(C)
    g64 = np.empty((C, D))
    for c in range(C):
        pe64[c], g64[c] = ref.pe_grad(Z[c].astype(np.float64))
    pe_d, g_d = device_eval(BNN(X, Y, H), Z, dev)
    pe_n, g_n = OB.BNNBatch(X, Y, H)(Z)
    out["bnn_device"] = stats(pe_d, g_d, pe64, g64)
    out["bnn_numpy_f32"] = stats(pe_n.astype(np.float64), g_n.astype(np.float64), pe64, g64)

    # whitening product at D: y = A x, A upper triangular (the forward product's shape)
    lib = native.lib()
    lda = lib.nmx_dense_padded_dim(D)
    Cg = 256
    ldc = Cg
    A64 = np.triu(rs.randn(D, D) / np.sqrt(D))
    x64 = rs.randn(D, Cg)
    A32, x32 = A64.astype(np.float32), x64.astype(np.float32)
    y64 = A32.astype(np.float64) @ x32.astype(np.float64)  # At holds A^T: the product is A x
    At = torch.zeros(lda, lda, device=dev)
    At[:D, :D] = torch.from_numpy(A32.T.copy()).to(dev)
    xd = torch.from_numpy(x32).to(dev)
    yd = torch.empty(D, ldc, device=dev)
    s = native.stream_ptr()
    nws = lib.nmx_gemm_chains_workspace_bytes(D, ldc)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev) if nws else None
    Ap = torch.empty(lib.nmx_gemm_x3_packed_a_bytes(lda), dtype=torch.uint8, device=dev)
    sp = torch.empty(lib.nmx_gemm_x3_split_bytes(lda, ldc), dtype=torch.uint8, device=dev)
    native.check(lib.nmx_gemm_x3_pack_a(native.ptr(At), lda, native.ptr(Ap), s))
    native.check(lib.nmx_gemm_chains_x3(native.ptr(Ap), lda, D, native.ptr(xd), native.ptr(yd), None, 1, ldc,
                                        None, None, Cg, native.ptr(sp), native.ptr(ws), s))
    torch.cuda.synchronize()
    y_d = yd.cpu().numpy().astype(np.float64)
    y_n = (A32 @ x32).astype(np.float64)
    sc = np.abs(y64).max(0)
    for name, y in (("gemm_device_x3", y_d), ("gemm_numpy_f32", y_n)):
        r = np.abs(y - y64).max(0) / sc
        out[name] = {"maxrel_median": float(np.median(r)), "maxrel_max": float(r.max()),
                     "medrel_median": float(np.median(np.median(np.abs(y - y64), 0) / sc))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
