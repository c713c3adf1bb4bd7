"""The C-ABI library loads and exports every symbol include/numpyro_amd.h declares."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "numpyro_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nmx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from numpyro_amd import native

    lib = native.lib()
    declared = _declared_symbols()
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in header but not exported"
    # every ctypes signature we bind is declared in the header
    assert set(native.SIGNATURES) <= set(declared)
    assert lib.nmx_version() >= 1


def test_struct_layouts_match():
    import ctypes

    from numpyro_amd import native

    assert native.lib().nmx_struct_size(0) == ctypes.sizeof(native.NutsConfig)
    assert native.lib().nmx_struct_size(1) == ctypes.sizeof(native.EvalBatch)


def test_field_enum_matches_header():
    from numpyro_amd import native

    src = open(os.path.join(ROOT, "include", "numpyro_amd.h")).read()
    body = src[src.index("enum nmx_field"):]
    body = body[:body.index("};")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = [n.strip().split("=")[0].strip() for n in body.split("{", 1)[1].split(",")]
    names = [n for n in names if n and n != "NMX_NUM_FIELDS"]
    assert [n[len("NMX_F_"):].lower() for n in names] == native.FIELDS


def test_invalid_argument_reports_error():
    from numpyro_amd import native

    st = native.lib().nmx_selftest_mfma(None, None, None, 3, None)
    assert st == 1
    assert b"even" in native.lib().nmx_last_error()


@pytest.mark.gpu
def test_mfma_f32_fragment_layout(device):
    """A = I (identity in the first 32 k), asymmetric B: C must equal B exactly."""
    import torch
    from numpyro_amd import native

    K = 64
    rs = np.random.RandomState(1)
    A = np.zeros((32, K), np.float32)
    A[:, :32] = np.eye(32, dtype=np.float32)
    A[:, 32:] = rs.randn(32, 32).astype(np.float32)
    B = rs.randn(K, 32).astype(np.float32)
    dA, dB = torch.from_numpy(A).to(device), torch.from_numpy(B).to(device)
    dC = torch.zeros(32, 32, device=device)
    native.check(native.lib().nmx_selftest_mfma(native.ptr(dA), native.ptr(dB), native.ptr(dC), K,
                                                 native.stream_ptr()))
    torch.cuda.synchronize()
    C = dC.cpu().numpy()
    ref = A.astype(np.float64) @ B.astype(np.float64)
    np.testing.assert_allclose(C, ref, rtol=1e-5, atol=1e-5)
