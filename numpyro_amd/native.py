"""ctypes binding of the C-ABI in ``include/numpyro_amd.h``.

``torch`` is imported first on purpose: torch-ROCm ships its own ``libamdhip64.so.7``;
loading it before our library makes the dynamic linker resolve our ``DT_NEEDED``
``libamdhip64.so.7`` to that same copy, so the ``hipStream_t`` handles torch gives us
belong to the runtime our kernels launch through.

The product path never falls back: if the library is missing this raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NMX_LIB", os.path.join(_HERE, "_lib", "libnumpyro_amd.so"))

_lib = None

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_size = ctypes.c_size_t
c_float = ctypes.c_float
c_double = ctypes.c_double
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); kept in sync with include/numpyro_amd.h (tests check it).
SIGNATURES: dict[str, tuple] = {
    "nmx_version": (c_int, []),
    "nmx_last_error": (ctypes.c_char_p, []),
    "nmx_selftest_philox": (c_int, [c_vp, c_vp, c_int, c_vp]),
    "nmx_selftest_mfma": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp]),
}


class NativeError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle; raises if the library is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"numpyro_amd native library not found at {LIB_PATH}; "
                "run `python -m numpyro_amd.build` (or __graft_entry__.build())"
            )
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().nmx_last_error().decode(errors="replace")
        raise NativeError(f"{what or 'numpyro_amd'} failed (status {status}): {msg}")


def stream_ptr(stream=None) -> int:
    """Raw hipStream_t of a torch stream (the current stream by default)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return 0
    return int(t.data_ptr())
