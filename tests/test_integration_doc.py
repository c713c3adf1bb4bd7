"""INTEGRATION.md's reference-side ctypes stub is executed against the built library: its
struct layouts must have the sizes the library reports (nmx_struct_size) and the fields of
numpyro_amd/native.py, and every argtypes list it declares must equal native.SIGNATURES -- the
published binding cannot drift from include/numpyro_amd.h silently."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", doc, flags=re.S)
    stub = [b for b in blocks if "class NutsConfig" in b]
    assert len(stub) == 1, "INTEGRATION.md must hold exactly one ctypes stub block"
    return stub[0]


def _ctype_key(t):
    """A comparable description of a ctypes type (arrays and pointers by their element)."""
    if hasattr(t, "_length_"):
        return ("array", _ctype_key(t._type_), t._length_)
    if hasattr(t, "_type_") and isinstance(t._type_, type) and issubclass(t._type_, ctypes.Structure):
        return ("ptr", t._type_.__name__)
    if t is None:
        return None
    return ctypes.sizeof(t), getattr(t, "_type_", t.__name__)


def test_integration_stub_matches_library_and_native_binding(monkeypatch):
    from numpyro_amd import native

    monkeypatch.setenv("NUMPYRO_AMD_LIB", native.LIB_PATH)
    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md", "exec"), ns)  # its own asserts check the sizes
    lib = ns["lib"]
    assert lib.nmx_struct_size(0) == ctypes.sizeof(ns["NutsConfig"]) == ctypes.sizeof(native.NutsConfig)
    assert lib.nmx_struct_size(1) == ctypes.sizeof(ns["EvalBatch"]) == ctypes.sizeof(native.EvalBatch)
    for doc_cls, nat_cls in ((ns["NutsConfig"], native.NutsConfig), (ns["EvalBatch"], native.EvalBatch)):
        assert [(n, _ctype_key(t)) for n, t in doc_cls._fields_] == \
            [(n, _ctype_key(t)) for n, t in nat_cls._fields_], doc_cls.__name__
        for (n, _), (m, _) in zip(doc_cls._fields_, nat_cls._fields_):
            assert getattr(doc_cls, n).offset == getattr(nat_cls, m).offset, n
    sig = ns["SIGNATURES"]
    assert len(sig) >= 10
    for name, (res, args) in sig.items():
        assert name in native.SIGNATURES, f"{name}: not in native.SIGNATURES"
        nres, nargs = native.SIGNATURES[name]
        assert _ctype_key(res) == _ctype_key(nres), name
        assert [_ctype_key(a) for a in args] == [_ctype_key(a) for a in nargs], name
        assert hasattr(lib, name)
