"""Resident persistent-kernel workgroups per CU (experiment build): python scripts/occ_probe.py lib dim..."""
import ctypes
import sys

lib = ctypes.CDLL(sys.argv[1])
for dim in map(int, sys.argv[2:]):
    b, c = ctypes.c_int(), ctypes.c_int()
    st = lib.nmx_debug_persist_occupancy(dim, ctypes.byref(b), ctypes.byref(c))
    print(f"dim {dim}: status {st}, carry {c.value}, workgroups per CU {b.value}")
