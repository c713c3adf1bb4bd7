"""Time the BNN potential alone vs the number of evaluated chains (all listed).
usage: python scripts/bench_bnn.py [H] [C1,C2,...]"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from numpyro_amd import datasets, native
from numpyro_amd.potentials import BNN

X, Y = datasets.bnn_data(N=100, D_X=3)
H = int(sys.argv[1]) if len(sys.argv) > 1 else 69
CS = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 8, 64, 256, 1024, 2048]
dev = torch.device("cuda:0")
for C in CS:
    ldc = (C + 63) // 64 * 64
    pot = BNN(X, Y, H)
    pot.bind(C, ldc, dev)
    D = pot.dim
    z = (0.3 * torch.randn(D, ldc, device=dev)).contiguous()
    g = torch.zeros(D, ldc, device=dev)
    pe = torch.zeros(ldc, device=dev)
    ev = native.EvalBatch(z=native.ptr(z), grad=native.ptr(g), pe=native.ptr(pe), num_chains=C, ldc=ldc)
    s = native.stream_ptr()
    for _ in range(3):
        pot.evaluate(ev, s)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    n = 20
    for _ in range(n):
        pot.evaluate(ev, s)
    b.record(); b.synchronize()
    ms = a.elapsed_time(b) / n
    flop = (6.0 * 100 * H * H + 6.0 * 100 * 3 * H) * C
    print(json.dumps({"H": H, "C": C, "ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 2)}), flush=True)
