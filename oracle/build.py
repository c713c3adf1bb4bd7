"""ORACLE build (test infrastructure only): compiles the C restatements under oracle/c/ into
oracle/_lib/*.so with gcc.  Called by __graft_entry__.build(); only bench.py's cpu_baseline
leg and tests load the result.  Built for x86-64-v4 (AVX-512: the covtype kernel's register
blocks are zmm intrinsics), which this container's Xeon and the GPU box's EPYC 9575F (Zen 5)
both implement, so the library built here runs there."""
from __future__ import annotations

import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "_lib")
FLAGS = ["-O3", "-march=x86-64-v4", "-ffast-math", "-fopenmp", "-fPIC", "-shared", "-std=c11", "-Wall"]
# per-file flags: the C NUTS keeps IEEE semantics (NaN energies, float32 operation order) and links
# the covtype potential of logreg_batch.c (built first: sorted order)
FILE_FLAGS = {"nuts_cpu": ["-O3", "-march=x86-64-v4", "-fno-math-errno", "-fopenmp", "-fPIC", "-shared", "-std=gnu11",
                           "-Wall"]}
FILE_LIBS = {"nuts_cpu": ["-L{lib}", "-llogreg_batch", "-Wl,-rpath,$ORIGIN"]}


def lib_path(name: str) -> str:
    return os.path.join(LIB_DIR, f"lib{name}.so")


def build(verbose: bool = False) -> None:
    os.makedirs(LIB_DIR, exist_ok=True)
    for src in sorted(glob.glob(os.path.join(HERE, "c", "*.c"))):
        name = os.path.splitext(os.path.basename(src))[0]
        out = lib_path(name)
        # a restatement may #include another (nuts_cpu.c includes logreg_batch.c): rebuild when any is newer
        newest = max(os.path.getmtime(p) for p in glob.glob(os.path.join(HERE, "c", "*.[ch]")))
        if os.path.exists(out) and os.path.getmtime(out) >= newest:
            continue
        libs = [a.format(lib=LIB_DIR) for a in FILE_LIBS.get(name, [])]
        r = subprocess.run(["gcc", *FILE_FLAGS.get(name, FLAGS), src, "-o", out, *libs, "-lm"], capture_output=True,
                           text=True)
        if r.returncode != 0:
            raise RuntimeError(f"gcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print("built", os.path.relpath(out, os.path.dirname(HERE)))
