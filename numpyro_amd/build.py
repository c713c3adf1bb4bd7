"""Build the HIP C-ABI library ``numpyro_amd/_lib/libnumpyro_amd.so`` for gfx950.

Plain ``hipcc`` invocations (no CMake, no torch extension): every ``csrc/*.hip`` and
``csrc/*.cpp`` is compiled to an object in ``build/``, then linked into one shared
library in-tree, so the built ``.so`` travels to the GPU box with the repo snapshot.
Objects are rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
LIB_DIR = os.path.join(HERE, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libnumpyro_amd.so")
# debug build: the NMX_DCHECK bounds / invariant checks compiled in (nmx_common.h), -g;
# loaded instead of the release library when NUMPYRO_AMD_DEBUG=1 (native.py)
DEBUG_OBJ_DIR = os.path.join(ROOT, "build", "obj_debug")
DEBUG_LIB_PATH = os.path.join(LIB_DIR, "libnumpyro_amd_debug.so")
DEBUG_FLAGS = ["-DNMX_DEBUG", "-g"]
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

COMMON_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-I" + os.path.join(ROOT, "include"),
    "-I" + CSRC,
    "-Wall",
    "-Wno-unused-function",
]


# per-file flags:
# * the covtype kernel's epilogue and residual split stay scalar VALU (the SLP vectorizer would
#   pair them into v_pk_*_f32, which issue slower beside MFMAs on gfx950; potential_logreg.hip
#   x3_epi_one);
# * no floating-point contraction in the step kernels and the small models' potentials: the
#   same device function is inlined into several kernels (the launched step, the persistent
#   schedule, the sync / async schedules), and whether the backend fuses a * b + c into an FMA
#   depends on each kernel's code generation -- with contraction off every kernel rounds every
#   product, so the schedules stay bitwise identical (and round like the NumPy oracle)
FILE_FLAGS = {"potential_logreg.hip": ["-fno-slp-vectorize"],
              "nuts.hip": ["-ffp-contract=off"],
              "potential_small.hip": ["-ffp-contract=off"]}


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def _stale(obj: str, src: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src, __file__, *headers])


def _compile(src: str, obj: str, extra=()) -> None:
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC, *COMMON_FLAGS, *extra, *lang, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")


def build(verbose: bool = False, jobs: int | None = None, debug: bool = False) -> str:
    obj_dir, lib_path = (DEBUG_OBJ_DIR, DEBUG_LIB_PATH) if debug else (OBJ_DIR, LIB_PATH)
    extra = DEBUG_FLAGS if debug else ()
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    headers = _headers()
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(obj_dir, os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(o, s, headers):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 4, max(1, len(todo)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, s, o, (*extra, *FILE_FLAGS.get(os.path.basename(s), ())))
                    for s, o in todo]
            for f in futs:
                f.result()
            if verbose:
                for s, _ in todo:
                    print("compiled", os.path.relpath(s, ROOT))
    if todo or not os.path.exists(lib_path):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print("linked", os.path.relpath(lib_path, ROOT))
    return lib_path


if __name__ == "__main__":
    build(verbose=True)
    if "--debug" in sys.argv:
        build(verbose=True, debug=True)
    sys.exit(0)
