"""Build A/B variants of the library for kernel experiments: each variant recompiles one
source with extra -D flags and links it with the other objects of build/obj into
build/ab/<name>/libnumpyro_amd.so.  usage: python scripts/ab_build.py src.hip name='-DX=1 -DY' ..."""
import glob
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from numpyro_amd import build as B  # noqa: E402

B.build()
src = os.path.join(ROOT, "numpyro_amd", "csrc", sys.argv[1])
objs = [o for o in glob.glob(os.path.join(B.OBJ_DIR, "*.o")) if os.path.basename(o) != os.path.basename(src) + ".o"]
for spec in sys.argv[2:]:
    name, _, flags = spec.partition("=")
    if flags.startswith("@"):  # name=@path/to/variant.hip [flags]: another version of the source
        path, _, flags = flags[1:].partition(" ")
        src_v = os.path.abspath(path)
    else:
        src_v = src
    # AB_DIR: a directory the GPU snapshot carries (build/ab itself is gpurun-ignored)
    out = os.path.join(ROOT, "build", os.environ.get("AB_DIR", "ab"), name)
    os.makedirs(out, exist_ok=True)
    obj = os.path.join(out, os.path.basename(src) + ".o")
    cmd = [B.HIPCC, *B.COMMON_FLAGS, *B.FILE_FLAGS.get(os.path.basename(src), ()), "-DNMX_EXPERIMENT",
           *shlex.split(flags), "-x", "hip",
           "-c", src_v, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(f"{name}: compile failed\n{r.stderr[-3000:]}")
    lib = os.path.join(out, "libnumpyro_amd.so")
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, obj, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(f"{name}: link failed\n{r.stderr[-3000:]}")
    print("built", os.path.relpath(lib, ROOT))
