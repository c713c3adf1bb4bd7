"""Write build/abx/potential_bnn_stamps.hip: potential_bnn.hip with s_memtime stamps at the
phase boundaries of k_bnn_c3 (experiment only; never shipped): thread 0 of each of the first
1024 workgroups stores its 11 stamps.  Build: AB_DIR=abx_bnnst python scripts/ab_build.py
potential_bnn.hip st=@build/abx/potential_bnn_stamps.hip; run: scripts/bnn_stamps.py."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "numpyro_amd", "csrc", "potential_bnn.hip")).read()
a = src.index("__global__ __launch_bounds__(THREADS, 2) void k_bnn_c3(")
b = src.index("size_t lds_bytes_c3()")
body = src[a:b]
ST = "  if (threadIdx.x == 0) st_[{i}] = __builtin_amdgcn_s_memtime();\n"
marks = [
    ("  const float* z = zr + (size_t)pos * D;\n", 0, "before"),
]
# stamp after every __syncthreads(); inside the kernel body, in order
parts = body.split("  __syncthreads();\n")
out = parts[0]
for i, p in enumerate(parts[1:]):
    out += "  __syncthreads();\n" + ST.format(i=i + 1) + p
body = out
body = body.replace("  const float* z = zr + (size_t)pos * D;\n",
                    "  unsigned long long st_[12];\n" + ST.format(i=0) + "  const float* z = zr + (size_t)pos * D;\n", 1)
n_sync = len(parts) - 1
body = body.replace("  const float esq_t = block_sum256(esq, red);",
                    ST.format(i=n_sync + 1) + "  const float esq_t = block_sum256(esq, red);", 1)
end = body.rindex("}")
body = body[:end] + ST.format(i=n_sync + 2) + '''  if (threadIdx.x == 0 && blockIdx.x < 1024)
    for (int q = 0; q < 12; ++q) __builtin_nontemporal_store(q <= N_ST ? st_[q] : 0ull, &g_bnn_st[blockIdx.x][q]);
''' + body[end:]
body = body.replace("N_ST", str(n_sync + 2))
src = src[:a] + body + src[b:]
src = src.replace("namespace {\n", "__device__ unsigned long long g_bnn_st[1024][12];\nnamespace {\n", 1)
src += '''
extern "C" int nmx_x_bnn_stamps(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bnn_st), sizeof(g_bnn_st)) == hipSuccess ? 0 : 1;
}
'''
os.makedirs(os.path.join(ROOT, "build", "abx"), exist_ok=True)
open(os.path.join(ROOT, "build", "abx", "potential_bnn_stamps.hip"), "w").write(src)
print("stamps:", n_sync + 3)
