"""Write build/abx/pl_fin_stamps.hip: potential_logreg.hip with s_memtime stamps in
k_logreg_finalize (experiment only)."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "numpyro_amd", "csrc", "potential_logreg.hip")).read()
src += '''
__device__ unsigned long long g_fin_stamps[64][4][8];
extern "C" int nmx_x_fin_stamps(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fin_stamps), sizeof(g_fin_stamps)) == hipSuccess ? 0 : 1;
}
'''
src = src.replace('namespace {\n', 'extern __device__ unsigned long long g_fin_stamps[64][4][8];\nnamespace {\n', 1)
rep = [('''  const int sp0 = w * S / FIN_WAVES, sp1 = (w + 1) * S / FIN_WAVES;
''', '''  const int sp0 = w * S / FIN_WAVES, sp1 = (w + 1) * S / FIN_WAVES;
  const unsigned long long f0 = __builtin_amdgcn_s_memtime(), fr0 = __builtin_amdgcn_s_memrealtime();
'''),
       ('''  __syncthreads();
  if (w != 0 || c < 0) return;
  if (d < D) {''', '''  const unsigned long long f1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  const unsigned long long f2 = __builtin_amdgcn_s_memtime();
  if (lane == 0 && blockIdx.x == 0 && blockIdx.y < 64) {
    unsigned long long* o = g_fin_stamps[blockIdx.y][w];
    __builtin_nontemporal_store(f0, o);
    __builtin_nontemporal_store(f1, o + 1);
    __builtin_nontemporal_store(f2, o + 2);
    __builtin_nontemporal_store(fr0, o + 4);
    __builtin_nontemporal_store(__builtin_amdgcn_s_memrealtime(), o + 5);
  }
  if (w != 0 || c < 0) return;
  if (d < D) {''')]
for a, b in rep:
    assert a in src, a[:60]
    src = src.replace(a, b, 1)
open(os.path.join(ROOT, "build", "abx", "pl_fin_stamps.hip"), "w").write(src)
