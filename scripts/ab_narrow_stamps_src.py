"""Write build/abx/potential_logreg_stamps.hip: potential_logreg.hip with s_memtime stamps in
the narrow tail form (experiment only; scripts/narrow_stamps.py reads them back)."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "numpyro_amd", "csrc", "potential_logreg.hip")).read()
src += '''
__device__ unsigned long long g_nx_stamps[8][8][160][4];
extern "C" int nmx_x_stamps(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nx_stamps), sizeof(g_nx_stamps)) == hipSuccess ? 0 : 1;
}
'''
src = src.replace('namespace {\n', 'extern __device__ unsigned long long g_nx_stamps[8][8][160][4];\nnamespace {\n', 1)
rep = [('''    auto iter = [&](int k, const f32x16& acc, f32x16& nxt) {
      x3_roles_barrier();  // DMA pair k landed; R(k - 1), SR(k - 2) written; pair k - 3's slots read
      issue_pair(k + 1);''', '''    const int wg = blockIdx.x;
    auto stamp = [&](int k, int f) {
      if (wg < 8 && lane == 0 && k < 158) {
        unsigned long long t = __builtin_amdgcn_s_memtime();
        __builtin_nontemporal_store(t, &g_nx_stamps[wg][w][k][f]);
      }
    };
    auto iter = [&](int k, const f32x16& acc, f32x16& nxt) {
      stamp(k, 0);
      x3_roles_barrier();  // DMA pair k landed; R(k - 1), SR(k - 2) written; pair k - 3's slots read
      stamp(k, 1);
      issue_pair(k + 1);
      stamp(k, 2);'''),
       ('''    for (int k = 0; k <= npairs + 1; k += 2) {
      iter(k, accA, accB);
      if (k + 1 <= npairs + 1) iter(k + 1, accB, accA);
    }
  }
  if (w >= 2 || pos >= ldc) return;''', '''    for (int k = 0; k <= npairs + 1; k += 2) {
      iter(k, accA, accB);
      stamp(k, 3);
      if (k + 1 <= npairs + 1) { iter(k + 1, accB, accA); stamp(k + 1, 3); }
    }
    if (wg < 8 && lane == 0) {
      unsigned long long rt = __builtin_amdgcn_s_memrealtime(), mt = __builtin_amdgcn_s_memtime();
      __builtin_nontemporal_store(rt, &g_nx_stamps[wg][w][159][0]);
      __builtin_nontemporal_store(mt, &g_nx_stamps[wg][w][159][1]);
    }
  }
  if (w >= 2 || pos >= ldc) return;'''),
       ('''  double pe = 0.0;
  if (nt > 0) {
    // the images of pair 0''', '''  double pe = 0.0;
  if (blockIdx.x < 8 && lane == 0) {
    unsigned long long rt = __builtin_amdgcn_s_memrealtime(), mt = __builtin_amdgcn_s_memtime();
    __builtin_nontemporal_store(rt, &g_nx_stamps[blockIdx.x][w][158][0]);
    __builtin_nontemporal_store(mt, &g_nx_stamps[blockIdx.x][w][158][1]);
  }
  if (nt > 0) {
    // the images of pair 0''')]
for a, b in rep:
    assert a in src, a[:60]
    src = src.replace(a, b)
os.makedirs(os.path.join(ROOT, "build", "abx"), exist_ok=True)
open(os.path.join(ROOT, "build", "abx", "potential_logreg_stamps.hip"), "w").write(src)
