"""Write build/abx/nuts_stamps.hip: nuts.hip with s_memtime stamps at the phase boundaries of
the launched fused step (k_nuts_step, LIST = true; experiment only).  A block records its
stamps only in launches where one of its chains evaluates a leaf."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "numpyro_amd", "csrc", "nuts.hip")).read()
src += '''
__device__ unsigned long long g_st_stamps[1024][12];
extern "C" int nmx_x_step_stamps(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_st_stamps), sizeof(g_st_stamps)) == hipSuccess ? 0 : 1;
}
'''
src = src.replace('namespace {\n', 'extern __device__ unsigned long long g_st_stamps[1024][12];\nnamespace {\n', 1)
ST = '  const unsigned long long st_%d = __builtin_amdgcn_s_memtime();\n'
rep = [
    ('''  if (LIST && blockIdx.x == 0 && threadIdx.x == 0) a.counters[list_counter(cfg, cfg.parity ^ 1)] = 0;
''', '''  const unsigned long long st_rt0 = __builtin_amdgcn_s_memrealtime();
''' + ST % 0 + '''  if (LIST && blockIdx.x == 0 && threadIdx.x == 0) a.counters[list_counter(cfg, cfg.parity ^ 1)] = 0;
'''),
    ('''  const int ph_in = S.phase;  // the stored phase (begin_step's return resolves WAIT)
''', '''  const int ph_in = S.phase;  // the stored phase (begin_step's return resolves WAIT)
''' + ST % 1 + '''  const int st_any = __syncthreads_or(A.leaf ? 1 : 0);
'''),
    ('''  vblock_sum<NV, CPW, NPART>(red, lds, vw, cl);
  leaf_phase(cfg, S, A, 0.5f * red[0], seed, gch);''', ST % 2 + '''  vblock_sum<NV, CPW, NPART>(red, lds, vw, cl);
''' + ST % 3 + '''  leaf_phase(cfg, S, A, 0.5f * red[0], seed, gch);'''),
    ('''  float ke0[1] = {0.0f};
  const bool vec2 =''', ST % 4 + '''  float ke0[1] = {0.0f};
  const bool vec2 ='''),
    ('''  vblock_sum<NV, CPW, 1>(ke0, lds, vw, cl);
  if (A.start_iter) {''', ST % 5 + '''  vblock_sum<NV, CPW, 1>(ke0, lds, vw, cl);
''' + ST % 6 + '''  if (A.start_iter) {'''),
    ('''  if (vw == 0) end_step(cfg, a, c, valid, ph_in, S, A, LIST);
}''', '''  if (vw == 0) end_step(cfg, a, c, valid, ph_in, S, A, LIST);
''' + ST % 7 + '''  if (LIST && st_any && threadIdx.x == 0 && blockIdx.x < 1024) {
    unsigned long long* o = g_st_stamps[blockIdx.x];
    const unsigned long long v[8] = {st_0, st_1, st_2, st_3, st_4, st_5, st_6, st_7};
    for (int q = 0; q < 8; ++q) __builtin_nontemporal_store(v[q], o + q);
    __builtin_nontemporal_store((unsigned long long)st_any, o + 8);
    __builtin_nontemporal_store(st_rt0, o + 10);
    __builtin_nontemporal_store(__builtin_amdgcn_s_memrealtime(), o + 11);
  }
}'''),
]
for a, b in rep:
    assert a in src, a[:70]
    src = src.replace(a, b, 1)
os.makedirs(os.path.join(ROOT, "build", "abx"), exist_ok=True)
open(os.path.join(ROOT, "build", "abx", "nuts_stamps.hip"), "w").write(src)
