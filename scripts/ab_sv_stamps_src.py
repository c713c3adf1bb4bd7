"""Write build/abx/nuts_svst.hip: nuts.hip with s_memtime phase accumulators in k_wide_persistent
(experiment only; never shipped).  Threads 0 (wave 0: the scalar logic) and 64 (wave 1: rows only)
of each workgroup add the cycles of every phase of every loop iteration and store the totals at
exit.  Build: AB_DIR=abx_svst python scripts/ab_build.py nuts.hip st=@build/abx/nuts_svst.hip;
run: scripts/sv_stamps.py."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "numpyro_amd", "csrc", "nuts.hip")).read()
a = src.index("void k_wide_persistent(StepArgs Pk, M m, int max_steps) {")
b = src.index("// ---- launched per-chain step for a chain-row arena")
body = src[a:b]
NPH = 12


def st(i):
    return f"{{ const unsigned long long t_ = __builtin_amdgcn_s_memtime(); acc_[{i}] += t_ - tp_; tp_ = t_; }}\n"


def ins(after, text, before=False):
    global body
    assert body.count(after) == 1, after
    body = body.replace(after, (text + after) if before else (after + text), 1)


ins("  for (int step = 0; step < max_steps; ++step) {\n",
    "  unsigned long long acc_[" + str(NPH) + "] = {}, tp_ = __builtin_amdgcn_s_memtime(); int nit_ = 0, nleaf_ = 0;\n",
    before=True)
ins("  for (int step = 0; step < max_steps; ++step) {\n", "    " + st(0) + "    ++nit_;\n")
ins("        wave_sums_to_lds<NW, NR>(red, lds, A, is_nuts);\n      }\n", "      " + st(1) + "      ++nleaf_;\n")
ins("      if (!CARRY && pl) lds_pre[lane] = pv;\n      __syncthreads();\n", "      " + st(3))
ins("      if (!CARRY && pl) lds_pre[lane] = pv;\n", "      " + st(2), before=True)
ins("    // scalar logic: wave 0 on the LDS state (lane 0 writes back)\n", "    " + st(4), before=True)
ins("        const float pe = m.fin(sums, gl, gs);\n",
    '        asm volatile("" :: "v"(pe), "v"(gs[0]), "v"(gs[1]));  // fin() complete before the stamp\n        ' + st(9))
ins("    __syncthreads();  // decisions published\n", "    " + st(5), before=True)
ins("    __syncthreads();  // decisions published\n", "    " + st(6))
ins("      if (D2.start_iter) {\n        const float t = wave_sum(ke0);\n",
    "      { const unsigned long long t_ = __builtin_amdgcn_s_memtime(), d_ = t_ - tp_; acc_[7] += d_;\n"
    "        if (act & ACT_TAKE_LEAF) { acc_[10] += d_; acc_[11] += 1; } tp_ = t_; }\n", before=True)
ins("      __syncthreads();  // this leaf's rows are written: the next leaf reads its neighbours' positions\n",
    "      " + st(8))
ins("  if (tid == 0) {\n    Arena al = Pk.a;  // addresses recomputed here",
    "  if ((tid == 0 || tid == 64) && blockIdx.x < 8192) {\n"
    "    unsigned long long* o_ = &g_sv_st[blockIdx.x][tid == 0 ? 0 : 1][0];\n"
    f"    for (int q = 0; q < {NPH}; ++q) __builtin_nontemporal_store(acc_[q], o_ + q);\n"
    f"    __builtin_nontemporal_store((unsigned long long)nit_, o_ + {NPH});\n"
    f"    __builtin_nontemporal_store((unsigned long long)nleaf_, o_ + {NPH + 1});\n"
    "  }\n", before=True)
src = src[:a] + body + src[b:]
decl = f"__device__ unsigned long long g_sv_st[8192][2][{NPH + 2}];\n"
i = src.index("template <int NT, int B, class M, bool CARRY>\n__global__ __launch_bounds__(NT, NMX_PX_OCC) void k_wide_persistent")
src = src[:i] + decl + src[i:]
src += f'''
extern "C" int nmx_x_sv_stamps(void* host) {{
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sv_st), sizeof(g_sv_st)) == hipSuccess ? 0 : 1;
}}
'''
os.makedirs(os.path.join(ROOT, "build", "abx"), exist_ok=True)
open(os.path.join(ROOT, "build", "abx", "nuts_svst.hip"), "w").write(src)
print("phases:", NPH)
