// Per-chain dense mass matrices (dim <= 4096): the reference's vmapped semantics (numpyro/infer/hmc.py:790-798
// runs init_kernel per chain, so every chain adapts its own dense M^-1 with
// welford_covariance(diagonal=False), hmc_util.py:133-239).
//
// As for the pooled matrix (dense.hip), chain c runs identity-mass NUTS on w with z = T_c w,
// T_c T_c^T = M_c^-1 (T_c upper triangular, T_c = tril_inv_c^T), so the state machine is
// unchanged and the model's potential is wrapped by two per-chain matrix-vector products:
//   z = T_c w  before,   g_w = T_c^T g_z  after.
// Both are  out[a] = sum_b M[c][b][a] in[b]  with M = T_c^T (row-major T^T = column-major T,
// forward) or M = T_c (row-major, backward): one wave per chain, lanes over `a` (coalesced row
// reads of M), `in` broadcast from LDS.  HBM traffic per product: D^2 x 4 B per chain (D = 55:
// 12 KB), memory-bound; a chain's products never depend on which chains share the launch.
//
// k_chain_welford: welford_covariance update_fn (hmc_util.py:172-196) for every chain in f32,
// the reference's arithmetic: n += 1; delta_pre = z - mean; mean += delta_pre / n;
// delta_post = z - mean; M2 += outer(delta_post, delta_pre).
#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

constexpr int CW_MAX_D = 256;    // one wave per chain (4 outputs per lane) up to this dim
constexpr int CWB_MAX_D = 4096;  // the block-per-(chain, 256 outputs) form above it

// one wave per list position; 4 waves per workgroup
__global__ __launch_bounds__(256) void k_chain_matvec(const float* __restrict__ M, int D, const float* __restrict__ in,
                                                      float* __restrict__ out, int ldc,
                                                      const int32_t* __restrict__ list,
                                                      const int32_t* __restrict__ count,
                                                      const int32_t* __restrict__ phase, int num_chains) {
  __shared__ float xs[4][CW_MAX_D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pos = blockIdx.x * 4 + w;
  int c = -1;
  if (list) {
    if (pos < *count) c = list[pos];
  } else if (pos < num_chains && (phase == nullptr || phase[pos] >= NMX_PH_LEAF)) {
    c = pos;
  }
  if (c < 0) return;  // wave-uniform: no block-wide barrier below
  for (int b = lane; b < D; b += 64) xs[w][b] = in[(size_t)b * ldc + c];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const float* Mc = M + (size_t)c * D * D;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int b = 0; b < D; ++b) {
    const float x = xs[w][b];
    const float* row = Mc + (size_t)b * D;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = lane + 64 * q;
      if (a < D) acc[q] = __builtin_fmaf(row[a], x, acc[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int a = lane + 64 * q;
    if (a < D) out[(size_t)a * ldc + c] = acc[q];
  }
}

// one wave per chain: mean [C][D], m2 [C][D][D] (row a = delta_post[a] x delta_pre[.])
__global__ __launch_bounds__(256) void k_chain_welford(const float* __restrict__ z, int D, int ldc, int C, int n,
                                                       float* __restrict__ mean, float* __restrict__ m2) {
  __shared__ float pre[4][CW_MAX_D], post[4][CW_MAX_D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 4 + w;
  if (c >= C) return;
  float* mc = mean + (size_t)c * D;
  for (int a = lane; a < D; a += 64) {
    const float x = z[(size_t)a * ldc + c];
    const float m = mc[a];
    const float dp = x - m;
    const float mn = m + dp / (float)n;
    mc[a] = mn;
    pre[w][a] = dp;
    post[w][a] = x - mn;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  float* m2c = m2 + (size_t)c * D * D;
  for (int a = 0; a < D; ++a) {
    const float pa = post[w][a];
    float* row = m2c + (size_t)a * D;
    for (int b = lane; b < D; b += 64) row[b] = row[b] + pa * pre[w][b];
  }
}

// D > CW_MAX_D (up to CWB_MAX_D): one workgroup per (listed chain, 256 outputs), one output
// per thread; the chain's input column staged in LDS once per workgroup.  Rows b of M[c] stream
// as 1 KB coalesced segments (four waves x 64 lanes x 4 B), eight rows in flight per thread;
// the sum over b runs in increasing b with one fma per row (the order of k_chain_matvec's, so a
// chain's result depends on D alone, never on which chains share the launch).  HBM-bound:
// D^2 x 4 B per chain and product, halved by `tri` (T_c upper triangular: forward M = T_c^T has
// zero rows b < a, backward M = T_c zero rows b > a; the skipped terms are exact zeros).
// An input of the wrong sign of infinity would make 0 x inf = NaN in the skipped terms: those
// positions are non-finite either way (the step maps their energies to +inf).
__global__ __launch_bounds__(256) void k_chain_matvec_big(const float* __restrict__ M, int D,
                                                          const float* __restrict__ in, float* __restrict__ out,
                                                          int ldc, const int32_t* __restrict__ list,
                                                          const int32_t* __restrict__ count,
                                                          const int32_t* __restrict__ phase, int num_chains, int tri) {
  extern __shared__ float xs[];  // D floats
  const int pos = blockIdx.x;
  int c = -1;
  if (list) {
    if (pos < *count) c = list[pos];
  } else if (pos < num_chains && (phase == nullptr || phase[pos] >= NMX_PH_LEAF)) {
    c = pos;
  }
  if (c < 0) return;  // block-uniform
  const int t = threadIdx.x;
  for (int b = t; b < D; b += 256) xs[b] = in[(size_t)b * ldc + c];
  __syncthreads();
  const int a0 = blockIdx.y * 256, a = a0 + t;
  const int b0 = tri == 1 ? a0 : 0;
  const int b1 = tri == 2 ? min(D, a0 + 256) : D;
  if (a >= D) return;
  const float* Mc = M + (size_t)c * D * D + a;
  float acc = 0.0f;
  int b = b0;
  for (; b + 8 <= b1; b += 8) {
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = Mc[(size_t)(b + j) * D];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_fmaf(m[j], xs[b + j], acc);
  }
  for (; b < b1; ++b) acc = __builtin_fmaf(Mc[(size_t)b * D], xs[b], acc);
  out[(size_t)a * ldc + c] = acc;
}

// welford_covariance update_fn for D > CW_MAX_D in two launches (a chain's m2 is D^2 floats:
// one wave per chain is too serial).  1: per chain, delta_pre = z - mean, the new mean and
// delta_post = z - mean_new (k_chain_welford's arithmetic) into work [C][2][D]; 2: per (chain,
// 16 rows of m2), row a += delta_post[a] * delta_pre (coalesced over the row).
__global__ __launch_bounds__(256) void k_chain_welford_vec(const float* __restrict__ z, int D, int ldc, int C, int n,
                                                           float* __restrict__ mean, float* __restrict__ work) {
  const int c = blockIdx.x;
  if (c >= C) return;
  float* mc = mean + (size_t)c * D;
  float* pre = work + (size_t)c * 2 * D;
  float* post = pre + D;
  for (int a = threadIdx.x; a < D; a += 256) {
    const float x = z[(size_t)a * ldc + c];
    const float m = mc[a];
    const float dp = x - m;
    const float mn = m + dp / (float)n;
    mc[a] = mn;
    pre[a] = dp;
    post[a] = x - mn;
  }
}

constexpr int CWB_ROWS = 16;
__global__ __launch_bounds__(256) void k_chain_welford_m2(int D, int C, const float* __restrict__ work,
                                                          float* __restrict__ m2) {
  const int c = blockIdx.x;
  const int a0 = blockIdx.y * CWB_ROWS;
  if (c >= C) return;
  const float* pre = work + (size_t)c * 2 * D;
  const float* post = pre + D;
  float* m2c = m2 + (size_t)c * D * D;
  const int a1 = min(D, a0 + CWB_ROWS);
  for (int a = a0; a < a1; ++a) {
    const float pa = post[a];
    float* row = m2c + (size_t)a * D;
    for (int b = threadIdx.x; b < D; b += 256) row[b] = row[b] + pa * pre[b];
  }
}

}  // namespace

extern "C" int nmx_chain_matvec_tri(const float* M, int dim, const float* in, float* out, int ldc,
                                    const int32_t* list, const int32_t* count, const int32_t* phase, int num_chains,
                                    int tri, void* stream) {
  if (!M || !in || !out) return nmx_fail(NMX_ERR_INVALID, "chain_matvec: NULL operand");
  if (dim <= 0 || dim > CWB_MAX_D || ldc % 64 || num_chains <= 0 || num_chains > ldc || (list && !count) || tri < 0 ||
      tri > 2)
    return nmx_fail(NMX_ERR_INVALID, "chain_matvec: bad sizes (dim=%d ldc=%d C=%d tri=%d)", dim, ldc, num_chains,
                    tri);
  if (in == out) return nmx_fail(NMX_ERR_INVALID, "chain_matvec: in and out must not alias");
  if (dim <= CW_MAX_D) {
    hipLaunchKernelGGL(k_chain_matvec, dim3((num_chains + 3) / 4), dim3(256), 0, (hipStream_t)stream, M, dim, in,
                       out, ldc, list, count, phase, num_chains);
    return nmx_check_launch("k_chain_matvec");
  }
  hipLaunchKernelGGL(k_chain_matvec_big, dim3(num_chains, (dim + 255) / 256), dim3(256), dim * sizeof(float),
                     (hipStream_t)stream, M, dim, in, out, ldc, list, count, phase, num_chains, tri);
  return nmx_check_launch("k_chain_matvec_big");
}

extern "C" size_t nmx_chain_welford_work_bytes(int dim, int num_chains) {
  return dim > CW_MAX_D ? (size_t)num_chains * 2 * dim * sizeof(float) : 0;
}

extern "C" int nmx_chain_welford_ws(const float* z, int dim, int ldc, int num_chains, int n, float* mean, float* m2,
                                    float* work, void* stream) {
  if (!z || !mean || !m2) return nmx_fail(NMX_ERR_INVALID, "chain_welford: NULL operand");
  if (dim <= 0 || dim > CWB_MAX_D || ldc % 64 || num_chains <= 0 || num_chains > ldc || n < 1)
    return nmx_fail(NMX_ERR_INVALID, "chain_welford: bad sizes (dim=%d ldc=%d C=%d n=%d)", dim, ldc, num_chains, n);
  if (dim <= CW_MAX_D) {
    hipLaunchKernelGGL(k_chain_welford, dim3((num_chains + 3) / 4), dim3(256), 0, (hipStream_t)stream, z, dim, ldc,
                       num_chains, n, mean, m2);
    return nmx_check_launch("k_chain_welford");
  }
  if (!work) return nmx_fail(NMX_ERR_INVALID, "chain_welford: dim > %d needs nmx_chain_welford_work_bytes", CW_MAX_D);
  hipLaunchKernelGGL(k_chain_welford_vec, dim3(num_chains), dim3(256), 0, (hipStream_t)stream, z, dim, ldc, num_chains,
                     n, mean, work);
  if (int st = nmx_check_launch("k_chain_welford_vec")) return st;
  hipLaunchKernelGGL(k_chain_welford_m2, dim3(num_chains, (dim + CWB_ROWS - 1) / CWB_ROWS), dim3(256), 0,
                     (hipStream_t)stream, dim, num_chains, work, m2);
  return nmx_check_launch("k_chain_welford_m2");
}

extern "C" int nmx_chain_matvec(const float* M, int dim, const float* in, float* out, int ldc, const int32_t* list,
                                const int32_t* count, const int32_t* phase, int num_chains, void* stream) {
  return nmx_chain_matvec_tri(M, dim, in, out, ldc, list, count, phase, num_chains, 0, stream);
}

extern "C" int nmx_chain_welford(const float* z, int dim, int ldc, int num_chains, int n, float* mean, float* m2,
                                 void* stream) {
  return nmx_chain_welford_ws(z, dim, ldc, num_chains, n, mean, m2, nullptr, stream);
}
