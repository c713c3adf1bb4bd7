// Potentials of wide-latent models whose cost is O(D) per chain: stochastic volatility
// (examples/stochastic_volatility.py:57-65, D = T + 2) and the centred funnel
// (examples/funnel.py:44-46, D = dim).  Both are HBM-bound.  The grid is chain groups x
// D-slices (so any C fills the GPU): a block owns 64 chains x one slice of 64 coordinates
// (256-byte coalesced rows of the chain-major layout), writes the coordinate gradients
// and per-slice partial sums; a finalize kernel sums the slices in a fixed order and
// writes U and the gradients of the global parameters.  Gradients are hand-derived
// (SURVEY.md Appendix A, C2 and C4).
#include <math.h>

#include <algorithm>

#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

// digamma for x > 0: recurrence up to x >= 6, then the asymptotic series.
__device__ __forceinline__ float nmx_digammaf(float x) {
  float acc = 0.0f;
  while (x < 6.0f) {
    acc -= 1.0f / x;
    x += 1.0f;
  }
  const float inv = 1.0f / x;
  const float inv2 = inv * inv;
  const float series =
      inv2 * (1.0f / 12.0f - inv2 * (1.0f / 120.0f - inv2 * (1.0f / 252.0f - inv2 * (1.0f / 240.0f - inv2 / 132.0f))));
  return acc + logf(x) - 0.5f * inv - series;
}

// D-split: block = 64 list positions x WAVES waves over one slice of SLICE coordinates;
// per-slice partial sums go to a workspace [NS][NSUM][ldc] and a finalize kernel adds the
// slices in a fixed order.  The slicing depends on D only, so a chain's U and dU do not
// depend on how many chains share a launch.
constexpr int WAVES = 4;
constexpr int SLICE = 64;
constexpr int NSUM = 4;

__host__ __device__ inline int num_slices(int D) { return (D + SLICE - 1) / SLICE; }

template <int N>
__device__ __forceinline__ void wave_block_sum(float (&v)[N], float* lds) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) lds[(i * WAVES + wv) * 64 + lane] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) s += lds[(i * WAVES + w) * 64 + lane];
    v[i] = s;
  }
}

// z = (a = log nu, s[0..T-1], b = log sigma); slices over t.
__global__ __launch_bounds__(64 * WAVES) void k_sv_part(const float* __restrict__ ret, int T, nmx_eval_batch ev,
                                                      float* __restrict__ part) {
  __shared__ float lds[NSUM * WAVES * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + lane);
  const bool act = c >= 0;
  if (!__syncthreads_or(act)) return;
  const int ldc = ev.ldc;
  const float* z = ev.z;
  const float a = act ? z[c] : 0.f;
  const float b = act ? z[(size_t)(T + 1) * ldc + c] : 0.f;
  const float nu = expf(a);
  const float inv_sig2 = expf(-2.0f * b);
  const float inv_nu = 1.0f / nu;
  float sums[NSUM] = {0.f, 0.f, 0.f, 0.f};  // sum d^2, sum log1p(q), sum q/(1+q), sum s
  const int t0 = blockIdx.y * SLICE, t1 = min(T, t0 + SLICE);
  if (act) {
    for (int t = t0 + wv; t < t1; t += WAVES) {
      const float s = z[(size_t)(1 + t) * ldc + c];
      const float sp = t > 0 ? z[(size_t)t * ldc + c] : 0.0f;
      const float sn = t + 1 < T ? z[(size_t)(2 + t) * ldc + c] : 0.0f;
      const float d = s - sp;
      const float dn = t + 1 < T ? sn - s : 0.0f;
      const float r = ret[t];
      const float q = r * r * expf(-2.0f * s) * inv_nu;
      const float qq = q / (1.0f + q);
      sums[0] += d * d;
      sums[1] += log1pf(q);
      sums[2] += qq;
      sums[3] += s;
      // dU/ds_t = -( -(d_t - d_{t+1})/sigma^2 + (nu+1) q/(1+q) - 1 )
      ev.grad[(size_t)(1 + t) * ldc + c] = (d - dn) * inv_sig2 - (nu + 1.0f) * qq + 1.0f;
    }
  }
  wave_block_sum<NSUM>(sums, lds);
  if (act && wv == 0) {
#pragma unroll
    for (int i = 0; i < NSUM; ++i) part[((size_t)blockIdx.y * NSUM + i) * ldc + c] = sums[i];
  }
}

// Slice sums in a fixed order: wave w adds slices w, w+WAVES, ..., then wave 0 adds the
// waves in order.
template <int N>
__device__ __forceinline__ bool slice_sums(const float* __restrict__ part, int ns, int ldc, int c, float (&v)[N],
                                           float* lds) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = 0.0f;
  if (c >= 0)
    for (int sl = wv; sl < ns; sl += WAVES)
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] += part[((size_t)sl * N + i) * ldc + c];
  wave_block_sum<N>(v, lds);
  return wv == 0 && c >= 0;
}

__global__ __launch_bounds__(64 * WAVES) void k_sv_fin(int T, nmx_eval_batch ev, const float* __restrict__ part) {
  __shared__ float lds[NSUM * WAVES * 64];
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + (threadIdx.x & 63));
  if (!__syncthreads_or(c >= 0)) return;
  const int ldc = ev.ldc;
  float sums[NSUM];
  if (!slice_sums<NSUM>(part, num_slices(T), ldc, c, sums, lds)) return;
  const float a = ev.z[c];
  const float b = ev.z[(size_t)(T + 1) * ldc + c];
  const float nu = expf(a);
  const float inv_sig2 = expf(-2.0f * b);
  const float inv_nu = 1.0f / nu;
  const float Tf = (float)T;
  const float sig = expf(b);
  const float lg = lgammaf(0.5f * nu) - lgammaf(0.5f * (nu + 1.0f));
  // log p
  float lp = 3.912023005428146f - 50.0f * sig + b;                        // Exponential(50) + log|J|
  lp += -0.5f * sums[0] * inv_sig2 - Tf * b - Tf * 0.9189385332046727f;  // GaussianRandomWalk
  lp += -2.302585092994046f - 0.1f * nu + a;                              // Exponential(0.1) + log|J|
  lp += -0.5f * (nu + 1.0f) * sums[1] - sums[3]
        - Tf * (0.5f * logf(nu) + 0.5723649429247001f + lg);              // StudentT(nu, 0, e^s)
  ev.pe[c] = -lp;
  const float dig = nmx_digammaf(0.5f * nu) - nmx_digammaf(0.5f * (nu + 1.0f));
  const float ga = nu * (-0.1f - 0.5f * sums[1] + 0.5f * (nu + 1.0f) * inv_nu * sums[2]
                         - 0.5f * Tf * inv_nu - 0.5f * Tf * dig) + 1.0f;
  const float gb = -50.0f * sig + 1.0f + sums[0] * inv_sig2 - Tf;
  ev.grad[c] = -ga;
  ev.grad[(size_t)(T + 1) * ldc + c] = -gb;
}

// funnel, centred: z = (x[K], y); U = y^2/18 + log(3 sqrt(2 pi)) + sum_i [x_i^2 e^-y / 2 + y/2 + log(2 pi)/2]
__global__ __launch_bounds__(64 * WAVES) void k_funnel_part(int D, nmx_eval_batch ev, float* __restrict__ part) {
  __shared__ float lds[WAVES * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + lane);
  const bool act = c >= 0;
  if (!__syncthreads_or(act)) return;
  const int ldc = ev.ldc;
  const int K = D - 1;
  const float y = act ? ev.z[(size_t)K * ldc + c] : 0.0f;
  const float e = expf(-y);
  float sx[1] = {0.0f};
  const int i0 = blockIdx.y * SLICE, i1 = min(K, i0 + SLICE);
  if (act) {
    for (int i = i0 + wv; i < i1; i += WAVES) {
      const size_t idx = (size_t)i * ldc + c;
      const float x = ev.z[idx];
      sx[0] += x * x;
      ev.grad[idx] = x * e;
    }
  }
  wave_block_sum<1>(sx, lds);
  if (act && wv == 0) part[(size_t)blockIdx.y * ldc + c] = sx[0];
}

__global__ __launch_bounds__(64 * WAVES) void k_funnel_fin(int D, nmx_eval_batch ev, const float* __restrict__ part) {
  __shared__ float lds[WAVES * 64];
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + (threadIdx.x & 63));
  if (!__syncthreads_or(c >= 0)) return;
  const int ldc = ev.ldc;
  const int K = D - 1;
  float sv[1];
  if (!slice_sums<1>(part, num_slices(K), ldc, c, sv, lds)) return;
  const float sx = sv[0];
  const float y = ev.z[(size_t)K * ldc + c];
  const float e = expf(-y);
  const float Kf = (float)K;
  ev.pe[c] = y * y / 18.0f + 2.0175508218727822f + 0.5f * e * sx + Kf * (0.5f * y + 0.9189385332046727f);
  ev.grad[(size_t)K * ldc + c] = y / 9.0f + 0.5f * Kf - 0.5f * e * sx;
}

// funnel, non-centred (examples/funnel.py:49, reparam(model, {"x": LocScaleReparam(0)}),
// numpyro/infer/reparam.py:104-145): z = (x_decentered[K], y), x = exp(y/2) x_decentered is a
// deterministic site (host side).  U = y^2/18 + log(3 sqrt(2 pi)) + sum_i [x_i^2/2 + log(2 pi)/2];
// dU/dx_i = x_i, dU/dy = y/9.
__global__ __launch_bounds__(64 * WAVES) void k_funnel_nc_part(int D, nmx_eval_batch ev, float* __restrict__ part) {
  __shared__ float lds[WAVES * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + lane);
  const bool act = c >= 0;
  if (!__syncthreads_or(act)) return;
  const int ldc = ev.ldc;
  const int K = D - 1;
  float sx[1] = {0.0f};
  const int i0 = blockIdx.y * SLICE, i1 = min(K, i0 + SLICE);
  if (act) {
    for (int i = i0 + wv; i < i1; i += WAVES) {
      const size_t idx = (size_t)i * ldc + c;
      const float x = ev.z[idx];
      sx[0] += x * x;
      ev.grad[idx] = x;
    }
  }
  wave_block_sum<1>(sx, lds);
  if (act && wv == 0) part[(size_t)blockIdx.y * ldc + c] = sx[0];
}

__global__ __launch_bounds__(64 * WAVES) void k_funnel_nc_fin(int D, nmx_eval_batch ev,
                                                            const float* __restrict__ part) {
  __shared__ float lds[WAVES * 64];
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + (threadIdx.x & 63));
  if (!__syncthreads_or(c >= 0)) return;
  const int ldc = ev.ldc;
  const int K = D - 1;
  float sv[1];
  if (!slice_sums<1>(part, num_slices(K), ldc, c, sv, lds)) return;
  const float y = ev.z[(size_t)K * ldc + c];
  ev.pe[c] = y * y / 18.0f + 2.0175508218727822f + 0.5f * sv[0] + (float)K * 0.9189385332046727f;
  ev.grad[(size_t)K * ldc + c] = y / 9.0f;
}

// chain-group blocks needed: positions >= num_chains hold no chain (with a compacted list,
// num_chains bounds its count -- nmx_eval_batch)
inline int groups_of(const nmx_eval_batch* ev) { return (std::min(ev->num_chains, ev->ldc) + 63) / 64; }

int check_ev(const nmx_eval_batch* ev, const void* workspace) {
  if (!ev || !ev->z || !ev->grad || !ev->pe) return nmx_fail(NMX_ERR_INVALID, "eval batch has NULL pointers");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains || ev->ldc % 64)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  if (!workspace) return nmx_fail(NMX_ERR_INVALID, "workspace is NULL (nmx_pe_wide_workspace_bytes)");
  return NMX_OK;
}

}  // namespace

extern "C" size_t nmx_pe_wide_workspace_bytes(int dim, int num_chains) {
  const int ldc = (num_chains + 63) / 64 * 64;
  return (size_t)num_slices(dim) * NSUM * ldc * sizeof(float);
}

extern "C" int nmx_pe_stochastic_volatility(const float* returns, int T, const nmx_eval_batch* ev, void* workspace,
                                            void* stream) {
  if (int st = check_ev(ev, workspace)) return st;
  if (!returns || T <= 1) return nmx_fail(NMX_ERR_INVALID, "stochastic_volatility: need T > 1 returns");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const int G = groups_of(ev);
  hipLaunchKernelGGL(k_sv_part, dim3(G, num_slices(T)), dim3(64 * WAVES), 0, s, returns, T, *ev, part);
  hipLaunchKernelGGL(k_sv_fin, dim3(G), dim3(64 * WAVES), 0, s, T, *ev, part);
  return nmx_check_launch("k_sv");
}

extern "C" int nmx_pe_funnel(int dim, const nmx_eval_batch* ev, void* workspace, void* stream) {
  if (int st = check_ev(ev, workspace)) return st;
  if (dim < 2) return nmx_fail(NMX_ERR_INVALID, "funnel: dim must be >= 2");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const int G = groups_of(ev);
  hipLaunchKernelGGL(k_funnel_part, dim3(G, num_slices(dim - 1)), dim3(64 * WAVES), 0, s, dim, *ev, part);
  hipLaunchKernelGGL(k_funnel_fin, dim3(G), dim3(64 * WAVES), 0, s, dim, *ev, part);
  return nmx_check_launch("k_funnel");
}

extern "C" int nmx_pe_funnel_noncentered(int dim, const nmx_eval_batch* ev, void* workspace, void* stream) {
  if (int st = check_ev(ev, workspace)) return st;
  if (dim < 2) return nmx_fail(NMX_ERR_INVALID, "funnel_noncentered: dim must be >= 2");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const int G = groups_of(ev);
  hipLaunchKernelGGL(k_funnel_nc_part, dim3(G, num_slices(dim - 1)), dim3(64 * WAVES), 0, s, dim, *ev, part);
  hipLaunchKernelGGL(k_funnel_nc_fin, dim3(G), dim3(64 * WAVES), 0, s, dim, *ev, part);
  return nmx_check_launch("k_funnel_nc");
}
