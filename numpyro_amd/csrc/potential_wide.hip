// Potentials of wide-latent models whose cost is O(D) per chain: stochastic volatility
// (examples/stochastic_volatility.py:57-65, D = T + 2) and the centred / non-centred funnel
// (examples/funnel.py:44-49, D = dim).  Both are HBM-bound.  The grid is chain groups x
// row slices (so any C fills the GPU): a block owns 64 chains x one slice of 64 rows
// (256-byte coalesced rows of the chain-major layout), writes the row gradients and
// per-slice partial sums; a finalize kernel sums the slices in a fixed order and writes U
// and the gradients of the scalar sites.  The per-row and finalize arithmetic is the
// model's (nmx_wide_models.h), shared with the fused leaf kernel of the wide NUTS step.
#include <math.h>

#include <algorithm>

#include "nmx_api_internal.h"
#include "nmx_common.h"
#include "nmx_wide_models.h"

namespace {

// D-split: block = 64 list positions x WAVES waves over one slice of SLICE rows; per-slice
// partial sums go to a workspace [NS][NSUM][ldc] and a finalize kernel adds the slices in a
// fixed order.  The slicing depends on D only, so a chain's U and dU do not depend on how
// many chains share a launch.
constexpr int WAVES = 4;
constexpr int SLICE = 64;
constexpr int NSUM_MAX = 4;

__host__ __device__ inline int num_slices(int rows) { return (rows + SLICE - 1) / SLICE; }

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

// rows lo + [blockIdx.y * SLICE, +SLICE) of the model's per-coordinate rows
template <class M>
__global__ __launch_bounds__(64 * WAVES) void k_wide_part(M m, nmx_eval_batch ev, float* __restrict__ part) {
  constexpr int NS = M::NSUM;
  __shared__ float lds[NS * WAVES * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + lane);
  const bool act = c >= 0;
  if (!__syncthreads_or(act)) return;
  const int ldc = ev.ldc;
  float sums[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) sums[i] = 0.0f;
  const int r0 = m.lo() + blockIdx.y * SLICE, r1 = min(m.hi(), r0 + SLICE);
  if (act) {
    const typename M::Glob g = m.globals(ev.z, ldc, c);
    for (int d = r0 + wv; d < r1; d += WAVES) {
      const uint32_t off = nmx_row_off(d, ldc, c);
      nmx_at(ev.grad, off) = m.row(ev.z, off, (uint32_t)ldc << 2, d, g, sums);
    }
  }
  wave_block_sum<NS>(sums, lds);
  if (act && wv == 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) part[((size_t)blockIdx.y * NS + i) * ldc + c] = sums[i];
  }
}

// Slice sums in a fixed order: wave w adds slices w, w+WAVES, ..., then the waves in order.
template <class M>
__global__ __launch_bounds__(64 * WAVES) void k_wide_fin(M m, nmx_eval_batch ev, const float* __restrict__ part) {
  constexpr int NS = M::NSUM;
  __shared__ float lds[NS * WAVES * 64];
  const int wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + (threadIdx.x & 63));
  if (!__syncthreads_or(c >= 0)) return;
  const int ldc = ev.ldc;
  const int ns = num_slices(m.hi() - m.lo());
  float v[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) v[i] = 0.0f;
  if (c >= 0)
    for (int sl = wv; sl < ns; sl += WAVES)
#pragma unroll
      for (int i = 0; i < NS; ++i) v[i] += part[((size_t)sl * NS + i) * ldc + c];
  wave_block_sum<NS>(v, lds);
  if (wv != 0 || c < 0) return;
  const typename M::Glob g = m.globals(ev.z, ldc, c);
  float gs[M::NSCALAR];
  ev.pe[c] = m.fin(v, g, gs);
#pragma unroll
  for (int i = 0; i < M::NSCALAR; ++i) ev.grad[(size_t)m.scalar_row(i) * ldc + c] = gs[i];
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

template <class M>
int launch(const M& m, const nmx_eval_batch* ev, void* workspace, void* stream, const char* what) {
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const int G = groups_of(ev);
  hipLaunchKernelGGL(k_wide_part<M>, dim3(G, num_slices(m.hi() - m.lo())), dim3(64 * WAVES), 0, s, m, *ev, part);
  hipLaunchKernelGGL(k_wide_fin<M>, dim3(G), dim3(64 * WAVES), 0, s, m, *ev, part);
  return nmx_check_launch(what);
}

}  // namespace

extern "C" size_t nmx_pe_wide_workspace_bytes(int dim, int num_chains) {
  const int ldc = (num_chains + 63) / 64 * 64;
  return (size_t)num_slices(dim) * NSUM_MAX * ldc * sizeof(float);
}

extern "C" int nmx_pe_stochastic_volatility(const float* returns, int T, const nmx_eval_batch* ev, void* workspace,
                                            void* stream) {
  if (int st = check_ev(ev, workspace)) return st;
  if (!returns || T <= 1) return nmx_fail(NMX_ERR_INVALID, "stochastic_volatility: need T > 1 returns");
  return launch(NmxWideSV{returns, T}, ev, workspace, stream, "k_sv");
}

extern "C" int nmx_pe_funnel(int dim, const nmx_eval_batch* ev, void* workspace, void* stream) {
  if (int st = check_ev(ev, workspace)) return st;
  if (dim < 2) return nmx_fail(NMX_ERR_INVALID, "funnel: dim must be >= 2");
  return launch(NmxWideFunnel{dim}, ev, workspace, stream, "k_funnel");
}

extern "C" int nmx_pe_funnel_noncentered(int dim, const nmx_eval_batch* ev, void* workspace, void* stream) {
  if (int st = check_ev(ev, workspace)) return st;
  if (dim < 2) return nmx_fail(NMX_ERR_INVALID, "funnel_noncentered: dim must be >= 2");
  return launch(NmxWideFunnelNC{dim}, ev, workspace, stream, "k_funnel_nc");
}
