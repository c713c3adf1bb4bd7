// Chain-batched dense transforms on f32 MFMA: Out[:, c] = A . In[:, c] (+ bias) for every
// 64-chain tile that holds an evaluated chain.  Used by the dense-mass path: with
// M^-1 = T T^T the reference's dense-mass NUTS (hmc_util.py:1203-1220 matvecs, hmc.py:103-108
// momentum) is identity-mass NUTS on w with z = mu + T w, so each leapfrog costs the two
// products z = T w and g_w = T^T g_z (4 D^2 FLOP per chain).
//
// The kernel takes At = A^T (row-major, padded to Dp x Dp with zeros, Dp = round_up(D, 128))
// so that both LDS tiles are filled by coalesced row reads: As[k][i] = At[k][i] (by
// global_load_lds) and Bs[k][c] = In[k][c] (register staged, rows >= D masked to zero).
// Wave w computes rows [32w, 32w+32) x 64 chains with two 32x32 accumulators of
// v_mfma_f32_32x32x2_f32; A operand lane l = As[2s + (l>>5)][32w + (l&31)], B operand
// = Bs[2s + (l>>5)][(l&31) + 32b] -- both bank-conflict free without padding.
#include <stdlib.h>

#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TM = 128;  // output rows per workgroup
constexpr int TN = 64;   // chains per workgroup
constexpr int BK = 32;   // k per stage

__global__ __launch_bounds__(256, 2) void k_gemm_chains(const float* __restrict__ At, int lda, int D,
                                                        const float* __restrict__ In, float* __restrict__ Out,
                                                        const float* __restrict__ bias, int triangle, int ldc,
                                                        const int32_t* __restrict__ phase,
                                                        const int32_t* __restrict__ count, int C,
                                                        float* __restrict__ part, int ksplit, int order,
                                                        int n_rt, int n_ct) {
  __shared__ __attribute__((aligned(16))) float As[2][BK * TM];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * TN];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l31 = lane & 31;
  int rt_i = blockIdx.x, ct_i = blockIdx.y;
  if (order) {
    // XCD-aware: blocks b, b+8, ... (one XCD) sweep the chain tiles of one row tile, so the
    // A stages they share stay in that XCD's L2
    const int b = blockIdx.x, xcd = b & 7, q = b >> 3;
    rt_i = (q / n_ct) * 8 + xcd;
    ct_i = q % n_ct;
    if (rt_i >= n_rt) return;
  }
  const int i0 = rt_i * TM;
  const int c0 = ct_i * TN;
  // tile has an evaluated chain?  (packed columns: the first *count positions)
  if (count) {
    if (c0 >= *count) return;
  } else {
    const int c = c0 + lane;
    const bool act = c < C && (phase == nullptr || phase[c] >= NMX_PH_LEAF);
    if (!__any(act)) return;  // same result in every wave
  }
  // A upper triangular (triangle 1): out rows [i0, i0+TM) need k >= i0 only; A lower
  // triangular (2): k < i0 + TM only.  Skipped K-tiles are exact zeros.
  const int kt_lo = triangle == 1 ? i0 / BK : 0;
  const int kt_hi = triangle == 2 ? min((D + BK - 1) / BK, (i0 + TM + BK - 1) / BK) : (D + BK - 1) / BK;
  // split-K: block z takes an even share of this row tile's K-tiles (boundaries depend on
  // D and the row tile only); partials are summed in a fixed order by k_gemm_reduce
  const int z = blockIdx.z;
  const int kt_begin = kt_lo + (int)((int64_t)(kt_hi - kt_lo) * z / ksplit);
  const int nk = kt_lo + (int)((int64_t)(kt_hi - kt_lo) * (z + 1) / ksplit);

  auto load_a = [&](int kt, int buf) {
    // BK rows x TM floats = 16 KiB = 16 wave-instructions of 1 KiB; 4 per wave
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int inst = w * 4 + q;             // 0..15
      const int row = inst * 2 + (lane >> 5); // two 512-byte rows per instruction
      const int col = (lane & 31) * 4;
      const float* src = At + (size_t)(kt * BK + row) * lda + i0 + col;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)(&As[buf][inst * 256]), 16, 0, 0);
    }
  };
  auto load_b = [&](int kt, float4 (&reg)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = (q * 256 + tid);  // float4 index in the 32 x 64 tile
      const int row = e >> 4;         // 16 float4 per row
      const int col = (e & 15) * 4;
      const int k = kt * BK + row;
      const int c = c0 + col;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < D && c < ldc) v = *reinterpret_cast<const float4*>(In + (size_t)k * ldc + c);
      reg[q] = v;
    }
  };
  auto store_b = [&](int buf, const float4 (&reg)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) reinterpret_cast<float4*>(Bs[buf])[q * 256 + tid] = reg[q];
  };

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.0f;
    acc1[r] = 0.0f;
  }
  float4 breg[2];
  if (kt_begin < nk) {
    load_a(kt_begin, 0);
    load_b(kt_begin, breg);
    store_b(0, breg);
  }
  __syncthreads();
  for (int kt = kt_begin; kt < nk; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_a(kt + 1, buf ^ 1);
      load_b(kt + 1, breg);
    }
    const float* as = As[buf];
    const float* bs = Bs[buf];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      const float a = as[k * TM + w * 32 + l31];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bs[k * TN + l31], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bs[k * TN + 32 + l31], acc1, 0, 0, 0);
    }
    if (more) store_b(buf ^ 1, breg);
    __syncthreads();
  }
  float* const dst = ksplit > 1 ? part + (size_t)z * D * ldc : Out;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = i0 + w * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (i < D) {
      const float bi = (bias && ksplit == 1) ? bias[i] : 0.0f;
      const int ca = c0 + l31, cb = c0 + 32 + l31;
      if (ca < ldc) dst[(size_t)i * ldc + ca] = acc0[r] + bi;
      if (cb < ldc) dst[(size_t)i * ldc + cb] = acc1[r] + bi;
    }
  }
}

// Same products, tiles and MFMA order as k_gemm_chains (bitwise equal results), with both
// operand tiles staged by buffer LDS-DMA through scalar descriptors (no register staging of
// B: fewer VGPRs, no VALU copies), BK-deep double-buffered stages in dynamic LDS, and one
// barrier per stage.  B rows >= D come back as zeros from the descriptor's range check
// (every B offset is in voffset, which the check covers).
template <int BKV>
__global__ __launch_bounds__(256, 2) void k_gemm_chains2(const float* __restrict__ At, int lda, int D,
                                                         const float* __restrict__ In, float* __restrict__ Out,
                                                         const float* __restrict__ bias, int triangle, int ldc,
                                                         const int32_t* __restrict__ phase,
                                                         const int32_t* __restrict__ count, int C,
                                                         float* __restrict__ part, int ksplit, int order, int n_rt,
                                                         int n_ct) {
  constexpr int A_PIECES = BKV * TM / 256;  // 1 KB pieces (2 rows of 128 floats)
  constexpr int B_PIECES = BKV * TN / 256;  // 1 KB pieces (4 rows of 64 floats)
  constexpr int STAGE = BKV * (TM + TN);    // floats per stage
  constexpr int PER_WAVE = (A_PIECES + B_PIECES) / 4;
  static_assert((A_PIECES + B_PIECES) % 4 == 0, "pieces split evenly over 4 waves");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int rt_i = blockIdx.x, ct_i = blockIdx.y;
  if (order) {
    const int b = blockIdx.x, xcd = b & 7, q = b >> 3;
    rt_i = (q / n_ct) * 8 + xcd;
    ct_i = q % n_ct;
    if (rt_i >= n_rt) return;
  }
  const int i0 = rt_i * TM;
  const int c0 = ct_i * TN;
  if (count) {
    if (c0 >= *count) return;
  } else {
    const int c = c0 + lane;
    const bool act = c < C && (phase == nullptr || phase[c] >= NMX_PH_LEAF);
    if (!__any(act)) return;
  }
  // K range and split-K boundaries in units of BK = 32 (those of k_gemm_chains), then in
  // BKV-tiles: every variant adds the same products in the same order
  constexpr int R = BK / BKV;
  static_assert(BK % BKV == 0, "BKV divides BK");
  const int kt_lo = triangle == 1 ? i0 / BK : 0;
  const int kt_hi = triangle == 2 ? min((D + BK - 1) / BK, (i0 + TM + BK - 1) / BK) : (D + BK - 1) / BK;
  const int z = blockIdx.z;
  const int kt_begin = R * (kt_lo + (int)((int64_t)(kt_hi - kt_lo) * z / ksplit));
  const int nk = R * (kt_lo + (int)((int64_t)(kt_hi - kt_lo) * (z + 1) / ksplit));

  const __amdgpu_buffer_rsrc_t ars =
      __builtin_amdgcn_make_buffer_rsrc((void*)At, 0, (int)min((int64_t)lda * lda * 4, (int64_t)0x7fffffff),
                                        0x00020000);
  const __amdgpu_buffer_rsrc_t brs =
      __builtin_amdgcn_make_buffer_rsrc((void*)In, 0, (int)min((int64_t)D * ldc * 4, (int64_t)0x7fffffff),
                                        0x00020000);
  const unsigned a_lane = (unsigned)(((lane >> 5) * lda + (lane & 31) * 4) * 4);
  const unsigned b_lane = (unsigned)(((lane >> 4) * ldc + (lane & 15) * 4) * 4);
  auto issue = [&](int kt, int buf) {
    float* st = lds + buf * STAGE;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) {
      const int p = wu * PER_WAVE + j;  // wave-uniform piece index
      if (p < A_PIECES) {
        const unsigned so = (unsigned)(((size_t)(kt * BKV + 2 * p) * lda + i0) * 4);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (__attribute__((address_space(3))) void*)(st + p * 256), 16,
                                                 a_lane, so, 0, 0);
      } else {
        const int pb = p - A_PIECES;
        const unsigned vo = b_lane + (unsigned)(((size_t)(kt * BKV + 4 * pb) * ldc + c0) * 4);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            brs, (__attribute__((address_space(3))) void*)(st + BKV * TM + pb * 256), 16, vo, 0, 0, 0);
      }
    }
  };

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.0f;
    acc1[r] = 0.0f;
  }
  if (kt_begin < nk) issue(kt_begin, 0);
  for (int kt = kt_begin; kt < nk; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage kt landed for every wave; every wave is done with stage kt-1
    if (kt + 1 < nk) issue(kt + 1, buf ^ 1);
    const float* as = lds + buf * STAGE;
    const float* bs = as + BKV * TM;
#pragma unroll
    for (int s = 0; s < BKV / 2; ++s) {
      const int k = 2 * s + h;
      const float a = as[k * TM + w * 32 + l31];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bs[k * TN + l31], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bs[k * TN + 32 + l31], acc1, 0, 0, 0);
    }
  }
  float* const dst = ksplit > 1 ? part + (size_t)z * D * ldc : Out;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = i0 + w * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (i < D) {
      const float bi = (bias && ksplit == 1) ? bias[i] : 0.0f;
      const int ca = c0 + l31, cb = c0 + 32 + l31;
      if (ca < ldc) dst[(size_t)i * ldc + ca] = acc0[r] + bi;
      if (cb < ldc) dst[(size_t)i * ldc + cb] = acc1[r] + bi;
    }
  }
}

// Out = sum_z part[z] (+ bias), z in order; same tile selection as k_gemm_chains.
__global__ __launch_bounds__(256) void k_gemm_reduce(const float* __restrict__ part, int ksplit, int D, int ldc,
                                                     float* __restrict__ Out, const float* __restrict__ bias,
                                                     const int32_t* __restrict__ phase,
                                                     const int32_t* __restrict__ count, int C) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = blockIdx.y * TN;
  const int c = c0 + lane;
  if (count) {
    if (c0 >= *count) return;
  } else {
    const bool act = c < C && (phase == nullptr || phase[c] >= NMX_PH_LEAF);
    if (!__any(act)) return;
  }
  const int d0 = blockIdx.x * 16;
  for (int i = d0 + w; i < min(D, d0 + 16); i += 4) {
    float s = 0.0f;
    for (int zz = 0; zz < ksplit; ++zz) s += part[((size_t)zz * D + i) * ldc + c];
    Out[(size_t)i * ldc + c] = s + (bias ? bias[i] : 0.0f);
  }
}

// pe[c] = 0.5 sum_d (z[d][c] - mu[d]) * g[d][c] for evaluated chains; 4 waves split d,
// partials combined in fixed order.
__global__ __launch_bounds__(256) void k_quad_pe(const float* __restrict__ mu, int D, nmx_eval_batch ev) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, blockIdx.x * 64 + lane);
  float s = 0.0f;
  if (c >= 0) {
    for (int d = w; d < D; d += 4) {
      const size_t idx = (size_t)d * ev.ldc + c;
      s += (ev.z[idx] - mu[d]) * ev.grad[idx];
    }
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && c >= 0) ev.pe[c] = 0.5f * (((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]);
}

// Column compaction for the dense products: packed[d][p] = in[d][list[p]] for p < *count.
constexpr int PACK_ROWS = 16;
__global__ __launch_bounds__(256) void k_pack(const float* __restrict__ in, int ldi, int D,
                                              const int32_t* __restrict__ list, const int32_t* __restrict__ count,
                                              float* __restrict__ out, int ldo) {
  const int p = blockIdx.y * 64 + (threadIdx.x & 63);
  if (blockIdx.y * 64 >= *count) return;
  if (p >= *count) return;
  const int c = list[p];
  const int d0 = blockIdx.x * PACK_ROWS;
  for (int d = d0 + (threadIdx.x >> 6); d < min(D, d0 + PACK_ROWS); d += 4)
    out[(size_t)d * ldo + p] = in[(size_t)d * ldi + c];
}

// Scatter back: out[d][list[p]] = packed[d][p]; pe_out[list[p]] = pe_packed[p].
__global__ __launch_bounds__(256) void k_unpack(const float* __restrict__ in, int ldi, int D,
                                                const int32_t* __restrict__ list, const int32_t* __restrict__ count,
                                                float* __restrict__ out, int ldo, const float* __restrict__ pe_in,
                                                float* __restrict__ pe_out) {
  const int p = blockIdx.y * 64 + (threadIdx.x & 63);
  if (blockIdx.y * 64 >= *count) return;
  if (p >= *count) return;
  const int c = list[p];
  const int d0 = blockIdx.x * PACK_ROWS;
  for (int d = d0 + (threadIdx.x >> 6); d < min(D, d0 + PACK_ROWS); d += 4)
    out[(size_t)d * ldo + c] = in[(size_t)d * ldi + p];
  if (pe_in && blockIdx.x == 0 && threadIdx.x < 64) pe_out[c] = pe_in[p];
}

// The same for a chain-row arena ([ldc][D] rows, nmx_nuts_config.layout = CHAIN_ROWS): a
// 64 x 64 transpose through LDS per block, coalesced on both sides.
constexpr int TR_TILE = 64;
__global__ __launch_bounds__(256) void k_pack_rows(const float* __restrict__ in, int D,
                                                   const int32_t* __restrict__ list, const int32_t* __restrict__ count,
                                                   float* __restrict__ out, int ldo) {
  __shared__ float t[TR_TILE][TR_TILE + 1];
  const int n = *count;
  const int p0 = blockIdx.y * TR_TILE, d0 = blockIdx.x * TR_TILE;
  if (p0 >= n) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < TR_TILE; i += 4) {  // row (chain) p0 + i, coordinates d0 + lane
    const int p = p0 + i, d = d0 + lane;
    if (p < n && d < D) t[i][lane] = in[(size_t)list[p] * D + d];
  }
  __syncthreads();
  for (int i = w; i < TR_TILE; i += 4) {  // coordinate d0 + i, positions p0 + lane
    const int p = p0 + lane, d = d0 + i;
    if (p < n && d < D) out[(size_t)d * ldo + p] = t[lane][i];
  }
}

__global__ __launch_bounds__(256) void k_unpack_rows(const float* __restrict__ in, int ldi, int D,
                                                     const int32_t* __restrict__ list,
                                                     const int32_t* __restrict__ count, float* __restrict__ out,
                                                     const float* __restrict__ pe_in, float* __restrict__ pe_out) {
  __shared__ float t[TR_TILE][TR_TILE + 1];
  const int n = *count;
  const int p0 = blockIdx.y * TR_TILE, d0 = blockIdx.x * TR_TILE;
  if (p0 >= n) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < TR_TILE; i += 4) {  // coordinate d0 + i, positions p0 + lane
    const int p = p0 + lane, d = d0 + i;
    if (p < n && d < D) t[lane][i] = in[(size_t)d * ldi + p];
  }
  __syncthreads();
  for (int i = w; i < TR_TILE; i += 4) {  // chain list[p0 + i], coordinates d0 + lane
    const int p = p0 + i, d = d0 + lane;
    if (p < n && d < D) out[(size_t)list[p] * D + d] = t[i][lane];
  }
  if (pe_in && blockIdx.x == 0 && threadIdx.x < 64 && p0 + lane < n) pe_out[list[p0 + lane]] = pe_in[p0 + lane];
}

// ---------------------------------------------------------------------------------------
// Split-bf16 chain products (f32-accurate on the bf16 matrix cores; the scheme of the covtype
// kernel, potential_logreg.hip "Split-bf16 kernel"): every f32 operand as three bf16 terms,
// six bf16 products per 16-deep k-step into f32 accumulators: a1b1 into the main accumulator,
// the five correction products (a3b1 + a2b2 + a1b3 + a2b1 + a1b2, ~2^-8 of it) into a second
// one, the two added once after the k loop.  One rounding of the main sum per k-step instead
// of six: at D = 5038 the products' largest error fell from 4x to ~1x a float32 GEMM's
// (scripts/bnn_accuracy.py), which is what the BNN parity leg's draw drift was made of.  A (= T or T^T, constant between adaptation windows) is packed once into
// MFMA-fragment order (nmx_gemm_x3_pack_a); each call splits In into fragment order first
// (k_x3_split_b, ~6 B written per f32 read), then k_gemm_x3 streams both through a 2-slot
// LDS ring by buffer LDS-DMA.  Tiles, triangle skipping, split-K boundaries, the XCD-aware
// order and the fixed-order reduction are those of k_gemm_chains; a column's result depends
// only on its own data (packed == dense-batch bitwise).
//   Ap piece ((ks * n_it + it) * 3 + p): lane (r, h) = A[32 it + r][16 ks + 8 h + j], plane p
//   Bp piece ((ks * n_ct + ct) * 3 + p): lane (r, h) = In[16 ks + 8 h + j][32 ct + r], plane p
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& b1, bf16x8& b2, bf16x8& b3) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h1 = (__bf16)v[j];
    const float e1 = v[j] - (float)h1;
    const __bf16 h2 = (__bf16)e1;
    const float e2 = e1 - (float)h2;
    b1[j] = h1;
    b2[j] = h2;
    b3[j] = (__bf16)e2;
  }
}

// one thread per (k-step, row tile, lane): the three planes of one A fragment lane
__global__ __launch_bounds__(256) void k_x3_pack_a(const float* __restrict__ At, int lda, bf16x8* __restrict__ Ap) {
  const int n_it = lda / 32, n_ks = lda / 16;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n_ks * n_it * 64) return;
  const int lane = (int)(i & 63);
  const int64_t q = i >> 6;
  const int it = (int)(q % n_it), ks = (int)(q / n_it);
  const int r = lane & 31, h = lane >> 5;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = At[(size_t)(16 * ks + 8 * h + j) * lda + 32 * it + r];
  bf16x8 b1, b2, b3;
  split3(v, b1, b2, b3);
  const size_t base = (size_t)q * 3 * 64 + lane;
  Ap[base] = b1;
  Ap[base + 64] = b2;
  Ap[base + 128] = b3;
}

// one thread per (k-step, chain tile, lane); rows >= D read as zero
__global__ __launch_bounds__(256) void k_x3_split_b(const float* __restrict__ In, int D, int ldc, int n_ks,
                                                    const int32_t* __restrict__ count, bf16x8* __restrict__ Bp) {
  const int n_ct = ldc / 32;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n_ks * n_ct * 64) return;
  const int lane = (int)(i & 63);
  const int64_t q = i >> 6;
  const int ct = (int)(q % n_ct), ks = (int)(q / n_ct);
  if (count && ct * 32 >= *count) return;  // packed columns: tiles past the count are never read
  const int r = lane & 31, h = lane >> 5;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * ks + 8 * h + j;
    v[j] = k < D ? In[(size_t)k * ldc + 32 * ct + r] : 0.0f;
  }
  bf16x8 b1, b2, b3;
  split3(v, b1, b2, b3);
  const size_t base = (size_t)q * 3 * 64 + lane;
  Bp[base] = b1;
  Bp[base + 64] = b2;
  Bp[base + 128] = b3;
}

// The same split with the operand gathered from a chain-row arena: column p of In is the row of
// chain list[p] (rows[list[p]][k], [ldc][D] rows, NMX_LAYOUT_CHAIN_ROWS) -- nmx_pack_rows and
// k_x3_split_b in one pass.  Each lane reads 8 consecutive floats of its chain's row (two
// 16-byte loads when D % 8 == 0); the k-steps run fastest over the grid, so one workgroup's
// four waves read 256 contiguous bytes of each of 32 rows (the split image is laid out chain
// tile fastest: each wave still writes 3 KB contiguous).  Positions >= *count split as zeros
// (their product columns are never read).
__global__ __launch_bounds__(256) void k_x3_split_b_rows(const float* __restrict__ rows, int D,
                                                         const int32_t* __restrict__ list, int ldc, int n_ks,
                                                         const int32_t* __restrict__ count, bf16x8* __restrict__ Bp) {
  const int n_ct = ldc / 32;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n_ks * n_ct * 64) return;
  const int lane = (int)(i & 63);
  const int64_t qg = i >> 6;
  const int ks = (int)(qg % n_ks), ct = (int)(qg / n_ks);
  const int n = *count;
  if (ct * 32 >= n) return;
  const int r = lane & 31, h = lane >> 5;
  const int p = 32 * ct + r;
  const int k0 = 16 * ks + 8 * h;
  float v[8];
  if (p < n && (D & 7) == 0) {
    const float4* src = reinterpret_cast<const float4*>(rows + (size_t)list[p] * D + k0);
    const float4 a = k0 < D ? src[0] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = k0 < D ? src[1] : make_float4(0.f, 0.f, 0.f, 0.f);
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
  } else {
    const float* row = p < n ? rows + (size_t)list[p] * D : nullptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (row && k0 + j < D) ? row[k0 + j] : 0.0f;
  }
  bf16x8 b1, b2, b3;
  split3(v, b1, b2, b3);
  const size_t base = ((size_t)ks * n_ct + ct) * 3 * 64 + lane;
  Bp[base] = b1;
  Bp[base + 64] = b2;
  Bp[base + 128] = b3;
}

// chain tiles of 32 per workgroup (2: 128 x 64 outputs per workgroup, two per CU; 4: 128 x 128,
// one per CU, 1.5x the MFMA work per staged byte)
#ifndef NMX_GEMM_CT
#define NMX_GEMM_CT 2
#endif
// row tiles of 32 per workgroup = its waves (4: 128 rows; 8: 256 rows, 512 threads)
#ifndef NMX_GEMM_RW
#define NMX_GEMM_RW 4
#endif
// 1: the 256 x 128 tile for launches it fills (nmx_gemm_chains_x3); 0: always RW x CT (A/B)
#ifndef NMX_GEMM_BIG_MIN
#define NMX_GEMM_BIG_MIN 512  // big-tile workgroups a launch must have to take the 256 x 128 tile
#endif
#ifndef NMX_GEMM_BIG
#define NMX_GEMM_BIG 1
#endif
// LDS ring depth in stages (3 with CT = 4: 144 KB, one stage more in flight for the lone
// workgroup of a CU)
#ifndef NMX_GEMM_NBUF
#define NMX_GEMM_NBUF 2
#endif
template <int N>
__device__ __forceinline__ void gemm_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
template <int CT, int RW = 4>
constexpr int x3_pieces() { return 2 * (RW * 3 + CT * 3); }  // per 32-deep stage: A 2 x 3 RW, B 2 x 3 CT pieces of 1 KB
constexpr int X3_PIECES = x3_pieces<2>();

constexpr int X3_BLK = 8;  // stages (of 32 k) per block sum in k_gemm_x3

template <int CT, int NBUF, int RW>
__global__ __launch_bounds__(64 * RW, (RW == 4 && CT == 2) ? 2 : 1) void k_gemm_x3(const char* __restrict__ Ap, int lda, int D,
                                                    const char* __restrict__ Bp, float* __restrict__ Out,
                                                    const float* __restrict__ bias, int triangle, int ldc,
                                                    const int32_t* __restrict__ phase,
                                                    const int32_t* __restrict__ count, int C,
                                                    float* __restrict__ part, int ksplit, int order, int n_rt,
                                                    int n_ct, const int32_t* __restrict__ out_list,
                                                    const float* __restrict__ pe_in, float* __restrict__ pe_out) {
  extern __shared__ __attribute__((aligned(16))) float lds_f[];  // (the TU's one dynamic-LDS symbol)
  char* const lds = reinterpret_cast<char*>(lds_f);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int rt_i = blockIdx.x, ct_i = blockIdx.y;
  if (order) {
    const int b = blockIdx.x, xcd = b & 7, q = b >> 3;
    // XCD xcd takes row tiles j = 0, 1, ... of the 8-wide row-tile rows, zigzagging (8j + xcd
    // for even j, 8j + 7 - xcd for odd j) so that every XCD's sum of triangular K lengths is
    // the same, and the longest-K row tiles first (j reversed for the lower triangle) so the
    // short ones fill the end: 3-17% faster triangular products than 8j + xcd
    int j = q / n_ct;
    if (triangle == 2) j = (n_rt + 7) / 8 - 1 - j;
    rt_i = j * 8 + ((j & 1) ? 7 - xcd : xcd);
    ct_i = q % n_ct;
    if (rt_i >= n_rt) return;
  }
  constexpr int TNC = 32 * CT;  // chains per workgroup
  constexpr int TMW = 32 * RW;  // rows per workgroup
  constexpr int NPC = x3_pieces<CT, RW>();
  constexpr int NPA = 6 * RW;   // A pieces per stage
  const int i0 = rt_i * TMW;
  const int c0 = ct_i * TNC;
  // 64-chain tiles with work (an inactive tile's outputs stay untouched)
  bool act64[TNC / 64];
  bool any_act = false;
#pragma unroll
  for (int q = 0; q < TNC / 64; ++q) {
    if (count) {
      act64[q] = c0 + 64 * q < *count;
    } else {
      const int c = c0 + 64 * q + lane;
      act64[q] = __any(c < C && (phase == nullptr || phase[c] >= NMX_PH_LEAF));
    }
    any_act |= act64[q];
  }
  if (!any_act) return;
  const int kt_lo = triangle == 1 ? i0 / BK : 0;
  const int kt_hi = triangle == 2 ? min((D + BK - 1) / BK, (i0 + TMW + BK - 1) / BK) : (D + BK - 1) / BK;
  const int z = blockIdx.z;
  const int kt_begin = kt_lo + (int)((int64_t)(kt_hi - kt_lo) * z / ksplit);
  const int nk = kt_lo + (int)((int64_t)(kt_hi - kt_lo) * (z + 1) / ksplit);

  const int n_it = lda / 32, n_ct32 = ldc / 32;
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Ap, 0, (int)min((int64_t)lda * lda * 6, (int64_t)0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Bp, 0, (int)min((int64_t)(lda / 16) * ldc * 16 * 6, (int64_t)0x7fffffff), 0x00020000);
  // stage kt (k-steps 2 kt, 2 kt + 1): pieces [s][3 RW A: row tile x plane] then [s][3 CT B:
  // chain tile x plane]; wave wu DMAs pieces PW wu .. PW wu + PW - 1, each at base + kt * stride
  static_assert(NPC % RW == 0, "pieces per wave");
  constexpr int PW = NPC / RW;
  unsigned pbase[PW], pstride[PW];
#pragma unroll
  for (int jj = 0; jj < PW; ++jj) {
    const int pc = wu * PW + jj;
    if (pc < NPA) {
      const int sb = pc / (3 * RW), e = pc % (3 * RW);
      pbase[jj] = (unsigned)(((sb * n_it + RW * rt_i) * 3 + e) * 1024);
      pstride[jj] = (unsigned)(2 * n_it * 3 * 1024);
    } else {
      const int sb = (pc - NPA) / (3 * CT), e = (pc - NPA) % (3 * CT);
      pbase[jj] = (unsigned)(((sb * n_ct32 + CT * ct_i) * 3 + e) * 1024);
      pstride[jj] = (unsigned)(2 * n_ct32 * 3 * 1024);
    }
  }
  auto issue = [&](int kt, int buf) {
    char* st = lds + buf * NPC * 1024;
#pragma unroll
    for (int jj = 0; jj < PW; ++jj) {
      const int pc = wu * PW + jj;  // wave-uniform
      const unsigned so = pbase[jj] + (unsigned)kt * pstride[jj];
      if (pc < NPA)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (__attribute__((address_space(3))) void*)(st + pc * 1024), 16,
                                                 lane * 16, so, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (__attribute__((address_space(3))) void*)(st + pc * 1024), 16,
                                                 lane * 16, so, 0, 0);
    }
  };

  // v_mfma_f32_16x16x32_bf16 on 16 x 16 sub-tiles: a wave's 32 x 32 output per chain tile is
  // 2 x 2 sub-tiles (m rows, n chains), each stage's 32-deep K in one instruction (the 16x16x32
  // shape holds a higher clock than 32x32x16 at equal cycles per FLOP, MI355X_MICROARCH.md DVFS
  // item 7).  The staged pieces keep the 32 x 16 fragment order of k_x3_pack_a / k_x3_split_b:
  // lane (r16, q) of a sub-tile reads row / chain 16 m + r16, k-group q of the stage, i.e.
  // k-step q >> 1, half q & 1 of the piece: lane index (q & 1) * 32 + 16 m + r16.
  // a1b1 of the current block of X3_BLK stages / the running total of the finished blocks / the
  // five correction products.  The MFMA rounds its running sum into the accumulator every few
  // products (the measured error of one accumulator over K = 5038 was 1.7x a float32 sgemm's,
  // which a model rounding every 8 products reproduces); summing each 256-deep block in a fresh
  // accumulator and the blocks in a second one rounds at the block sum's scale instead: 0.4x
  // sgemm's in that model.  Block boundaries are absolute stage indices (multiples of
  // X3_BLK), so skipped all-zero triangle stages and the tile shape leave the sums unchanged.
  f32x4 acc[CT][2][2], tot[CT][2][2], cor[CT][2][2];
#pragma unroll
  for (int cl = 0; cl < CT; ++cl)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[cl][m][n][r] = tot[cl][m][n][r] = cor[cl][m][n][r] = 0.0f;
  auto flush = [&]() {
#pragma unroll
    for (int cl = 0; cl < CT; ++cl)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            tot[cl][m][n][r] += acc[cl][m][n][r];
            acc[cl][m][n][r] = 0.0f;
          }
  };
  const int r16 = lane & 15, q = lane >> 4;
  const int qs = q >> 1, ql = (q & 1) * 32 + r16;  // k-step and lane index within the piece
  if (kt_begin < nk) issue(kt_begin, 0);
  if (NBUF == 3 && kt_begin + 1 < nk) issue(kt_begin + 1, 1);
  int buf = 0;
  for (int kt = kt_begin; kt < nk; ++kt) {
    if (NBUF == 3 && kt + 1 < nk)
      gemm_wait_vm<PW>();  // stage kt landed, stage kt + 1 may still be in flight
    else
      gemm_wait_vm<0>();
    asm volatile("s_barrier" ::: "memory");  // stage kt landed in every wave; stage kt-1 consumed
    if (NBUF == 2) {
      if (kt + 1 < nk) issue(kt + 1, buf ^ 1);
    } else {
      if (kt + 2 < nk) issue(kt + 2, buf == 0 ? 2 : buf - 1);
    }
    const bf16x8* fr = reinterpret_cast<const bf16x8*>(lds + buf * NPC * 1024) + ql;
    bf16x8 a[2][3];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int p = 0; p < 3; ++p) a[m][p] = fr[(qs * 3 * RW + w * 3 + p) * 64 + 16 * m];
#pragma unroll
    for (int cl = 0; cl < CT; ++cl) {
      bf16x8 b[2][3];
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int p = 0; p < 3; ++p) b[n][p] = fr[(NPA + qs * 3 * CT + cl * 3 + p) * 64 + 16 * n];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          f32x4& cr = cor[cl][m][n];
          cr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][2], b[n][0], cr, 0, 0, 0);
          cr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][1], b[n][1], cr, 0, 0, 0);
          cr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][0], b[n][2], cr, 0, 0, 0);
          cr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][1], b[n][0], cr, 0, 0, 0);
          cr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][0], b[n][1], cr, 0, 0, 0);
          acc[cl][m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][0], b[n][0], acc[cl][m][n], 0, 0, 0);
        }
    }
    buf = buf + 1 == NBUF ? 0 : buf + 1;
    if ((kt + 1) % X3_BLK == 0) flush();
  }
  flush();
#pragma unroll
  for (int cl = 0; cl < CT; ++cl)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[cl][m][n][r] = tot[cl][m][n][r] + cor[cl][m][n][r];
  // lane (c16, q) of sub-tile (m, n) holds rows 16 m + 4 q + j (j = 0..3) of chain 16 n + c16
  if (out_list) {
    // scattered to the listed chains' rows (Out [.][D], NMX_LAYOUT_CHAIN_ROWS; one K-split): 4
    // consecutive coordinates per (m, n) -- 16-byte stores when D % 4 == 0
    const int n_cnt = *count;
#pragma unroll
    for (int cl = 0; cl < CT; ++cl)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int cc = c0 + 32 * cl + 16 * n + r16;
        if (cc >= n_cnt) continue;
        float* const row = Out + (size_t)out_list[cc] * D;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int i = i0 + w * 32 + 16 * m + 4 * q;
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = acc[cl][m][n][j] + ((bias && i + j < D) ? bias[i + j] : 0.0f);
          if ((D & 3) == 0) {
            if (i < D) *reinterpret_cast<float4*>(row + i) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (i + j < D) row[i + j] = v[j];
          }
        }
        if (pe_in && rt_i == 0 && w == 0 && q == 0) pe_out[out_list[cc]] = pe_in[cc];
      }
    return;
  }
  float* const dst = ksplit > 1 ? part + (size_t)z * D * ldc : Out;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + w * 32 + 16 * m + 4 * q + j;
      if (i < D) {
        const float bi = (bias && ksplit == 1) ? bias[i] : 0.0f;
#pragma unroll
        for (int cl = 0; cl < CT; ++cl)
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const int cc = c0 + 32 * cl + 16 * n + r16;
            if (act64[cl / 2] && cc < ldc) dst[(size_t)i * ldc + cc] = acc[cl][m][n][j] + bi;
          }
      }
    }
}

}  // namespace

extern "C" int nmx_pack_columns(const float* in, int ldi, int dim, const int32_t* list, const int32_t* count,
                                float* out, int ldo, void* stream) {
  if (!in || !list || !count || !out || dim <= 0 || ldo % 64 || ldi <= 0)
    return nmx_fail(NMX_ERR_INVALID, "pack_columns: bad arguments");
  hipLaunchKernelGGL(k_pack, dim3((dim + PACK_ROWS - 1) / PACK_ROWS, ldo / 64), dim3(256), 0, (hipStream_t)stream,
                     in, ldi, dim, list, count, out, ldo);
  return nmx_check_launch("k_pack");
}

extern "C" int nmx_unpack_columns(const float* in, int ldi, int dim, const int32_t* list, const int32_t* count,
                                  float* out, int ldo, const float* pe_in, float* pe_out, void* stream) {
  if (!in || !list || !count || !out || dim <= 0 || ldi % 64 || ldo <= 0 || (pe_in && !pe_out))
    return nmx_fail(NMX_ERR_INVALID, "unpack_columns: bad arguments");
  hipLaunchKernelGGL(k_unpack, dim3((dim + PACK_ROWS - 1) / PACK_ROWS, ldi / 64), dim3(256), 0,
                     (hipStream_t)stream, in, ldi, dim, list, count, out, ldo, pe_in, pe_out);
  return nmx_check_launch("k_unpack");
}

extern "C" int nmx_pack_rows(const float* in, int ldc, int dim, const int32_t* list, const int32_t* count,
                             float* out, int ldo, void* stream) {
  if (!in || !list || !count || !out || dim <= 0 || ldo % 64 || ldc <= 0)
    return nmx_fail(NMX_ERR_INVALID, "pack_rows: bad arguments");
  hipLaunchKernelGGL(k_pack_rows, dim3((dim + TR_TILE - 1) / TR_TILE, (ldo + TR_TILE - 1) / TR_TILE), dim3(256), 0,
                     (hipStream_t)stream, in, dim, list, count, out, ldo);
  return nmx_check_launch("k_pack_rows");
}

extern "C" int nmx_unpack_rows(const float* in, int ldi, int dim, const int32_t* list, const int32_t* count,
                               float* out, int ldc, const float* pe_in, float* pe_out, void* stream) {
  if (!in || !list || !count || !out || dim <= 0 || ldi % 64 || ldc <= 0 || (pe_in && !pe_out))
    return nmx_fail(NMX_ERR_INVALID, "unpack_rows: bad arguments");
  hipLaunchKernelGGL(k_unpack_rows, dim3((dim + TR_TILE - 1) / TR_TILE, (ldi + TR_TILE - 1) / TR_TILE), dim3(256), 0,
                     (hipStream_t)stream, in, ldi, dim, list, count, out, pe_in, pe_out);
  return nmx_check_launch("k_unpack_rows");
}

extern "C" int nmx_dense_padded_dim(int D) { return (D + TM - 1) / TM * TM; }

// K-splits of the chain products: a function of D only (results never depend on C).
static int ksplit_for(int D) { return D <= 2048 ? 1 : (D + 2559) / 2560; }

extern "C" size_t nmx_gemm_chains_workspace_bytes(int dim, int ldc) {
  const int ks = ksplit_for(dim);
  return ks > 1 ? (size_t)ks * dim * ldc * sizeof(float) : 0;
}

extern "C" int nmx_gemm_chains(const float* At, int lda, int D, const float* In, float* Out, const float* bias,
                               int triangle, int ldc, const int32_t* phase, const int32_t* active_count,
                               int num_chains, void* workspace, void* stream) {
  if (!At || !In || !Out) return nmx_fail(NMX_ERR_INVALID, "gemm_chains: NULL operand");
  if (D <= 0 || ldc % 64 || num_chains <= 0 || num_chains > ldc)
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains: bad sizes (D=%d ldc=%d C=%d)", D, ldc, num_chains);
  if (lda % TM || lda < nmx_dense_padded_dim(D))
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains: lda must be a multiple of %d >= padded D", TM);
  if (In == Out) return nmx_fail(NMX_ERR_INVALID, "gemm_chains: In and Out must not alias");
  if (triangle < 0 || triangle > 2) return nmx_fail(NMX_ERR_INVALID, "gemm_chains: triangle must be 0, 1 or 2");
  // k_gemm_chains2 (LDS-DMA staged); operands past 2 GiB (lda > 23170) take the register-
  // staged k_gemm_chains (64-bit offsets).  Both give bitwise equal products.
  const int ks = workspace ? ksplit_for(D) : 1;
  // block order only permutes blocks (results identical): XCD-aware sweep measured +20-30%
  // on the triangular products at D=5038 (BNN), neutral at D=10000 (profiles/r01)
  const int n_rt = lda / TM, n_ct = ldc / TN;
  const int order = n_rt <= 48 ? 1 : 0;
  dim3 grid = order ? dim3((n_rt + 7) / 8 * 8 * n_ct, 1, ks) : dim3(n_rt, n_ct, ks);
  const bool fits32 = (int64_t)lda * lda * 4 < 0x7fffffff && (int64_t)D * ldc * 4 < 0x7fffffff;
  if (fits32) {
    const size_t lds = 2 * (size_t)BK * (TM + TN) * sizeof(float);
    hipLaunchKernelGGL(k_gemm_chains2<BK>, grid, dim3(256), lds, (hipStream_t)stream, At, lda, D, In, Out, bias,
                       triangle, ldc, phase, active_count, num_chains, (float*)workspace, ks, order, n_rt, n_ct);
  } else {
    hipLaunchKernelGGL(k_gemm_chains, grid, dim3(256), 0, (hipStream_t)stream, At, lda, D, In, Out, bias, triangle,
                       ldc, phase, active_count, num_chains, (float*)workspace, ks, order, n_rt, n_ct);
  }
  if (ks > 1)
    hipLaunchKernelGGL(k_gemm_reduce, dim3((D + 15) / 16, ldc / TN), dim3(256), 0, (hipStream_t)stream,
                       (const float*)workspace, ks, D, ldc, Out, bias, phase, active_count, num_chains);
  return nmx_check_launch("k_gemm_chains");
}

extern "C" size_t nmx_gemm_x3_packed_a_bytes(int lda) {
  return lda > 0 && lda % TM == 0 ? (size_t)lda * lda * 6 : 0;
}

extern "C" int nmx_gemm_x3_pack_a(const float* At, int lda, void* Ap, void* stream) {
  if (!At || !Ap || lda <= 0 || lda % TM) return nmx_fail(NMX_ERR_INVALID, "gemm_x3_pack_a: bad arguments");
  const int64_t n = (int64_t)(lda / 16) * (lda / 32) * 64;
  hipLaunchKernelGGL(k_x3_pack_a, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, At, lda,
                     (bf16x8*)Ap);
  return nmx_check_launch("k_x3_pack_a");
}

extern "C" size_t nmx_gemm_x3_split_bytes(int lda, int ldc) {
  return lda > 0 && ldc > 0 ? (size_t)(lda / 16) * 16 * ldc * 6 : 0;
}

namespace {
template <int CT, int NBUF, int RW>
int launch_gemm_x3(const void* Ap, int lda, int D, const void* split, float* Out, const float* bias, int triangle,
                   int ldc, const int32_t* phase, const int32_t* active_count, int num_chains, void* workspace,
                   int ks, hipStream_t s, const int32_t* out_list, const float* pe_in, float* pe_out) {
  const int n_rt = (lda + 32 * RW - 1) / (32 * RW), n_ct = (ldc + 32 * CT - 1) / (32 * CT);
  const dim3 grid((n_rt + 7) / 8 * 8 * n_ct, 1, ks);
  constexpr size_t lds = (size_t)NBUF * x3_pieces<CT, RW>() * 1024;
  if (const int st = nmx_lds_limit((const void*)k_gemm_x3<CT, NBUF, RW>, lds, s, "gemm_x3")) return st;
  hipLaunchKernelGGL((k_gemm_x3<CT, NBUF, RW>), grid, dim3(64 * RW), lds, s, (const char*)Ap, lda, D,
                     (const char*)split, Out, bias, triangle, ldc, phase, active_count, num_chains, (float*)workspace,
                     ks, 1, n_rt, n_ct, out_list, pe_in, pe_out);
  return NMX_OK;
}
}  // namespace

namespace {
int gemm_chains_x3(const void* Ap, int lda, int D, const float* In, const int32_t* rows_list, float* Out,
                   const float* bias, int triangle, int ldc, const int32_t* phase, const int32_t* active_count,
                   int num_chains, void* split, void* workspace, void* stream, const int32_t* out_list = nullptr,
                   const float* pe_in = nullptr, float* pe_out = nullptr);
}  // namespace

extern "C" int nmx_gemm_chains_x3(const void* Ap, int lda, int D, const float* In, float* Out, const float* bias,
                                  int triangle, int ldc, const int32_t* phase, const int32_t* active_count,
                                  int num_chains, void* split, void* workspace, void* stream) {
  return gemm_chains_x3(Ap, lda, D, In, nullptr, Out, bias, triangle, ldc, phase, active_count, num_chains, split,
                        workspace, stream);
}

extern "C" int nmx_gemm_chains_x3_rows(const void* Ap, int lda, int D, const float* rows, const int32_t* list,
                                       float* Out, const float* bias, int triangle, int ldc,
                                       const int32_t* active_count, int num_chains, void* split, void* workspace,
                                       void* stream) {
  if (!list || !active_count) return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3_rows: needs the list and its count");
  return gemm_chains_x3(Ap, lda, D, rows, list, Out, bias, triangle, ldc, nullptr, active_count, num_chains, split,
                        workspace, stream);
}

extern "C" int nmx_gemm_chains_x3_to_rows(const void* Ap, int lda, int D, const float* In, const int32_t* list,
                                          float* rows, const float* bias, int triangle, int ldc,
                                          const int32_t* active_count, int num_chains, void* split,
                                          const float* pe_in, float* pe_out, void* stream) {
  if (!list || !active_count || (pe_in && !pe_out))
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3_to_rows: needs the list and its count (and pe_out with pe_in)");
  return gemm_chains_x3(Ap, lda, D, In, nullptr, rows, bias, triangle, ldc, nullptr, active_count, num_chains, split,
                        nullptr, stream, list, pe_in, pe_out);
}

extern "C" int nmx_gemm_chains_x3_lists(const void* Ap, int lda, int D, const float* In, const int32_t* in_list,
                                        float* Out, const int32_t* out_list, const float* bias, int triangle, int ldc,
                                        const int32_t* active_count, int num_chains, void* split, const float* pe_in,
                                        float* pe_out, void* stream) {
  if (!active_count || (pe_in && (!pe_out || !out_list)))
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3_lists: needs the count (and out_list, pe_out with pe_in)");
  return gemm_chains_x3(Ap, lda, D, In, in_list, Out, bias, triangle, ldc, nullptr, active_count, num_chains, split,
                        nullptr, stream, out_list, pe_in, pe_out);
}

namespace {
int gemm_chains_x3(const void* Ap, int lda, int D, const float* In, const int32_t* rows_list, float* Out,
                   const float* bias, int triangle, int ldc, const int32_t* phase, const int32_t* active_count,
                   int num_chains, void* split, void* workspace, void* stream, const int32_t* out_list,
                   const float* pe_in, float* pe_out) {
  if (!Ap || !In || !Out || !split) return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3: NULL operand");
  if (D <= 0 || ldc % 64 || num_chains <= 0 || num_chains > ldc)
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3: bad sizes (D=%d ldc=%d C=%d)", D, ldc, num_chains);
  if (lda % TM || lda < nmx_dense_padded_dim(D))
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3: lda must be a multiple of %d >= padded D", TM);
  if (In == Out) return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3: In and Out must not alias");
  if (triangle < 0 || triangle > 2) return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3: triangle must be 0, 1 or 2");
  if ((int64_t)lda * lda * 6 > 0x7fffffff || (int64_t)lda * ldc * 6 > 0x7fffffff)
    return nmx_fail(NMX_ERR_INVALID, "gemm_chains_x3: operands exceed 2 GiB (lda=%d ldc=%d)", lda, ldc);
  hipStream_t s = (hipStream_t)stream;
  const int n_ks = lda / 16;
  const int64_t nb = (int64_t)n_ks * (ldc / 32) * 64;
  if (rows_list)
    hipLaunchKernelGGL(k_x3_split_b_rows, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, In, D, rows_list, ldc,
                       n_ks, active_count, (bf16x8*)split);
  else
    hipLaunchKernelGGL(k_x3_split_b, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, In, D, ldc, n_ks,
                       active_count, (bf16x8*)split);
  if (int st = nmx_check_launch("k_x3_split_b")) return st;
  // K-splits: a function of D only (never of C), at most ksplit_for(D) (the workspace size);
  // measured at D = 10000 (profiles/r01): no split is fastest all-active (2.2 vs 2.4 ms per
  // triangular product at C = 4096), 2 splits at C = 512 (0.33 vs 0.37)
  const int ks = (workspace && !out_list) ? (D <= 16384 ? 1 : (D + 8191) / 8192) : 1;
  // XCD-aware order always: the chain tiles of a row tile run on one XCD and share its A
  // stages in L2 (the split operand is 1.5x the f32 bytes; 2.7 vs 4.2 ms at D = 10000)
  // Two workgroup tiles, the same products bitwise (an output's k sequence and its MFMAs do
  // not depend on the tile; the tile only decides which workgroup computes it): 256 rows x 128
  // chains (8 waves, one workgroup per CU, half the staged bytes per MFMA: 214 vs 186 TF/s at
  // D = 10000, C = 4096) when that grid still gives two workgroups per CU, else 128 x 64 (two
  // workgroups per CU: better for few chains or small D)
  // (K-split launches keep the 128 x 64 tile: their split points depend on the tile's K range)
  const bool big = NMX_GEMM_BIG && ks == 1 && (int64_t)((lda + 255) / 256) * ((num_chains + 127) / 128) >= NMX_GEMM_BIG_MIN;
  if (big) {
    if (int st = launch_gemm_x3<4, 2, 8>(Ap, lda, D, split, Out, bias, triangle, ldc, phase, active_count,
                                         num_chains, workspace, ks, s, out_list, pe_in, pe_out))
      return st;
  } else {
    if (int st = launch_gemm_x3<NMX_GEMM_CT, NMX_GEMM_NBUF, NMX_GEMM_RW>(Ap, lda, D, split, Out, bias, triangle, ldc,
                                                                       phase, active_count, num_chains, workspace,
                                                                       ks, s, out_list, pe_in, pe_out))
      return st;
  }
  if (ks > 1)
    hipLaunchKernelGGL(k_gemm_reduce, dim3((D + 15) / 16, ldc / TN), dim3(256), 0, s, (const float*)workspace, ks,
                       D, ldc, Out, bias, phase, active_count, num_chains);
  return nmx_check_launch("k_gemm_x3");
}
}  // namespace

extern "C" int nmx_pe_mvn(const float* prec_t, int lda, const float* mu, const float* neg_prec_mu, int dim,
                          const nmx_eval_batch* ev, void* stream) {
  if (!ev || !ev->z || !ev->grad || !ev->pe || !mu || !neg_prec_mu)
    return nmx_fail(NMX_ERR_INVALID, "mvn: NULL operand");
  // the product selects chains by phase over chain indices; with a compacted list of chain
  // indices, ev->num_chains bounds the list count, not the indices (a listed chain can sit
  // anywhere below ldc), so the index range is the whole batch then
  const int nc = (ev->active_idx && ev->phase) ? ev->ldc : ev->num_chains;
  if (int st = nmx_gemm_chains(prec_t, lda, dim, ev->z, ev->grad, neg_prec_mu, 0, ev->ldc, ev->phase, nullptr, nc,
                               nullptr, stream))
    return st;
  hipLaunchKernelGGL(k_quad_pe, dim3(ev->ldc / 64), dim3(256), 0, (hipStream_t)stream, mu, dim, *ev);
  return nmx_check_launch("k_quad_pe");
}
