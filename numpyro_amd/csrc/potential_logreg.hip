// Logistic-regression potential + gradient for thousands of chains (examples/covtype.py:66-71).
//
//   U(b)  = sum_n [max(l_n,0) + log1p(exp(-|l_n|)) - y_n l_n] + sum_d [b_d^2/2 + log(2pi)/2]
//   dU/db = X^T (sigmoid(l) - y) + b,      l = X b          
//
// Default kernel: k_logreg_x3 (variant 36), f32-accurate split-bf16 GEMMs on the bf16 matrix
// cores (section "Split-bf16 kernel" below).  f32-MFMA forms (variant 22 k_logreg_rowlanes,
// the generic k_logreg_tiles) stay as A/B references.  In all of them, for a 32-row tile and
// 32 chains a wave computes L = X.Z, applies the Bernoulli epilogue to the accumulator
// registers in place and feeds them as the B operand of G += X^T.R: the 32x32 result holds
// chains on the lane and rows in the registers, which is the B-operand layout (for the
// 32x32x16 bf16 form with the k order permuted) -- no shuffle, no LDS round trip, and the
// N x C logit matrix never exists in memory.
//
// Packed X (nmx_logreg_pack): f32 rows for the f32 kernels (128-row padding, each row K+1
// floats, K = round_up(D, 2): x_0..x_{D-1}, zero pad, label; the odd stride makes the GEMM1
// operand read bank-conflict free), the float64 column terms w, then the split-bf16 tiles.
//
// Work split: grid = chain groups x S row splits.  S depends on n_rows only, and each split
// sums its rows in a fixed order, so a chain's U and dU do not depend on how many chains
// share the launch (GPU-count invariance).  Per-split partials go to slabs reduced in fixed
// order by k_logreg_finalize.  Workgroups of the same split are placed on one XCD
// (blockIdx % 8) so the chain groups share X tiles in L2.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BR = 64;       // rows per LDS stage of the generic kernel
constexpr int PACK = 128;    // packed row padding (= stage of the row-lane kernel)
constexpr int NW = 4;        // waves per workgroup
constexpr int CPB = NW * 32; // chains per workgroup
constexpr int MAX_S = 128;   // row splits
constexpr int LDS_SLACK = 64;

inline int k_of(int D) { return (D + 1) / 2 * 2; }
inline int xs_of(int D) { return k_of(D) + 1; }
inline int64_t npad_of(int64_t n) { return (n + PACK - 1) / PACK * PACK; }
inline int64_t ntiles_of(int64_t n) { return npad_of(n) / BR; }

int num_splits(int64_t n_rows) {
  int64_t t = npad_of(n_rows) / PACK;
  int64_t s = t / 16;
  s = s / 8 * 8;
  if (s < 8) s = 8;
  if (s > MAX_S) s = MAX_S;
  return (int)s;
}

__global__ void k_logreg_pack(const float* X, const float* y, int64_t n, int D, int XS, int64_t npad,
                              float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = npad * XS;
  if (i >= total) return;
  const int64_t row = i / XS;
  const int k = (int)(i - row * XS);
  float v = 0.0f;
  if (row < n) {
    if (k < D) v = X[row * D + k];
    else if (k == XS - 1) v = y[row];
  }
  out[i] = v;
}

// w[d] = sum_n X[n,d] / 2 - sum_n y_n X[n,d] in float64 (the per-chain linear part of U used
// by epilogue_abs).  One workgroup per column, fixed thread count and a fixed-order tree, so
// the value does not depend on anything but the data.
constexpr int CS_THREADS = 256;
__global__ __launch_bounds__(CS_THREADS) void k_logreg_colsums(const float* X, const float* y, int64_t n, int D,
                                                              double* w) {
  __shared__ double red[CS_THREADS];
  const int d = blockIdx.x;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CS_THREADS) {
    const double x = X[i * D + d];
    acc += 0.5 * x - (double)y[i] * x;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int k = CS_THREADS / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) w[d] = red[0];
}

// byte offset of the float64 column terms behind the packed rows
inline size_t colterm_offset(int64_t n_rows, int dim) {
  return ((size_t)npad_of(n_rows) * xs_of(dim) * sizeof(float) + 255) / 256 * 256;
}

// KS = K/2 MFMA k-steps.  EXACT: the dim's KS equals the template (compile-time strides);
// otherwise KS is an upper bound and the packed stride comes at run time.
template <int KS, bool EXACT>
__global__ __launch_bounds__(NW * 64) void k_logreg_tiles(const float* __restrict__ Xp, int64_t n_rows,
                                                          int ntiles, int D, int S, int Gc,
                                                          nmx_eval_batch ev, float* __restrict__ gpart,
                                                          double* __restrict__ pepart) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int ks = EXACT ? KS : (D + 1) / 2;
  const int XS = EXACT ? 2 * KS + 1 : 2 * ks + 1;
  const int b = blockIdx.x;
  const int xcd = b & 7;
  const int q = b >> 3;
  const int cg = q % Gc;
  const int split = (q / Gc) * 8 + xcd;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int h = lane >> 5;
  const int l31 = lane & 31;
  const int ldc = ev.ldc;
  const int pos = cg * CPB + w * 32 + l31;  // batch position (slab column)
  const bool cin = pos < ldc;
  const int c = cin ? nmx_eval_chain(ev, pos) : -1;
  const bool act = c >= 0;
  const bool wave_active = __any(act);
  if (!__syncthreads_or(wave_active)) return;

  if (tid < LDS_SLACK) xs[BR * XS + tid] = 0.0f;

  const int per = (ntiles + S - 1) / S;
  const int t0 = split * per;
  const int t1 = min(t0 + per, ntiles);

  // B operand of GEMM1 for this wave's 32 chains: Z[k = 2s + h][chain]
  float zb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    zb[s] = (k < D && act) ? ev.z[(size_t)k * ldc + c] : 0.0f;
  }
  f32x16 g0, g1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    g0[r] = 0.0f;
    g1[r] = 0.0f;
  }
  double pe = 0.0;
  const bool two_blocks = D > 32;

  for (int t = t0; t < t1; ++t) {
    __syncthreads();
    {
      const float4* src = reinterpret_cast<const float4*>(Xp + (size_t)t * BR * XS);
      float4* dst = reinterpret_cast<float4*>(xs);
      const int NCH = BR * XS / 4;
      for (int i = tid; i < NCH; i += NW * 64) dst[i] = src[i];
    }
    __syncthreads();
    if (!wave_active) continue;
#pragma unroll 1
    for (int sub = 0; sub < BR / 32; ++sub) {
      const float* xt = xs + sub * 32 * XS;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        if (EXACT || s < ks)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xt[l31 * XS + 2 * s + h], zb[s], acc, 0, 0, 0);
      // Bernoulli-logits epilogue in place: acc[r] <- sigmoid(l) - y (masked past n_rows)
      const int64_t rowbase = (int64_t)t * BR + sub * 32;
      float pes = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float y = xt[rr * XS + (XS - 1)];
        const float lg = acc[r];
        const bool ok = rowbase + rr < n_rows;
        const float e = __expf(-fabsf(lg));
        const float onepe = 1.0f + e;
        const float bce = fmaxf(lg, 0.0f) + __logf(onepe) - lg * y;  // util.py:295-298
        const float inv = __builtin_amdgcn_rcpf(onepe);
        const float sig = lg >= 0.0f ? inv : e * inv;
        pes += ok ? bce : 0.0f;
        acc[r] = ok ? sig - y : 0.0f;
      }
      pe += (double)pes;
      // G += X^T R: A[d][row] from LDS, B = the epilogue registers
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
        g0 = __builtin_amdgcn_mfma_f32_32x32x2f32(xt[rr * XS + l31], acc[r], g0, 0, 0, 0);
        if (two_blocks)
          g1 = __builtin_amdgcn_mfma_f32_32x32x2f32(xt[rr * XS + 32 + l31], acc[r], g1, 0, 0, 0);
      }
    }
  }

  if (wave_active && cin) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = (r & 3) + 8 * (r >> 2) + 4 * h;
      if (d < D) gpart[((size_t)split * D + d) * ldc + pos] = g0[r];
      if (d + 32 < D) gpart[((size_t)split * D + d + 32) * ldc + pos] = g1[r];
    }
  }
  pe += __shfl_xor(pe, 32);
  if (wave_active && cin && h == 0) pepart[(size_t)split * ldc + pos] = pe;
}

// ---------------------------------------------------------------------------------------
// f32-MFMA row-lane kernel (variant 22, D = 55): see k_logreg_rowlanes below.
// ---------------------------------------------------------------------------------------
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// acc <- sigmoid(l) - y in place, with the linear part of U taken out of the row loop:
//   max(l,0) - l y = (|l| + l)/2 - l y,   sum_n l_n = (sum_n x_n) . b,   sum_n l_n y_n = (X^T y) . b,
// the rows only accumulate |l| and the chain adds w . b once, w = sum_n x_n / 2 - X^T y
// (k_logreg_colsums, float64); log(1+e) summed as log2 of the product of the 16 factors.
template <int KS, bool MASK>
__device__ __forceinline__ void epilogue_abs(const float* xt, int h, int64_t rowbase, int64_t n_rows, f32x16& acc,
                                             float& lin, float& lg2) {
  constexpr int XS = 2 * KS + 1;
  float prod = 1.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
    const float y = xt[rr * XS + (XS - 1)];
    const float l = acc[r];
    float al = fabsf(l);
    const float e = __builtin_amdgcn_exp2f(-al * LOG2E);
    float ope = 1.0f + e;
    const float inv = __builtin_amdgcn_rcpf(ope);
    const float num = l >= 0.0f ? 1.0f : e;
    float res = __builtin_fmaf(num, inv, -y);
    if (MASK) {
      const bool ok = rowbase + rr < n_rows;
      res = ok ? res : 0.0f;
      al = ok ? al : 0.0f;
      ope = ok ? ope : 1.0f;
    }
    lin += al;
    prod *= ope;
    acc[r] = res;
  }
  lin *= 0.5f;
  lg2 += __builtin_amdgcn_logf(prod);
}

constexpr int RL_WAVES = 4;             // row lanes per workgroup
constexpr int RL_ROWS = 32 * RL_WAVES;  // rows per stage (= PACK)
static_assert(RL_ROWS == PACK, "row-lane stage must equal the packing granularity");

// f32-MFMA row-lane kernel (variant 22; the default before the split-bf16 kernel, kept as the
// f32 A/B reference).  Workgroup = 4 waves sharing ONE 32-chain tile; each wave is a "row
// lane" taking one 32-row subtile of each 128-row stage, DMA'd into its own LDS slice by
// buffer LDS-DMA (no workgroup barrier in the row loop); the last stage (rows >= N) is peeled
// so the unmasked epilogue is branch-free.  The 4 lanes' partials are combined in a fixed
// order at the end; S row splits depend on n_rows only.
template <int KS>
__global__ __launch_bounds__(RL_WAVES * 64, 2) void k_logreg_rowlanes(const float* __restrict__ Xp, int64_t n_rows,
                                                                     int nstages, int D, int S, int Gt,
                                                                     nmx_eval_batch ev, float* __restrict__ gpart,
                                                                     double* __restrict__ pepart) {
  constexpr int XS = 2 * KS + 1;
  constexpr int STAGE = RL_ROWS * XS;
  constexpr int WPIECES = (32 * XS + 255) / 256;  // 1 KB DMA pieces per wave subtile
  constexpr int WSLICE = WPIECES * 256;           // floats per wave slice
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int b = blockIdx.x;
  const int xcd = b & 7;
  const int q = b >> 3;
  const int ct = q % Gt;
  const int split = (q / Gt) * 8 + xcd;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int h = lane >> 5;
  const int l31 = lane & 31;
  const int ldc = ev.ldc;
  const int pos = ct * 32 + l31;
  const int cc = pos < ldc ? nmx_eval_chain(ev, pos) : -1;
  if (!__any(cc >= 0)) return;  // identical in all waves of the workgroup
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)Xp, 0, nstages * STAGE * 4, 0x00020000);

  const int per = (nstages + S - 1) / S;
  const int t0 = split * per;
  const int t1 = min(t0 + per, nstages);

  float zb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    zb[s] = (k < D && cc >= 0) ? ev.z[(size_t)k * ldc + cc] : 0.0f;
  }
  f32x16 g0, g1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    g0[r] = 0.0f;
    g1[r] = 0.0f;
  }
  double pe = 0.0;
  // TAIL: the stage holds rows >= n_rows (only the last one can): masked epilogue
  auto stage = [&](int st, auto tailc) {
    constexpr bool TAIL = decltype(tailc)::value;
    // wave-private pipeline: each wave DMAs only its own 32-row subtile into its own LDS slice
    // and waits for its own loads; its previous reads of the slice were consumed (MFMA/VALU
    // operands) before this point
    float* xt = xs + wu * WSLICE;
    const unsigned base = (unsigned)(((int64_t)st * RL_ROWS + wu * 32) * XS * 4);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < WPIECES; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(xt + i * 256), 16,
                                               lane * 16, base + i * 1024, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int64_t rb = (int64_t)st * RL_ROWS + w * 32;
    f32x16 a;
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.0f;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < KS; ++s) a = __builtin_amdgcn_mfma_f32_32x32x2f32(xt[l31 * XS + 2 * s + h], zb[s], a, 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    float lin = 0.0f, lg2 = 0.0f;
    // only the waves holding rows >= n_rows mask
    if (TAIL && rb + 32 > n_rows) epilogue_abs<KS, true>(xt, h, rb, n_rows, a, lin, lg2);
    else epilogue_abs<KS, false>(xt, h, rb, n_rows, a, lin, lg2);
    pe += (double)lin + (double)lg2 * (double)LN2;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
      g0 = __builtin_amdgcn_mfma_f32_32x32x2f32(xt[rr * XS + l31], a[r], g0, 0, 0, 0);
      if (KS > 16) g1 = __builtin_amdgcn_mfma_f32_32x32x2f32(xt[rr * XS + 32 + l31], a[r], g1, 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  const int t_full = (int)min((int64_t)t1, n_rows / RL_ROWS);  // stages with all 128 rows < n_rows
  int st = t0;
  for (; st < t_full; ++st) stage(st, std::false_type{});
  for (; st < t1; ++st) stage(st, std::true_type{});

  __syncthreads();  // every wave is done with its slice
  // fixed-order combination of the 4 row lanes: waves 1-3 park their partials in LDS, wave 0
  // adds them to its registers in wave order
  float* red = xs;                                                            // [RL_WAVES-1][32][64]
  double* red_pe = reinterpret_cast<double*>(xs + (RL_WAVES - 1) * 32 * 64);  // [RL_WAVES-1][64]
  const double p = pe + __shfl_xor(pe, 32);
  if (w > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      red[((w - 1) * 32 + r) * 64 + lane] = g0[r];
      red[((w - 1) * 32 + 16 + r) * 64 + lane] = g1[r];
    }
    red_pe[(w - 1) * 64 + lane] = p;
  }
  __syncthreads();
  if (w == 0 && pos < ldc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s0 = g0[r], s1 = g1[r];
#pragma unroll
      for (int ww = 1; ww < RL_WAVES; ++ww) {
        s0 += red[((ww - 1) * 32 + r) * 64 + lane];
        s1 += red[((ww - 1) * 32 + 16 + r) * 64 + lane];
      }
      const int d = (r & 3) + 8 * (r >> 2) + 4 * h;
      if (d < D) gpart[((size_t)split * D + d) * ldc + pos] = s0;
      if (d + 32 < D) gpart[((size_t)split * D + d + 32) * ldc + pos] = s1;
    }
    if (h == 0) {
      double sp = p;
#pragma unroll
      for (int ww = 1; ww < RL_WAVES; ++ww) sp += red_pe[(ww - 1) * 64 + lane];
      pepart[(size_t)split * ldc + pos] = sp;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 kernel (variant 30): f32-accurate products on the bf16 matrix cores.
//
// Every f32 operand v is split into three bf16 terms, v1 = bf16(v), v2 = bf16(v - v1),
// v3 = bf16(v - v1 - v2) (round to nearest; the remainders are exact in f32), which
// represents v to within 2^-24 |v| -- the f32 rounding unit.  A product a.b keeps the six
// terms with i + j <= 4 (a3b1 + a2b2 + a1b3 + a2b1 + a1b2 + a1b1, small terms first); the
// three dropped ones are each below 2^-24 |ab|.  A bf16 x bf16 product is exact in f32 and
// v_mfma_f32_32x32x16_bf16 accumulates in f32, so each output carries f32-level accuracy
// (tests/test_gpu_potentials.py compares its error against the f32-MFMA kernel's, both
// vs float64) for 6 bf16 MFMAs per 16-deep k-step, against 8 f32 MFMAs (32x32x2) at 2x the
// cycles each: 32 vs 64 cycles per MFMA, 6 x 32 = 192 vs 8 x 64 = 512 cycles per k-step.
//
// Packed layout (nmx_logreg_pack, behind the f32 rows): per 32-row tile NP = 3 KB + 6 DT + 1
// pieces of 1 KB, each a 64-lane x 16-byte MFMA operand fragment in lane order, so a wave
// reads an operand with one conflict-free ds_read_b128 and the LDS-DMA copy is linear:
//   piece p*KB + kb                 GEMM1 A = X[32 rows][16 cols], plane p, k-block kb:
//                                   lane (r, h) holds X[r][16 kb + 8 h + j]
//   piece 3KB + p*2DT + 2 dt + s    GEMM2 A = X^T[32 cols][16 rows], plane p, col tile dt,
//                                   k-step s: lane (r, h) element j holds
//                                   X[16 s + 8 (j>>2) + 4 h + (j&3)][32 dt + r] -- the k order
//                                   of the GEMM1 accumulator used as the B operand
//   piece NP-1                      labels y[h][i] of row (i&3) + 8 (i>>2) + 4 h, then zeros
// Rows >= n_rows are zero (l = 0: no gradient, an exact log(2) each in U, removed in the
// finalize), columns >= D are zero.  KB = ceil(D/16), DT = ceil(D/32).
//
// Workgroup = 4 waves = 4 chain tiles of 32 sharing each X tile; X tiles stream through a
// 3-slot LDS ring by buffer LDS-DMA, one workgroup barrier per tile.  Grid = chain groups x
// S2 row splits, S2 a function of n_rows only (fixed summation order, as for the f32
// kernels); the partials go through the same slabs and finalize.
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int X3_ROWS = 32;
constexpr int X3_MAX_S = 256;

inline int x3_kb(int D) { return (D + 15) / 16; }
inline int x3_dt(int D) { return (D + 31) / 32; }
inline int x3_np(int D) { return 3 * x3_kb(D) + 6 * x3_dt(D) + 1; }
inline int64_t x3_ntiles(int64_t n) { return (n + X3_ROWS - 1) / X3_ROWS; }

int x3_num_splits(int64_t n_rows) {
  static const int max_s = [] {
    const char* e = getenv("NMX_X3_MAX_SPLITS");  // experiments only; must not change between bind and use
    return e ? atoi(e) : X3_MAX_S;
  }();
  int64_t s = x3_ntiles(n_rows) / 16;
  s = s / 8 * 8;
  if (s < 8) s = 8;
  if (s > max_s) s = max_s;
  return (int)s;
}

// three-term bf16 split of 8 floats (round to nearest even at every step)
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

// one thread per (tile, piece, lane): 16 bytes of one operand fragment
__global__ void k_logreg_pack_x3(const float* __restrict__ X, const float* __restrict__ y, int64_t n, int D,
                                 int KB, int DT, int64_t ntiles, bf16x8* __restrict__ out) {
  const int NP = 3 * KB + 6 * DT + 1;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ntiles * NP * 64) return;
  const int lane = (int)(i & 63);
  const int64_t q = i >> 6;
  const int piece = (int)(q % NP);
  const int64_t t = q / NP;
  const int r = lane & 31, h = lane >> 5;
  const int64_t r0 = t * X3_ROWS;
  float v[8];
  int plane = 0;
  if (piece < 3 * KB) {
    plane = piece / KB;
    const int kb = piece % KB;
    const int64_t row = r0 + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 16 * kb + 8 * h + j;
      v[j] = (row < n && d < D) ? X[row * D + d] : 0.0f;
    }
  } else if (piece < NP - 1) {
    const int qq = piece - 3 * KB;
    plane = qq / (2 * DT);
    const int rem = qq % (2 * DT);
    const int dt = rem >> 1, s = rem & 1;
    const int d = 32 * dt + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t row = r0 + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
      v[j] = (row < n && d < D) ? X[row * D + d] : 0.0f;
    }
  } else {
    // labels as floats: lane L < 8 holds y[h = L/4][i = 4 (L%4) .. +3] (bytes 16 L .. 16 L + 15)
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (lane < 8) {
      const int hh = lane >> 2;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ii = 4 * (lane & 3) + k;
        const int64_t row = r0 + (ii & 3) + 8 * (ii >> 2) + 4 * hh;
        f[k] = row < n ? y[row] : 0.0f;
      }
    }
    float4* o = reinterpret_cast<float4*>(out + i);
    *o = make_float4(f[0], f[1], f[2], f[3]);
    return;
  }
  bf16x8 b1, b2, b3;
  split3(v, b1, b2, b3);
  out[i] = plane == 0 ? b1 : (plane == 1 ? b2 : b3);
}

template <int N>
__device__ __forceinline__ void x3_wait_vm() {
  // s_waitcnt vmcnt(N), other counters untouched (gfx9 encoding: vmcnt[3:0] | expcnt 7 << 4
  // | lgkmcnt 15 << 8 | vmcnt[5:4] << 14)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// GEMM1 of one tile: L = X . Z (32 rows x 32 chains), six split products per k-block
template <int KB>
__device__ __forceinline__ f32x16 x3_gemm1(const bf16x8* fr, const bf16x8 (&z1)[KB], const bf16x8 (&z2)[KB],
                                           const bf16x8 (&z3)[KB]) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const bf16x8 a1 = fr[(0 * KB + kb) * 64], a2 = fr[(1 * KB + kb) * 64], a3 = fr[(2 * KB + kb) * 64];
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, z1[kb], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z2[kb], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z3[kb], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z1[kb], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z2[kb], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z1[kb], acc, 0, 0, 0);
  }
  return acc;
}

// Labels of a tile (16 per lane, rows of the accumulator layout), read by inline asm: a
// compiler-visible LDS read here gets an s_waitcnt vmcnt(0) (the wait tracking cannot tell
// it from the ring slots still being filled), which would drain the prefetch.  x3_labels_wait
// must run before the values are used.
__device__ __forceinline__ void x3_labels(const char* ybase, int h, f32x4 (&y4)[4]) {
  const unsigned ya = (unsigned)(size_t)((__attribute__((address_space(3))) const char*)ybase) + 64 * h;
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:16\n\t"
      "ds_read_b128 %2, %4 offset:32\n\t"
      "ds_read_b128 %3, %4 offset:48"
      : "=&v"(y4[0]), "=&v"(y4[1]), "=&v"(y4[2]), "=&v"(y4[3])
      : "v"(ya));
}
__device__ __forceinline__ void x3_labels_wait(f32x4 (&y4)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(y4[0]), "+v"(y4[1]), "+v"(y4[2]), "+v"(y4[3]));
}

// Bernoulli-logits epilogue (epilogue_abs arithmetic; no row mask: padded rows have l = 0):
// acc -> sigmoid(l) - y, U terms into pe
// L2E: the accumulator holds m = -l log2(e) (Z pre-scaled by -log2 e before its split), so
// e = 2^-|m| needs no multiply and sum |l| = ln 2 sum |m|
template <bool L2E = false>
__device__ __forceinline__ void x3_epilogue(const f32x16& acc, const f32x4 (&y4)[4], float (&res)[16], double& pe) {
  float lin = 0.0f, prod = 1.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = 4 * q + u;
      const float l = acc[r];
      const float al = fabsf(l);
      const float e = __builtin_amdgcn_exp2f(L2E ? -al : -al * LOG2E);
      const float ope = 1.0f + e;
      const float inv = __builtin_amdgcn_rcpf(ope);
      const float num = (L2E ? l <= 0.0f : l >= 0.0f) ? 1.0f : e;
      res[r] = __builtin_fmaf(num, inv, -y4[q][u]);
      lin += al;
      prod *= ope;
    }
  }
  pe += (double)(0.5f * lin) * (L2E ? (double)LN2 : 1.0) + (double)__builtin_amdgcn_logf(prod) * (double)LN2;
}

// GEMM2 of one tile: G += X^T . R, R split into three bf16 terms (k-step s = registers 8s..8s+7)
template <int KB, int DT>
__device__ __forceinline__ void x3_gemm2(const bf16x8* fr, const float (&res)[16], f32x16 (&g)[DT]) {
  constexpr int G2 = 3 * KB;  // first GEMM2 piece
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = res[8 * s + j];
    bf16x8 r1, r2, r3;
    split3(v, r1, r2, r3);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const bf16x8 b1 = fr[(G2 + 0 * 2 * DT + 2 * dt + s) * 64];
      const bf16x8 b2 = fr[(G2 + 1 * 2 * DT + 2 * dt + s) * 64];
      const bf16x8 b3 = fr[(G2 + 2 * 2 * DT + 2 * dt + s) * 64];
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b3, r1, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r2, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r3, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r1, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r2, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r1, g[dt], 0, 0, 0);
    }
  }
}

// PIPE: software-pipelined -- GEMM1 of tile k+1 is issued beside the epilogue of tile k (they
// are independent), then GEMM2 of tile k; needs RING = 3 (slots k, k+1 read, k+2 filling).
// The per-chain arithmetic and its order are the same in both forms (bitwise equal results).
//
template <int KB, int DT, int RING, bool PIPE, int SCHED, bool L2E>
__device__ __forceinline__ void x3_item(const char* __restrict__ Xq, int64_t ntiles, int D, int S, int split, int ct,
                                        nmx_eval_batch ev, float* __restrict__ gpart,
                                        double* __restrict__ pepart) {
  constexpr int NP = 3 * KB + 6 * DT + 1;
  constexpr int PPW = (NP + 3) / 4;     // DMA pieces per wave per tile (max)
  static_assert(!PIPE || RING == 3 || RING == 4, "the pipelined loop reads two slots while a third fills");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const int l31 = lane & 31;
  const int ldc = ev.ldc;
  const int pos = (ct * 4 + wu) * 32 + l31;
  const int c = pos < ldc ? nmx_eval_chain(ev, pos) : -1;
  const bool active = __any(c >= 0);  // wave-uniform
  if (!__syncthreads_or(active)) return;  // workgroup-uniform

  const int64_t per = (ntiles + S - 1) / S;
  const int64_t t0 = min((int64_t)split * per, ntiles);
  const int64_t t1 = min(t0 + per, ntiles);
  const int nt = (int)(t1 - t0);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Xq + (size_t)t0 * NP * 1024), 0, (int)((size_t)nt * NP * 1024), 0x00020000);
  // pieces of this wave: wu, wu + 4, ... (PPW of them, or PPW - 1)
  const bool full = wu < NP - 4 * (PPW - 1);

  // Z through a buffer descriptor: coordinates >= D and inactive lanes (c = -1) fall outside
  // its range and read 0, so the loads need no per-element conditions (conditions and 64-bit
  // addresses hoisted out of the item loop spilled)
  const __amdgpu_buffer_rsrc_t zrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)ev.z, 0, D * ldc * 4, 0x00020000);
  const unsigned zoff = c >= 0 ? (unsigned)((8 * h * ldc + c) * 4) : 0xFFFFFFF0u;
  bf16x8 z1[KB], z2[KB], z3[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zrs, zoff, (16 * kb + j) * ldc * 4, 0));
    if constexpr (L2E) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= -LOG2E;
    }
    split3(v, z1[kb], z2[kb], z3[kb]);
  }
  f32x16 g[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) g[dt][r] = 0.0f;
  double pe = 0.0;

  auto issue = [&](int k) {  // tile t0 + k into ring slot k % RING
    char* dst = lds + (k % RING) * NP * 1024;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int i = wu + 4 * j;
      if (i < NP)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16,
                                                 lane * 16, (unsigned)((k * NP + i) * 1024), 0, 0);
    }
  };
  auto slot = [&](int k) { return lds + (k % RING) * NP * 1024; };
  if constexpr (PIPE && RING == 4) {
    // Split rings: GEMM1 reads only the A part of a tile (pieces < 3 KB), GEMM2 and the labels
    // only the B part.  Iteration k reads A(k+1) and B(k) while A(k+2) and B(k+1) fill, so two
    // slots of each part suffice: 2 x (12 + 13) KB for covtype, three workgroups per CU.
    constexpr int NA = 3 * KB, NBP = NP - NA;
    char* aring = lds;
    char* bring = lds + 2 * NA * 1024;
    auto issue_a = [&](int k) {
      char* dst = aring + (k & 1) * NA * 1024;
#pragma unroll
      for (int j = 0; j < (NA + 3) / 4; ++j) {
        const int i = wu + 4 * j;
        if (i < NA)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16,
                                                   lane * 16, (unsigned)((k * NP + i) * 1024), 0, 0);
      }
    };
    auto issue_b = [&](int k) {
      char* dst = bring + (k & 1) * NBP * 1024;
#pragma unroll
      for (int j = 0; j < (NBP + 3) / 4; ++j) {
        const int i = wu + 4 * j;
        if (i < NBP)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16,
                                                   lane * 16, (unsigned)((k * NP + NA + i) * 1024), 0, 0);
      }
    };
    if (nt > 0) {
      issue_a(0);
      x3_wait_vm<0>();
      asm volatile("s_barrier" ::: "memory");  // A(0) is in
      if (nt > 1) issue_a(1);
      issue_b(0);
      f32x16 acc;
      if (active) acc = x3_gemm1<KB>(reinterpret_cast<const bf16x8*>(aring) + lane, z1, z2, z3);
      for (int k = 0; k < nt; ++k) {
        // A(k+1) and B(k) have landed in every wave; A slot k&1 (GEMM1(k)) and B slot
        // (k+1)&1 (GEMM2(k-1)) were last read in iteration k-1
        x3_wait_vm<0>();
        asm volatile("s_barrier" ::: "memory");
        if (k + 2 < nt) issue_a(k + 2);
        if (k + 1 < nt) issue_b(k + 1);
        if (!active) continue;
        const char* bs = bring + (k & 1) * NBP * 1024;
        f32x4 y4[4];
        x3_labels(bs + (NBP - 1) * 1024, h, y4);
        x3_labels_wait(y4);
        // GEMM1 of tile k+1 (a stale slot past the last tile: computed, never used) beside
        // the epilogue of tile k
        const bf16x8* fa = reinterpret_cast<const bf16x8*>(aring + ((k + 1) & 1) * NA * 1024) + lane;
        float res[16];
        f32x16 nxt;
        if constexpr (SCHED && KB == 4) {
          // Hand-interleaved (in-order issue within a wave): each GEMM1(k+1) MFMA is followed
          // by one row's epilogue of tile k, which fills the MFMA's dependency stall; the first
          // split half then rides on the last k-block.  sched_barrier(0) pins the order; the
          // operations and their per-value order equal x3_gemm1 / x3_epilogue / x3_gemm2.
#pragma unroll
          for (int r = 0; r < 16; ++r) nxt[r] = 0.0f;
          float lin = 0.0f, prod = 1.0f;
          auto epi1 = [&](int r) {  // x3_epilogue<L2E>'s row r
            const float l = acc[r];
            const float al = fabsf(l);
            const float e = __builtin_amdgcn_exp2f(L2E ? -al : -al * LOG2E);
            const float ope = 1.0f + e;
            const float inv = __builtin_amdgcn_rcpf(ope);
            const float num = (L2E ? l <= 0.0f : l >= 0.0f) ? 1.0f : e;
            res[r] = __builtin_fmaf(num, inv, -y4[r >> 2][r & 3]);
            lin += al;
            prod *= ope;
          };
          bf16x8 a1 = fa[0 * 64], a2 = fa[KB * 64], a3 = fa[2 * KB * 64];
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            bf16x8 n1, n2, n3;
            if (kb + 1 < KB) {
              n1 = fa[(kb + 1) * 64];
              n2 = fa[(KB + kb + 1) * 64];
              n3 = fa[(2 * KB + kb + 1) * 64];
            }
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, z1[kb], nxt, 0, 0, 0);
            epi1(4 * kb + 0);
            __builtin_amdgcn_sched_barrier(0);
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z2[kb], nxt, 0, 0, 0);
            epi1(4 * kb + 1);
            __builtin_amdgcn_sched_barrier(0);
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z3[kb], nxt, 0, 0, 0);
            epi1(4 * kb + 2);
            __builtin_amdgcn_sched_barrier(0);
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z1[kb], nxt, 0, 0, 0);
            epi1(4 * kb + 3);
            __builtin_amdgcn_sched_barrier(0);
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z2[kb], nxt, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z1[kb], nxt, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (kb + 1 < KB) {
              a1 = n1;
              a2 = n2;
              a3 = n3;
            }
          }
          pe += (double)(0.5f * lin) * (L2E ? (double)LN2 : 1.0) + (double)__builtin_amdgcn_logf(prod) * (double)LN2;
        } else {
          nxt = x3_gemm1<KB>(fa, z1, z2, z3);
          x3_epilogue<L2E>(acc, y4, res, pe);
        }
        x3_gemm2<KB, DT>(reinterpret_cast<const bf16x8*>(bs) - NA * 64 + lane, res, g);
        acc = nxt;
      }
    }
  } else if constexpr (PIPE) {
    if (nt > 0) {
      issue(0);
      if (nt > 1) issue(1);
      if (nt > 1) {
        if (full) x3_wait_vm<PPW>();
        else x3_wait_vm<PPW - 1>();
      } else {
        x3_wait_vm<0>();
      }
      asm volatile("s_barrier" ::: "memory");  // tile 0 is in
      f32x16 acc;
      if (active) acc = x3_gemm1<KB>(reinterpret_cast<const bf16x8*>(slot(0)) + lane, z1, z2, z3);
      for (int k = 0; k < nt; ++k) {
        // tile k+1 has landed (in every wave); slot (k+2) % 3 was last read by GEMM2(k-1)
        x3_wait_vm<0>();
        asm volatile("s_barrier" ::: "memory");
        if (k + 2 < nt) issue(k + 2);
        if (!active) continue;
        const bf16x8* frk = reinterpret_cast<const bf16x8*>(slot(k)) + lane;
        f32x4 y4[4];
        x3_labels(slot(k) + (NP - 1) * 1024, h, y4);
        x3_labels_wait(y4);
        // GEMM1 of tile k+1 (junk slot past the last tile: computed, never used) beside the
        // epilogue of tile k
        const f32x16 nxt = x3_gemm1<KB>(reinterpret_cast<const bf16x8*>(slot(k + 1)) + lane, z1, z2, z3);
        float res[16];
        x3_epilogue<L2E>(acc, y4, res, pe);
        x3_gemm2<KB, DT>(frk, res, g);
        acc = nxt;
      }
    }
  } else {
    // RING slots, RING - 1 tiles in flight ahead of the one being computed
    for (int k = 0; k < RING - 1 && k < nt; ++k) issue(k);
    for (int k = 0; k < nt; ++k) {
      // this wave's pieces of tile k have landed (those of tile k + 1 may still fly)
      if (RING == 2 || k + 1 >= nt) x3_wait_vm<0>();
      else if (full) x3_wait_vm<PPW>();
      else x3_wait_vm<PPW - 1>();
      asm volatile("s_barrier" ::: "memory");  // ... and every wave's; slot (k-1) % RING is free
      if (k + RING - 1 < nt) issue(k + RING - 1);
      if (!active) continue;
      const bf16x8* fr = reinterpret_cast<const bf16x8*>(slot(k)) + lane;
      f32x4 y4[4];
      x3_labels(slot(k) + (NP - 1) * 1024, h, y4);
      const f32x16 acc = x3_gemm1<KB>(fr, z1, z2, z3);
      x3_labels_wait(y4);
      float res[16];
      x3_epilogue<L2E>(acc, y4, res, pe);
      x3_gemm2<KB, DT>(fr, res, g);
    }
  }
  if (!active || pos >= ldc) return;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = 32 * dt + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (d < D) gpart[((size_t)split * D + d) * ldc + pos] = g[dt][r];
    }
  const double p = pe + __shfl_xor(pe, 32);
  if (h == 0) pepart[(size_t)split * ldc + pos] = p;
}

// Grid = chain groups (128 batch positions) x S row splits.  Splits sp = x (mod 8) run on XCD x
// (workgroup b = x mod 8), the chain groups of a split on consecutive workgroups of that XCD, so
// they share X tiles in its L2.  A workgroup whose chain group lies past the compacted list's
// count leaves after one scalar load: the tail of a NUTS run launches thousands of them.
template <int KB, int DT, int RING, int MINB, bool PIPE, int SCHED = 0, bool L2E = false>
__global__ __launch_bounds__(256, MINB) void k_logreg_x3(const char* __restrict__ Xq, int64_t ntiles, int D, int S,
                                                     int Gt, nmx_eval_batch ev, float* __restrict__ gpart,
                                                     double* __restrict__ pepart) {
  const int b = blockIdx.x;
  const int qb = b >> 3;
  const int ct = qb % Gt;
  const int npos = ev.active_idx ? *ev.active_count : ev.ldc;
  if (ct * 128 >= npos) return;
  x3_item<KB, DT, RING, PIPE, SCHED, L2E>(Xq, ntiles, D, S, (qb / Gt) * 8 + (b & 7), ct, ev, gpart, pepart);
}

// Sum of slots sp0 .. sp1-1 at stride st (in slot order; 32 loads issued ahead of their adds)
template <class T>
__device__ __forceinline__ T sum_slots(const T* __restrict__ p, size_t st, int sp0, int sp1) {
  T s = 0;
  int sp = sp0;
  for (; sp + 32 <= sp1; sp += 32) {
    T v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(p + (size_t)(sp + j) * st);
#pragma unroll
    for (int j = 0; j < 32; ++j) s += v[j];
  }
  for (; sp < sp1; ++sp) s += p[(size_t)sp * st];
  return s;
}

// One workgroup per (64 batch positions, coordinate d or the U row d = D).  Wave w sums the
// slots [w S / 4, (w + 1) S / 4) in order, then the four are added in wave order: a fixed
// order that depends on S (a function of n_rows) only, and four independent load streams per
// output, so the small launches of a NUTS tail are not one long dependent chain of loads.
// wcol (epilogue_abs variants): U gains the per-chain linear term w . b; pe_shift removes the
// log(2) terms of the zero rows that pad the split-bf16 tiles
constexpr int FIN_WAVES = 4;
__global__ __launch_bounds__(64 * FIN_WAVES) void k_logreg_finalize(const float* __restrict__ gpart,
                                                                    const double* __restrict__ pepart, int S, int D,
                                                                    nmx_eval_batch ev,
                                                                    const double* __restrict__ wcol,
                                                                    double pe_shift) {
  __shared__ double part[FIN_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pos = blockIdx.x * 64 + lane;
  const int d = blockIdx.y;
  const int c = nmx_eval_chain(ev, pos);
  const int ldc = ev.ldc;
  const int sp0 = w * S / FIN_WAVES, sp1 = (w + 1) * S / FIN_WAVES;
  if (c >= 0) {
    if (d < D) part[w][lane] = sum_slots(gpart + (size_t)d * ldc + pos, (size_t)D * ldc, sp0, sp1);
    else part[w][lane] = sum_slots(pepart + pos, (size_t)ldc, sp0, sp1);
  }
  __syncthreads();
  if (w != 0 || c < 0) return;
  if (d < D) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < FIN_WAVES; ++i) s += (float)part[i][lane];
    const size_t idx = (size_t)d * ldc + c;
    ev.grad[idx] = s + ev.z[idx];
  } else {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < FIN_WAVES; ++i) s += part[i][lane];
    // every z load in flight at once (D <= 64), then the sums in coordinate order
    float zf[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) zf[k] = k < D ? ev.z[(size_t)k * ldc + c] : 0.0f;
    double zz = 0.0, wz = 0.0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      if (k < D) {
        const double z = zf[k];
        zz += z * z;
        if (wcol) wz += wcol[k] * z;
      }
    }
    ev.pe[c] = (float)(s + pe_shift + wz + 0.5 * zz + 0.9189385332046727 * D);
  }
}

// Launches over at most this many 128-chain tiles run the hand-interleaved form of the
// default kernel (NMX_X3_TAIL_GT: A/B override, 0 disables).
int x3_tail_tiles() {
  static const int v = [] {
    const char* e = getenv("NMX_X3_TAIL_GT");
    return e ? atoi(e) : 2;
  }();
  return v;
}

int check_ev(const nmx_eval_batch* ev) {
  if (!ev || !ev->z || !ev->grad || !ev->pe) return nmx_fail(NMX_ERR_INVALID, "eval batch has NULL pointers");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains || ev->ldc % 64)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  return NMX_OK;
}

// Kernel variant (A/B experiments).
//   36 (default) split-bf16 k_logreg_x3: split rings (A/B parts, 2 slots each, 50 KB ->
//      3 workgroups/CU), GEMM1 of tile k+1 issued beside the epilogue of tile k, Z pre-scaled
//      by -log2(e) (no multiply before v_exp).  30 = 2-slot ring, unpipelined; 31 = 3-slot;
//      32 = pipelined on one 3-slot ring; 33 = 36 without the pre-scale; 34/35 = 33 hand-
//      interleaved with sched_barrier at 3/2 workgroups per CU.  30-35 are bitwise equal.
//      C=4096 all-active, f32-equivalent TFLOP/s (scripts/logreg_variant_check.py, one box):
//      36: 180.9, 33: 178.1, 30: 175.0 (others 165-175); f32-MFMA 22: 116.5.
// f32-MFMA forms: 22 = k_logreg_rowlanes (117.2 TFLOP/s all-active, 75% of the f32 peak);
//   any other value < 30 = the generic tile kernel k_logreg_tiles (also the path for D != 55).
//   Earlier f32 experiments (shared stages + barrier, two chain tiles per wave, 5 workgroups
//   per CU, register-prefetch pipelines, epilogue forms) measured 97-117 TFLOP/s and were
//   removed; the numbers are in DESIGN.md.
int variant() {
  const char* e = getenv("NMX_LOGREG_VARIANT");
  return e ? atoi(e) : 36;
}

template <int KS>
void launch_rowlanes(const float* Xp, int64_t n_rows, int D, const nmx_eval_batch* ev, float* gpart, double* pepart,
                     hipStream_t s) {
  const int nstages = (int)(npad_of(n_rows) / RL_ROWS);
  const int S = num_splits(n_rows);
  const int Gt = ev->ldc / 32;
  constexpr int WBUF = RL_WAVES * ((32 * (2 * KS + 1) + 255) / 256 * 256);
  size_t lds = (size_t)WBUF * sizeof(float);
  const size_t red = (size_t)(RL_WAVES - 1) * 32 * 64 * sizeof(float) + (RL_WAVES - 1) * 64 * sizeof(double);
  if (lds < red) lds = red;
  hipLaunchKernelGGL((k_logreg_rowlanes<KS>), dim3(Gt * S), dim3(RL_WAVES * 64), lds, s, Xp, n_rows, nstages, D, S,
                     Gt, *ev, gpart, pepart);
}

template <int KS, bool EXACT>
void launch_tiles(const float* Xp, int64_t n_rows, int D, const nmx_eval_batch* ev, float* gpart,
                  double* pepart, hipStream_t s) {
  const int ntiles = (int)ntiles_of(n_rows);
  const int S = num_splits(n_rows);
  const int Gc = (ev->ldc + CPB - 1) / CPB;
  const size_t lds = (size_t)(BR * xs_of(D) + LDS_SLACK) * sizeof(float);
  hipLaunchKernelGGL((k_logreg_tiles<KS, EXACT>), dim3(Gc * S), dim3(NW * 64), lds, s, Xp, n_rows, ntiles, D,
                     S, Gc, *ev, gpart, pepart);
}

}  // namespace

extern "C" int nmx_logreg_num_splits(int64_t n_rows) { return num_splits(n_rows); }

// packed buffer: f32 rows | w[64] (k_logreg_colsums) | split-bf16 tiles (k_logreg_pack_x3)
inline size_t x3_offset(int64_t n_rows, int dim) {
  return (colterm_offset(n_rows, dim) + 64 * sizeof(double) + 255) / 256 * 256;
}

extern "C" size_t nmx_logreg_packed_bytes(int64_t n_rows, int dim) {
  if (n_rows <= 0 || dim <= 0) return 0;
  return x3_offset(n_rows, dim) + (size_t)x3_ntiles(n_rows) * x3_np(dim) * 1024;
}

extern "C" int nmx_logreg_pack(const float* X, const float* y, int64_t n_rows, int dim, void* packed,
                               void* stream) {
  if (!X || !y || !packed) return nmx_fail(NMX_ERR_INVALID, "logreg_pack: NULL pointer");
  if (n_rows <= 0 || dim <= 0 || dim > 64)
    return nmx_fail(NMX_ERR_INVALID, "logreg_pack: need n_rows > 0 and 0 < dim <= 64 (got %lld, %d)",
                    (long long)n_rows, dim);
  const int XS = xs_of(dim);
  const int64_t npad = npad_of(n_rows);
  const int64_t total = npad * XS;
  hipLaunchKernelGGL(k_logreg_pack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     X, y, n_rows, dim, XS, npad, (float*)packed);
  if (int st = nmx_check_launch("k_logreg_pack")) return st;
  hipLaunchKernelGGL(k_logreg_colsums, dim3(dim), dim3(CS_THREADS), 0, (hipStream_t)stream, X, y, n_rows, dim,
                     (double*)((char*)packed + colterm_offset(n_rows, dim)));
  if (int st = nmx_check_launch("k_logreg_colsums")) return st;
  const int64_t nt = x3_ntiles(n_rows);
  const int64_t nthreads = nt * x3_np(dim) * 64;
  hipLaunchKernelGGL(k_logreg_pack_x3, dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, X,
                     y, n_rows, dim, x3_kb(dim), x3_dt(dim), nt, (bf16x8*)((char*)packed + x3_offset(n_rows, dim)));
  return nmx_check_launch("k_logreg_pack_x3");
}

extern "C" size_t nmx_logreg_workspace_bytes(int64_t n_rows, int dim, int num_chains) {
  const size_t ldc = (size_t)(num_chains + 63) / 64 * 64;
  const size_t S = std::max(num_splits(n_rows), x3_num_splits(n_rows));
  const size_t g = S * dim * ldc * sizeof(float);
  const size_t p = S * ldc * sizeof(double);
  return (g + 255) / 256 * 256 + p;
}

extern "C" int nmx_logreg_pe_grad(const void* packed, int64_t n_rows, int dim, const nmx_eval_batch* ev,
                                  void* workspace, void* stream) {
  if (int st = check_ev(ev)) return st;
  if (!packed || !workspace) return nmx_fail(NMX_ERR_INVALID, "logreg_pe_grad: NULL packed/workspace");
  if (n_rows <= 0 || dim <= 0 || dim > 64)
    return nmx_fail(NMX_ERR_INVALID, "logreg_pe_grad: need 0 < dim <= 64 (got %d)", dim);
  hipStream_t s = (hipStream_t)stream;
  const int S = num_splits(n_rows);
  const size_t gbytes = (size_t)S * dim * ev->ldc * sizeof(float);
  float* gpart = (float*)workspace;
  double* pepart = (double*)((char*)workspace + (gbytes + 255) / 256 * 256);
  const float* Xp = (const float*)packed;
  const int KS = k_of(dim) / 2;
  const int var = variant();
  if (var >= 30 && var <= 36) {
    const int S2 = x3_num_splits(n_rows);
    pepart = (double*)((char*)workspace + ((size_t)S2 * dim * ev->ldc * sizeof(float) + 255) / 256 * 256);
    const int64_t nt = x3_ntiles(n_rows);
    const int KB = x3_kb(dim), DT = x3_dt(dim);
    const int ring = var == 30 ? 2 : 3;
    const size_t lds = var >= 33 ? (size_t)2 * x3_np(dim) * 1024 : (size_t)ring * x3_np(dim) * 1024;
    const char* Xq = (const char*)packed + x3_offset(n_rows, dim);
    // fixed grid: workgroups per XCD = 32 CUs x workgroups per CU (3 for the 2-slot ring)
    const int nb = std::min(ev->num_chains, ev->ldc);  // batch positions that can hold a chain
    const int Gt = (nb + 127) / 128;
    const dim3 grid(Gt * S2), blk(256);
#define NMX_X3(kb, dt)                                                                                           \
  if (var == 30) hipLaunchKernelGGL((k_logreg_x3<kb, dt, 2, 3, false>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart); \
  else if (var == 31) hipLaunchKernelGGL((k_logreg_x3<kb, dt, 3, 2, false>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart); \
  else if (var == 32) hipLaunchKernelGGL((k_logreg_x3<kb, dt, 3, 2, true>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart); \
  else if (var == 33) hipLaunchKernelGGL((k_logreg_x3<kb, dt, 4, 3, true>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart); \
  else if (var == 34) hipLaunchKernelGGL((k_logreg_x3<kb, dt, 4, 3, true, 6>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart); \
  else if (var == 35) hipLaunchKernelGGL((k_logreg_x3<kb, dt, 4, 2, true, 6>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart); \
  else hipLaunchKernelGGL((k_logreg_x3<kb, dt, 4, 3, true, 0, true>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart, pepart);
    if (KB == 4 && var == 36 && Gt <= x3_tail_tiles()) {
      // few chain tiles (one or two workgroups per CU, one wave per SIMD): GEMM1(k+1)'s
      // MFMAs hand-interleaved with tile k's epilogue rows -- the same arithmetic in the same
      // order as the default (bitwise equal), no other wave on the SIMD to fill the gaps
      hipLaunchKernelGGL((k_logreg_x3<4, 2, 4, 2, true, 6, true>), grid, blk, lds, s, Xq, nt, dim, S2, Gt, *ev, gpart,
                         pepart);
    } else if (KB == 4) { NMX_X3(4, 2) }
    else if (KB == 3) { NMX_X3(3, 2) }
    else if (KB == 2) { NMX_X3(2, 1) }
    else { NMX_X3(1, 1) }
#undef NMX_X3
    if (int st = nmx_check_launch("k_logreg_x3")) return st;
    const double* wcol = (const double*)((const char*)packed + colterm_offset(n_rows, dim));
    const double shift = -(double)(nt * X3_ROWS - n_rows) * 0.6931471805599453;
    hipLaunchKernelGGL(k_logreg_finalize, dim3((nb + 63) / 64, dim + 1), dim3(64 * FIN_WAVES), 0, s, gpart, pepart, S2, dim,
                       *ev, wcol, shift);
    return nmx_check_launch("k_logreg_finalize");
  }
  const bool epi_abs = KS == 28 && var == 22;  // w.b linear term (epilogue_abs)
  if (KS == 28 && var == 22) launch_rowlanes<28>(Xp, n_rows, dim, ev, gpart, pepart, s);  // covtype, D = 55
  else if (KS == 28) launch_tiles<28, true>(Xp, n_rows, dim, ev, gpart, pepart, s);
  else if (KS <= 4) launch_tiles<4, false>(Xp, n_rows, dim, ev, gpart, pepart, s);
  else if (KS <= 8) launch_tiles<8, false>(Xp, n_rows, dim, ev, gpart, pepart, s);
  else if (KS <= 16) launch_tiles<16, false>(Xp, n_rows, dim, ev, gpart, pepart, s);
  else launch_tiles<32, false>(Xp, n_rows, dim, ev, gpart, pepart, s);
  if (int st = nmx_check_launch("k_logreg_tiles")) return st;
  const double* wcol = epi_abs ? (const double*)((const char*)packed + colterm_offset(n_rows, dim)) : nullptr;
  hipLaunchKernelGGL(k_logreg_finalize, dim3(ev->ldc / 64, dim + 1), dim3(64 * FIN_WAVES), 0, s, gpart, pepart, S, dim, *ev,
                     wcol, 0.0);
  return nmx_check_launch("k_logreg_finalize");
}
