// Logistic-regression potential + gradient for thousands of chains (examples/covtype.py:66-71).
//
//   U(b)  = sum_n [max(l_n,0) + log1p(exp(-|l_n|)) - y_n l_n] + sum_d [b_d^2/2 + log(2pi)/2]
//   dU/db = X^T (sigmoid(l) - y) + b,      l = X b          
//
// k_logreg_x3: both GEMMs f32-accurate on the bf16 matrix cores (section "Split-bf16 kernel"
// below).  For a 32-row tile and 32 chains a wave computes L = X.Z, applies the Bernoulli
// epilogue to the accumulator registers in place and feeds them as the B operand of
// G += X^T.R: the 32x32 result holds chains on the lane and rows in the registers, which is the
// B-operand layout of the 32x32x16 bf16 form with the k order permuted -- no shuffle, no LDS
// round trip, and the N x C logit matrix never exists in memory.
//
// Packed X (nmx_logreg_pack): the float64 column terms w (k_logreg_colsums), then the
// split-bf16 tiles in MFMA-fragment order.
//
// Work split: grid = chain groups x S row splits.  S depends on n_rows only, and each split
// sums its rows in a fixed order, so a chain's U and dU do not depend on how many chains
// share the launch (GPU-count invariance).  Per-split partials go to slabs reduced in fixed
// order by k_logreg_finalize.  Workgroups of the same split are placed on one XCD
// (blockIdx % 8) so the chain groups share X tiles in L2.
//
// The f32-MFMA kernels that preceded this one (117 TFLOP/s all-active at best) and the
// split-bf16 schedule experiments are described, with their measurements, in DESIGN.md.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// w[d] = sum_n X[n,d] / 2 - sum_n y_n X[n,d] in float64: the per-chain linear part of U
// (max(l,0) - l y = (|l| + l)/2 - l y, so the rows only accumulate |l| and the chain adds
// w . b once).  One workgroup per column, fixed thread count and a fixed-order tree, so the
// value does not depend on anything but the data.
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

constexpr size_t COLTERM_BYTES = 64 * sizeof(double);  // w[64] at the start of the packed buffer
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// ---------------------------------------------------------------------------------------
// Split-bf16 kernel: f32-accurate products on the bf16 matrix cores.
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
// Workgroup = 4 waves = 4 chain tiles of 32 sharing each X tile; X tiles stream through split
// LDS rings by buffer LDS-DMA, one workgroup barrier per tile.  Grid = chain groups x S row
// splits, S a function of n_rows only (fixed summation order); the partials go through slabs
// and the fixed-order finalize.
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// One 32x32x16 bf16 product (the 16x16x32 shape's clock / issue trade was measured in round 4 by
// a timing probe, DESIGN.md "headline kernel clock"; the probe is not in the product sources).
template <int S = 0>
__device__ __forceinline__ f32x16 x3_mma(const bf16x8& a, const bf16x8& b, f32x16 acc) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}

// VALU instructions the scheduling hints place after each GEMM1(k+1) / GEMM2(k) MFMA (x3_item)
#ifndef NMX_X3_VALU1
#define NMX_X3_VALU1 5
#endif
#ifndef NMX_X3_VALU2
#define NMX_X3_VALU2 3
#endif

constexpr int X3_ROWS = 32;
constexpr int X3_MAX_S = 256;

inline int x3_kb(int D) { return (D + 15) / 16; }
inline int x3_dt(int D) { return (D + 31) / 32; }
// Combined last k-block (H = 1: KB = 4 and D % 16 in 1..8, the covtype D = 55): the last
// k-block has at most 8 real columns, so two products fit one 16-deep MFMA (columns in the
// k-slots 0..7 of one term, 8..15 of the other) and its six split products run as three MFMAs
// on two extra pieces behind the A pieces (x3_gemm1): 45 instead of 48 MFMAs per tile.
inline int x3_h(int D) {
  const int r = D % 16;
  return (x3_kb(D) == 4 && r != 0 && r <= 8) ? 1 : 0;
}
inline int x3_np(int D) { return 3 * x3_kb(D) + 2 * x3_h(D) + 6 * x3_dt(D) + 1; }
inline int64_t x3_ntiles(int64_t n) { return (n + X3_ROWS - 1) / X3_ROWS; }

int x3_num_splits(int64_t n_rows) {
  int64_t s = x3_ntiles(n_rows) / 16;
  s = s / 8 * 8;
  if (s < 8) s = 8;
  if (s > X3_MAX_S) s = X3_MAX_S;
  return (int)s;
}

// three-term bf16 split of 8 floats (round to nearest even at every step), one pair of values
// per conversion: v_cvt_pk_bf16_f32 rounds both, and the f32 values of the two terms come
// back from the packed word by a shift (low half) and a mask (high half).  Per-value
// conversions made the compiler convert each value a second time for its f32 image (7 instead
// of 3 conversions per pair, 56 instead of 24 per tile in the GEMM2 residual split).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ float pk_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float pk_hi(unsigned u) { return __uint_as_float(u & 0xFFFF0000u); }
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& b1, bf16x8& b2, bf16x8& b3) {
  u32x4 w1, w2, w3;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float x0 = v[2 * p], x1 = v[2 * p + 1];
    const unsigned u1 = pk_bf16(x0, x1);
    const float e0 = x0 - pk_lo(u1), e1 = x1 - pk_hi(u1);
    const unsigned u2 = pk_bf16(e0, e1);
    const float f0 = e0 - pk_lo(u2), f1 = e1 - pk_hi(u2);
    w1[p] = u1;
    w2[p] = u2;
    w3[p] = pk_bf16(f0, f1);
  }
  b1 = __builtin_bit_cast(bf16x8, w1);
  b2 = __builtin_bit_cast(bf16x8, w2);
  b3 = __builtin_bit_cast(bf16x8, w3);
}

// one thread per (tile, piece, lane): 16 bytes of one operand fragment
__global__ void k_logreg_pack_x3(const float* __restrict__ X, const float* __restrict__ y, int64_t n, int D,
                                 int KB, int DT, int H, int64_t ntiles, bf16x8* __restrict__ out) {
  const int NP = 3 * KB + 2 * H + 6 * DT + 1;
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
  } else if (piece < 3 * KB + 2 * H) {
    // combined pieces of the last k-block: every lane holds its columns 16 (KB - 1) + j; piece
    // 3 KB: terms 1 (h = 0) and 2 (h = 1), piece 3 KB + 1: terms 3 (h = 0) and 1 (h = 1)
    const int cp = piece - 3 * KB;
    plane = cp == 0 ? h : (h == 0 ? 2 : 0);
    const int64_t row = r0 + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 16 * (KB - 1) + j;
      v[j] = (row < n && d < D) ? X[row * D + d] : 0.0f;
    }
  } else if (piece < NP - 1) {
    const int qq = piece - 3 * KB - 2 * H;
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
    // labels as y - 1/2 (x3_epi_pair): lane L < 8 holds row labels [h = L/4][i = 4 (L%4) .. +3]
    // (bytes 16 L .. 16 L + 15); padded rows 0 (their X is zero)
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (lane < 8) {
      const int hh = lane >> 2;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ii = 4 * (lane & 3) + k;
        const int64_t row = r0 + (ii & 3) + 8 * (ii >> 2) + 4 * hh;
        f[k] = row < n ? y[row] - 0.5f : 0.0f;
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

// A-piece (plane p, k-block kb) and combined-piece (c) positions in an LDS ring slot: the tile
// image in HBM order, or (COMPACT, the main kernel with H = 1) the slot without the last
// k-block's plane pieces, which only the transposed GEMM2 reads of the TR / tail forms need
template <int KB, bool COMPACT>
__device__ constexpr int x3_ai(int p, int kb) { return COMPACT ? p * (KB - 1) + kb : p * KB + kb; }
template <int KB, bool COMPACT>
__device__ constexpr int x3_ci(int c) { return COMPACT ? 3 * (KB - 1) + c : 3 * KB + c; }

// GEMM1 of one tile: L = X . Z (32 rows x 32 chains), six split products per k-block; with H
// the last k-block's six as three MFMAs on the combined pieces (columns in k-slots 0..7 of
// one term and 8..15 of the other; x3_load_z builds the matching Z fragments):
//   (a3 | a1) . (z1 | z3) = a3 z1 + a1 z3,  (a1 | a2) . (z2 | z1) = a1 z2 + a2 z1,
//   (a1 | a2) . (z1 | z2) = a1 z1 + a2 z2
template <int KB, int H, bool COMPACT = false>
__device__ __forceinline__ f32x16 x3_gemm1(const bf16x8* fr, const bf16x8 (&z1)[KB], const bf16x8 (&z2)[KB],
                                           const bf16x8 (&z3)[KB]) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
  for (int kb = 0; kb < KB - H; ++kb) {
    const bf16x8 a1 = fr[x3_ai<KB, COMPACT>(0, kb) * 64], a2 = fr[x3_ai<KB, COMPACT>(1, kb) * 64],
                 a3 = fr[x3_ai<KB, COMPACT>(2, kb) * 64];
    acc = x3_mma<0>(a3, z1[kb], acc);
    acc = x3_mma<1>(a2, z2[kb], acc);
    acc = x3_mma<0>(a1, z3[kb], acc);
    acc = x3_mma<1>(a2, z1[kb], acc);
    acc = x3_mma<0>(a1, z2[kb], acc);
    acc = x3_mma<1>(a1, z1[kb], acc);
  }
  if constexpr (H) {
    const bf16x8 c0 = fr[x3_ci<KB, COMPACT>(0) * 64], c1 = fr[x3_ci<KB, COMPACT>(1) * 64];
    acc = x3_mma<0>(c1, z3[KB - 1], acc);
    acc = x3_mma<1>(c0, z2[KB - 1], acc);
    acc = x3_mma<0>(c0, z1[KB - 1], acc);
  }
  return acc;
}

// Z fragments of a chain tile (B operand: lane (n, h) holds Z[16 kb + 8 h + j][chain n]),
// pre-scaled by -log2(e) and split.  Through a buffer descriptor: coordinates >= D and inactive
// lanes (c = -1) fall outside its range and read 0.  With H the last k-block's lanes all hold
// columns 16 (KB - 1) + j, as (z1 | z2), (z2 | z1), (z1 | z3) for x3_gemm1's combined products.
template <int KB, int H>
__device__ __forceinline__ void x3_load_z(const __amdgpu_buffer_rsrc_t zrs, int c, int h, int ldc, bf16x8 (&z1)[KB],
                                          bf16x8 (&z2)[KB], bf16x8 (&z3)[KB]) {
  const unsigned zoff = c >= 0 ? (unsigned)((8 * h * ldc + c) * 4) : 0xFFFFFFF0u;
  const unsigned zoff0 = c >= 0 ? (unsigned)(c * 4) : 0xFFFFFFF0u;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const bool comb = H && kb == KB - 1;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(zrs, comb ? zoff0 : zoff, (16 * kb + j) * ldc * 4, 0));
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= -LOG2E;
    bf16x8 t1, t2, t3;
    split3(v, t1, t2, t3);
    if (comb) {
      z1[kb] = h ? t2 : t1;
      z2[kb] = h ? t1 : t2;
      z3[kb] = h ? t3 : t1;
    } else {
      z1[kb] = t1;
      z2[kb] = t2;
      z3[kb] = t3;
    }
  }
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

// Bernoulli-logits epilogue on the GEMM1 accumulator, rows 2p and 2p+1 (no row mask: padded
// rows have l = 0 and zero X).  The accumulator holds m = -l log2(e) (Z pre-scaled by -log2 e
// before its split), so e = 2^-|m| needs no multiply and sum |l| = ln 2 sum |m|.
//   U terms:   |l|/2 + log1p(e)   (the linear part (1/2 - y) l is the per-chain w . b of the
//              finalize), log1p summed as log of the product of the factors 1 + e
//   residual:  R' = y - sigmoid(l) = (y - 1/2) + copysign(1/(1+e) - 1/2, m)
//              (sigmoid(l) - 1/2 = copysign(1/(1+e) - 1/2, l), sign(l) = -sign(m)); GEMM2
//              accumulates X^T R' = -X^T (sigmoid(l) - y) and the finalize subtracts it.
// Labels come as y - 1/2.  Per value: exp and rcp, one add (1 + e), one mul (product), one
// add (- 1/2), one bitfield insert (copysign), one add (+ label), one add (|m|); the even and
// odd rows keep separate products (each <= 2^8).  All scalar VALU: packed f32 (v_pk_*_f32)
// beside MFMAs costs extra issue cycles per pair on gfx950 (MI355X_MICROARCH.md, VALU/MFMA
// co-issue), so this file is also compiled without the SLP vectorizer (build.py FILE_FLAGS).
__device__ __forceinline__ void x3_epi_one(float m, float yh, float& res, float& lin, float& prod) {
  const float e = __builtin_amdgcn_exp2f(-fabsf(m));
  const float ope = e + 1.0f;
  prod = prod * ope;
  const float hh = __builtin_amdgcn_rcpf(ope) - 0.5f;
  constexpr unsigned SB = 0x80000000u;
  const float sg = __uint_as_float((__float_as_uint(m) & SB) | (__float_as_uint(hh) & ~SB));
  res = sg + yh;
  lin += fabsf(m);
}

__device__ __forceinline__ void x3_epi_pair(const f32x16& acc, const f32x4 (&yh4)[4], int p, float (&res)[16],
                                            float& lin, float (&prod)[2]) {
  const int r0 = 2 * p, r1 = 2 * p + 1;
  x3_epi_one(acc[r0], yh4[r0 >> 2][r0 & 3], res[r0], lin, prod[0]);
  x3_epi_one(acc[r1], yh4[r1 >> 2][r1 & 3], res[r1], lin, prod[1]);
}

// a tile's U term (per lane, double); x3_epi_finish adds it to the running sum
__device__ __forceinline__ double x3_epi_term(float lin, const float (&prod)[2]) {
  return (double)(0.5f * lin) * (double)LN2 + (double)__builtin_amdgcn_logf(prod[0] * prod[1]) * (double)LN2;
}
__device__ __forceinline__ void x3_epi_finish(float lin, const float (&prod)[2], double& pe) {
  pe += x3_epi_term(lin, prod);
}

__device__ __forceinline__ void x3_epilogue(const f32x16& acc, const f32x4 (&yh4)[4], float (&res)[16], double& pe) {
  float lin = 0.0f;
  float prod[2] = {1.0f, 1.0f};
#pragma unroll
  for (int p = 0; p < 8; ++p) x3_epi_pair(acc, yh4, p, res, lin, prod);
  x3_epi_finish(lin, prod, pe);
}

// GEMM2 of one tile: G += X^T . R, R split into three bf16 terms (k-step s = registers 8s..8s+7);
// G2 = the first GEMM2 piece (3 KB + 2 H)
template <int G2, int DT>
__device__ __forceinline__ void x3_gemm2(const bf16x8* fr, const float (&res)[16], f32x16 (&g)[DT]) {
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
      g[dt] = x3_mma<1>(b3, r1, g[dt]);
      g[dt] = x3_mma<0>(b2, r2, g[dt]);
      g[dt] = x3_mma<1>(b1, r3, g[dt]);
      g[dt] = x3_mma<0>(b2, r1, g[dt]);
      g[dt] = x3_mma<1>(b1, r2, g[dt]);
      g[dt] = x3_mma<0>(b1, r1, g[dt]);
    }
  }
}

// GEMM2's X^T operand of a tile taken from its GEMM1 image (the A pieces: lane r + 32 h of piece
// (plane, kb) holds X[r][16 kb + 8 h .. + 7]) with gfx950's transposed LDS read
// ds_read_b64_tr_b16 (cdna_hip_programming.md T10: lane 4q + p of a 16-lane group supplies the
// address of row q, columns 4p .. 4p + 3 of a 4 x 16 block; lane i receives column i), so the
// B pieces (X^T in fragment order, the other half of the packed tile) need not be streamed.
// Fragment (plane, dt, s) of lane L = (d = L & 31, h = L >> 5) is X[16 s + 8 jh + 4 h + q][32 dt +
// d] for j = 4 jh + q: exactly the B piece's bytes, so the products are bitwise the same.
// The reads are inline asm (a compiler-visible LDS read after the ring's DMA issue gets a
// vmcnt(0) wait that would drain the prefetch, as for x3_labels); x3_tr_wait before use.
//
// COMPACT (the tail form with H): the slot holds the A part without the last k-block's plane
// pieces (x3_ai / x3_ci COMPACT positions), whose columns 48..55 the combined pieces carry:
// piece c0 = (plane 0 | plane 1) in lane halves h = 0 | 1, c1 = (plane 2 | plane 0).  The last
// k-block's reads (lane bit g1 of dt = DT - 1) take plane 0 and 2 from the h = 0 halves of c0 /
// c1 and plane 1 from the h = 1 half of c0 (32 lanes = 512 bytes further).  Those reads'
// columns 56..63 (zero in the plane pieces) then read the neighbouring half instead: they only
// feed GEMM2 output rows >= 56 > D, which are never stored.  Columns < D read the same bytes.
template <int KB, int DT, bool COMPACT, int DTI>
__device__ __forceinline__ void x3_tr_load_dt(const char* aslot, bf16x8 (&fb)[3][2]) {
  static_assert(KB >= 2 * DT, "the GEMM1 image must cover GEMM2's 32 DT columns");
  static_assert(!COMPACT || KB == 2 * DT, "compact slot: the last k-block is GEMM2's last column half");
  const int L = threadIdx.x & 63;
  const int p = L & 3, q = (L >> 2) & 3, g1 = (L >> 4) & 1, h = L >> 5;
  const unsigned base0 = (unsigned)(size_t)((__attribute__((address_space(3))) const char*)aslot) +
                         (q + 32 * (p >> 1) + 4 * h) * 16 + 8 * (p & 1);
#pragma unroll
  for (int plane = 0; plane < 3; ++plane) {
    // byte offsets of the k-blocks 2 dt (g1 = 0) and 2 dt + 1 (g1 = 1) in the slot
    constexpr int dt = DTI, kb0 = 2 * dt, kb1 = 2 * dt + 1;
    int o0, o1;
    if constexpr (COMPACT) {
      o0 = x3_ai<KB, true>(plane, kb0) * 1024;
      o1 = kb1 < KB - 1 ? x3_ai<KB, true>(plane, kb1) * 1024
                        : (plane == 2 ? x3_ci<KB, true>(1) * 1024 : x3_ci<KB, true>(0) * 1024 + (plane == 1 ? 512 : 0));
    } else {
      o0 = (plane * KB + kb0) * 1024;
      o1 = (plane * KB + kb1) * 1024;
    }
    const unsigned base = base0 + (g1 ? o1 : o0);
#pragma unroll
    for (int sidx = 0; sidx < 2; ++sidx) {
      typedef short s4 __attribute__((ext_vector_type(4)));
      s4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
                   : "=&v"(lo), "=&v"(hi)
                   : "v"(base), "i"((16 * sidx) * 16), "i"((16 * sidx + 8) * 16));
      const s4 lh[2] = {lo, hi};
      bf16x8 f;
      __builtin_memcpy(&f, lh, 16);
      fb[plane][sidx] = f;
    }
  }
}
template <int KB, int DT, bool COMPACT = false>
__device__ __forceinline__ void x3_gemm2_tr_load(const char* aslot, bf16x8 (&fb)[3][DT][2]) {
  bf16x8 f0[3][2];
  x3_tr_load_dt<KB, DT, COMPACT, 0>(aslot, f0);
#pragma unroll
  for (int plane = 0; plane < 3; ++plane)
#pragma unroll
    for (int sidx = 0; sidx < 2; ++sidx) fb[plane][0][sidx] = f0[plane][sidx];
  if constexpr (DT > 1) {
    bf16x8 f1[3][2];
    x3_tr_load_dt<KB, DT, COMPACT, (DT > 1 ? 1 : 0)>(aslot, f1);
#pragma unroll
    for (int plane = 0; plane < 3; ++plane)
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx) fb[plane][1][sidx] = f1[plane][sidx];
  }
  static_assert(DT <= 2, "x3_gemm2_tr_load: DT <= 2");
}
template <int DT>
__device__ __forceinline__ void x3_tr_wait(bf16x8 (&fb)[3][DT][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int plane = 0; plane < 3; ++plane)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx) asm volatile("" : "+v"(fb[plane][dt][sidx]));
}
// x3_gemm2 with the operands read just in time (three fragments per (s, dt), 12 VGPRs instead
// of 48 held across GEMM1: the main kernel's register budget)
template <int KB, int DT>
__device__ __forceinline__ void x3_gemm2_tr(const char* aslot, const float (&res)[16], f32x16 (&g)[DT]) {
  static_assert(KB >= 2 * DT, "the GEMM1 image must cover GEMM2's 32 DT columns");
  const int L = threadIdx.x & 63;
  const int p = L & 3, q = (L >> 2) & 3, g1 = (L >> 4) & 1, h = L >> 5;
  const unsigned base = (unsigned)(size_t)((__attribute__((address_space(3))) const char*)aslot) + g1 * 1024 +
                        (q + 32 * (p >> 1) + 4 * h) * 16 + 8 * (p & 1);
#pragma unroll
  for (int sidx = 0; sidx < 2; ++sidx) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = res[8 * sidx + j];
    bf16x8 r1, r2, r3;
    split3(v, r1, r2, r3);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      typedef short s4 __attribute__((ext_vector_type(4)));
      s4 t[6];
      asm volatile(
          "ds_read_b64_tr_b16 %0, %6 offset:%7\n\tds_read_b64_tr_b16 %1, %6 offset:%8\n\t"
          "ds_read_b64_tr_b16 %2, %6 offset:%9\n\tds_read_b64_tr_b16 %3, %6 offset:%10\n\t"
          "ds_read_b64_tr_b16 %4, %6 offset:%11\n\tds_read_b64_tr_b16 %5, %6 offset:%12\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5])
          : "v"(base), "i"((0 * KB + 2 * dt) * 1024 + 16 * sidx * 16), "i"((0 * KB + 2 * dt) * 1024 + (16 * sidx + 8) * 16),
            "i"((1 * KB + 2 * dt) * 1024 + 16 * sidx * 16), "i"((1 * KB + 2 * dt) * 1024 + (16 * sidx + 8) * 16),
            "i"((2 * KB + 2 * dt) * 1024 + 16 * sidx * 16), "i"((2 * KB + 2 * dt) * 1024 + (16 * sidx + 8) * 16));
      bf16x8 b1, b2, b3;
      __builtin_memcpy(&b1, &t[0], 16);
      __builtin_memcpy(&b2, &t[2], 16);
      __builtin_memcpy(&b3, &t[4], 16);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b3, r1, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r2, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r3, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r1, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r2, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r1, g[dt], 0, 0, 0);
    }
  }
}

// x3_gemm2 on register operands (same products in the same order)
template <int DT>
__device__ __forceinline__ void x3_gemm2_regs(const bf16x8 (&fb)[3][DT][2], const float (&res)[16],
                                              f32x16 (&g)[DT]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = res[8 * s + j];
    bf16x8 r1, r2, r3;
    split3(v, r1, r2, r3);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const bf16x8 b1 = fb[0][dt][s], b2 = fb[1][dt][s], b3 = fb[2][dt][s];
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b3, r1, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r2, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r3, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r1, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r2, g[dt], 0, 0, 0);
      g[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r1, g[dt], 0, 0, 0);
    }
  }
}

// Software-pipelined: GEMM1 of tile k+1 is issued beside the epilogue of tile k (they are
// independent), then GEMM2 of tile k.  SCHED 0 adds the igrouplp placement hints below.
//
#ifndef NMX_X3_TR
#define NMX_X3_TR 0
#endif
// the main kernel's GEMM2 operand from transposed reads of the GEMM1 image (needs KB >= 2 DT)
template <int KB, int DT>
constexpr bool x3_tr() { return NMX_X3_TR && KB >= 2 * DT; }
// A pieces of a main-kernel LDS A slot: without the last k-block's plane pieces when the
// combined pieces replace them (H) and GEMM2 does not read the slot (not TR)
template <int KB, int DT, int H>
constexpr int x3_nal() { return (H && !x3_tr<KB, DT>()) ? 3 * (KB - 1) + 2 : 3 * KB + 2 * H; }
template <int KB, int DT, int H>
inline size_t x3_lds_bytes() {
  constexpr int NA = 3 * KB + 2 * H, NP = NA + 6 * DT + 1;
  return x3_tr<KB, DT>() ? (size_t)(3 * NA + 2) * 1024 : (size_t)2 * (x3_nal<KB, DT, H>() + NP - NA) * 1024;
}


template <int KB, int DT, int H, int SCHED>
__device__ __forceinline__ void x3_item(const char* __restrict__ Xq, int64_t ntiles, int D, int S, int split, int ct,
                                        nmx_eval_batch ev, float* __restrict__ gpart,
                                        double* __restrict__ pepart) {
  constexpr int NP = 3 * KB + 2 * H + 6 * DT + 1;
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
  NMX_DCHECK(split < S && t1 <= ntiles && nt >= 0);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Xq + (size_t)t0 * NP * 1024), 0, (int)((size_t)nt * NP * 1024), 0x00020000);

  // Z through a buffer descriptor (no per-element conditions: conditions and 64-bit addresses
  // hoisted out of the item loop spilled)
  const __amdgpu_buffer_rsrc_t zrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)ev.z, 0, D * ldc * 4, 0x00020000);
  bf16x8 z1[KB], z2[KB], z3[KB];
  x3_load_z<KB, H>(zrs, c, h, ldc, z1, z2, z3);
  f32x16 g[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) g[dt][r] = 0.0f;
  double pe = 0.0;

  {
    // Split rings: GEMM1 reads only the A part of a tile (pieces < 3 KB), GEMM2 and the labels
    // only the B part.  Iteration k reads A(k+1) and B(k) while A(k+2) and B(k+1) fill, so two
    // slots of each part suffice: 2 x (12 + 13) KB for covtype, three workgroups per CU.
    // TR (x3_tr<KB, DT>()): GEMM2 reads X^T from the GEMM1 image by transposed LDS reads, so
    // only the A pieces and the labels are streamed (half the bytes); the A ring then keeps
    // tile k for GEMM2(k) beside tile k+1 (GEMM1) and tile k+2 landing: 3 slots, and B slots
    // hold the label piece only (3 x 12 + 2 x 1 KB)
    // With H the A part also holds the two combined pieces; the non-TR slot skips the last
    // k-block's plane pieces (NAL = 11 of 14 for covtype, x3_ai / x3_ci COMPACT positions).
    constexpr int NA = 3 * KB + 2 * H, NBP = NP - NA;
    constexpr bool TR = x3_tr<KB, DT>();
    constexpr int NAL = x3_nal<KB, DT, H>();
    constexpr bool CMP = NAL != NA;
    constexpr int ASL = TR ? 3 : 2, BSZ = TR ? 1 : NBP;
    char* aring = lds;
    char* bring = lds + ASL * NAL * 1024;
    auto issue_a = [&](int k) {
      char* dst = aring + (k % ASL) * NAL * 1024;
#pragma unroll
      for (int j = 0; j < (NAL + 3) / 4; ++j) {
        const int il = wu + 4 * j;  // slot position; i = the tile's piece
        const int i = !CMP ? il
                           : (il < 3 * (KB - 1) ? (il / (KB - 1)) * KB + il % (KB - 1) : 3 * KB + (il - 3 * (KB - 1)));
        if (il < NAL)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + il * 1024), 16,
                                                   lane * 16, (unsigned)((k * NP + i) * 1024), 0, 0);
      }
    };
    auto issue_b = [&](int k) {
      char* dst = bring + (k & 1) * BSZ * 1024;
      if constexpr (TR) {
        if (wu == 3)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)dst, 16, lane * 16,
                                                   (unsigned)((k * NP + NP - 1) * 1024), 0, 0);
      } else {
#pragma unroll
        for (int j = 0; j < (NBP + 3) / 4; ++j) {
          const int i = wu + 4 * j;
          if (i < NBP)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + i * 1024),
                                                     16, lane * 16, (unsigned)((k * NP + NA + i) * 1024), 0, 0);
        }
      }
    };
    if (nt > 0) {
      issue_a(0);
      x3_wait_vm<0>();
      asm volatile("s_barrier" ::: "memory");  // A(0) is in
      if (nt > 1) issue_a(1);
      issue_b(0);
      f32x16 accA, accB;
      if (active) accA = x3_gemm1<KB, H, CMP>(reinterpret_cast<const bf16x8*>(aring) + lane, z1, z2, z3);
      // one tile: epilogue + GEMM2 of tile k on `acc`, GEMM1 of tile k+1 into `nxt`; the loop
      // below alternates the two accumulators (no register copy between tiles)
      auto step = [&](int k, const f32x16& acc, f32x16& nxt) {
        // A(k+1) and B(k) have landed in every wave; A slot k&1 (GEMM1(k)) and B slot
        // (k+1)&1 (GEMM2(k-1)) were last read in iteration k-1
        x3_wait_vm<0>();
        asm volatile("s_barrier" ::: "memory");
        if (k + 2 < nt) issue_a(k + 2);
        if (k + 1 < nt) issue_b(k + 1);
        if (!active) return;
        const char* bs = bring + (k & 1) * BSZ * 1024;
        f32x4 y4[4];
        x3_labels(bs + (BSZ - 1) * 1024, h, y4);
        x3_labels_wait(y4);
        // GEMM1 of tile k+1 (a stale slot past the last tile: computed, never used) beside
        // the epilogue of tile k
        const bf16x8* fa = reinterpret_cast<const bf16x8*>(aring + ((k + 1) % ASL) * NAL * 1024) + lane;
        float res[16];
        nxt = x3_gemm1<KB, H, CMP>(fa, z1, z2, z3);
        x3_epilogue(acc, y4, res, pe);
        if constexpr (TR) x3_gemm2_tr<KB, DT>(aring + (k % ASL) * NAL * 1024, res, g);
        else x3_gemm2<NA, DT>(reinterpret_cast<const bf16x8*>(bs) - NA * 64 + lane, res, g);
        if constexpr (SCHED == 0) {
          // scheduling hints (LLVM igrouplp): each GEMM1(k+1) MFMA followed by 5 VALU (tile k's
          // epilogue and the first split half), each GEMM2(k) MFMA by 3 (the second split half),
          // so one wave's MFMA dependency stalls are filled with its own vector work.  Measured
          // (scripts/ab_logreg.py, C = 4096 all active): 2.74 vs 2.85 ms without the hints; 4-7
          // and 1-3 VALU per group all within 1.5%.
#pragma unroll
          for (int i = 0; i < 6 * KB - 3 * H; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);            // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, NMX_X3_VALU1, 0);  // VALU
          }
#pragma unroll
          for (int i = 0; i < 12 * DT; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, NMX_X3_VALU2, 0);
          }
        }
      };
      for (int k = 0; k < nt; k += 2) {
        step(k, accA, accB);
        if (k + 1 < nt) step(k + 1, accB, accA);
      }
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
template <int KB, int DT, int H, int MINB, int SCHED>
__global__ __launch_bounds__(256, MINB) void k_logreg_x3(const char* __restrict__ Xq, int64_t ntiles, int D, int S,
                                                     int Gt, nmx_eval_batch ev, float* __restrict__ gpart,
                                                     double* __restrict__ pepart) {
  const int b = blockIdx.x;
  const int qb = b >> 3;
  const int ct = qb % Gt;
  const int npos = ev.active_idx ? *ev.active_count : ev.ldc;
  if (ct * 128 >= npos) return;
  x3_item<KB, DT, H, SCHED>(Xq, ntiles, D, S, (qb / Gt) * 8 + (b & 7), ct, ev, gpart, pepart);
}

// ---------------------------------------------------------------------------------------
// Tail form with split roles (launches over <= X3_TAIL_TILES chain groups).  In a NUTS run's
// tail one wave per chain tile and split ran the dependent GEMM1 -> epilogue -> split ->
// GEMM2 chain of each of its tiles alone on its SIMD (~2.9k cycles a tile for 1.5k of MFMA
// work).  Here a workgroup of 8 waves pairs every chain tile t with two waves on different
// SIMDs: wave t (role A) runs GEMM1 of tile k+1 beside the epilogue of tile k (the
// hand-interleaved order below) and hands the residual R(k) to its role-B wave (on another
// SIMD) through LDS; B splits it and runs GEMM2(k) one tile behind.  Every product, its operands and
// its accumulation order are those of x3_item (bitwise equal results; the residual crosses
// LDS as an exact f32 copy).  LDS: the A ring (2 slots) as before, a 3-slot B ring (B still
// reads tile k-1 while tile k+1 lands), two residual slots per chain tile.  One workgroup per
// CU in these launches.
__device__ __forceinline__ void x3_res_store(char* base, const float (&res)[16]) {
  const unsigned a = (unsigned)(size_t)((__attribute__((address_space(3))) char*)base);
  const f32x4 v0 = {res[0], res[1], res[2], res[3]}, v1 = {res[4], res[5], res[6], res[7]};
  const f32x4 v2 = {res[8], res[9], res[10], res[11]}, v3 = {res[12], res[13], res[14], res[15]};
  asm volatile(
      "ds_write_b128 %0, %1\n\t"
      "ds_write_b128 %0, %2 offset:1024\n\t"
      "ds_write_b128 %0, %3 offset:2048\n\t"
      "ds_write_b128 %0, %4 offset:3072" ::"v"(a), "v"(v0), "v"(v1), "v"(v2), "v"(v3)
      : "memory");
}
__device__ __forceinline__ void x3_res_load(const char* base, float (&res)[16]) {
  const unsigned a = (unsigned)(size_t)((__attribute__((address_space(3))) const char*)base);
  f32x4 v[4];
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:1024\n\t"
      "ds_read_b128 %2, %4 offset:2048\n\t"
      "ds_read_b128 %3, %4 offset:3072\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(a)
      : "memory");
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) res[4 * q + j] = v[q][j];
}

// workgroup barrier after this wave's LDS-DMA loads and LDS writes have completed
__device__ __forceinline__ void x3_roles_barrier() {
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (0 << 8) | (0 << 14));  // vmcnt(0) lgkmcnt(0)
  asm volatile("s_barrier" ::: "memory");
}
// the same with up to N of this wave's youngest LDS-DMA loads still in flight (the prefetch of
// later tiles), its LDS writes complete
template <int N>
__device__ __forceinline__ void x3_roles_barrier_n() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (0 << 8) | ((N >> 4) << 14));
  asm volatile("s_barrier" ::: "memory");
}
__device__ __forceinline__ void x3_roles_barrier_rt(int n) {  // n wave-uniform
  switch (n) {
    case 0: x3_roles_barrier_n<0>(); break;
    case 1: x3_roles_barrier_n<1>(); break;
    case 2: x3_roles_barrier_n<2>(); break;
    case 3: x3_roles_barrier_n<3>(); break;
    case 4: x3_roles_barrier_n<4>(); break;
    case 5: x3_roles_barrier_n<5>(); break;
    case 6: x3_roles_barrier_n<6>(); break;
    case 7: x3_roles_barrier_n<7>(); break;
    case 8: x3_roles_barrier_n<8>(); break;
    case 9: x3_roles_barrier_n<9>(); break;
    case 10: x3_roles_barrier_n<10>(); break;
    case 11: x3_roles_barrier_n<11>(); break;
    default: x3_roles_barrier_n<12>(); break;  // (n > 12: waits for more than needed)
  }
}

// Role A's tile: GEMM1 of the next tile (fa, into nxt) hand-interleaved with the epilogue of
// the current one (acc -> res, lin, prod)
template <int KB, int H, bool CMP>
__device__ __forceinline__ void x3_a_tile(const bf16x8* fa, const bf16x8 (&z1)[KB], const bf16x8 (&z2)[KB],
                                          const bf16x8 (&z3)[KB], const f32x16& acc, const f32x4 (&y4)[4],
                                          f32x16& nxt, float (&res)[16], float& lin, float (&prod)[2]) {
  // hand-interleaved (in-order issue within a wave): GEMM1(k+1)'s MFMAs alternate with row
  // pairs of tile k's epilogue; sched_barrier(0) pins the order; the operations and their
  // per-value order equal x3_gemm1 / x3_epilogue (bitwise equal results)
#pragma unroll
  for (int r = 0; r < 16; ++r) nxt[r] = 0.0f;
  bf16x8 a1 = fa[x3_ai<KB, CMP>(0, 0) * 64], a2 = fa[x3_ai<KB, CMP>(1, 0) * 64],
         a3 = fa[x3_ai<KB, CMP>(2, 0) * 64];
#pragma unroll
  for (int kb = 0; kb < KB - H; ++kb) {
    bf16x8 n1, n2, n3;
    if (kb + 1 < KB - H) {
      n1 = fa[x3_ai<KB, CMP>(0, kb + 1) * 64];
      n2 = fa[x3_ai<KB, CMP>(1, kb + 1) * 64];
      n3 = fa[x3_ai<KB, CMP>(2, kb + 1) * 64];
    } else if (H && kb + 1 == KB - 1) {  // the combined pieces (a1 | a2), (a3 | a1)
      n1 = fa[x3_ci<KB, CMP>(0) * 64];
      n2 = fa[x3_ci<KB, CMP>(1) * 64];
    }
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, z1[kb], nxt, 0, 0, 0);
    x3_epi_pair(acc, y4, 2 * kb, res, lin, prod);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z2[kb], nxt, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z3[kb], nxt, 0, 0, 0);
    x3_epi_pair(acc, y4, 2 * kb + 1, res, lin, prod);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z1[kb], nxt, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z2[kb], nxt, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z1[kb], nxt, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (kb + 1 < KB - H) {
      a1 = n1;
      a2 = n2;
      a3 = n3;
    } else if (H && kb + 1 == KB - 1) {
      a1 = n1;
      a2 = n2;
    }
  }
  if constexpr (H) {  // x3_gemm1's combined products (a1 = (a1 | a2), a2 = (a3 | a1) here)
    constexpr int kb = KB - 1;
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, z3[kb], nxt, 0, 0, 0);
    x3_epi_pair(acc, y4, 2 * kb, res, lin, prod);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z2[kb], nxt, 0, 0, 0);
    x3_epi_pair(acc, y4, 2 * kb + 1, res, lin, prod);
    __builtin_amdgcn_sched_barrier(0);
    nxt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, z1[kb], nxt, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

constexpr int X3_ROLE_WAVES = 8;
// Prefetch depth: tile k + PA is issued in iteration k, and the barrier of iteration k waits
// only for the DMAs of the tile pair it needs (A(k+1), labels(k)), leaving the later PA - 2
// pairs in flight (counted vmcnt: with a plain vmcnt(0) every barrier waited for the DMAs
// issued one iteration earlier, so the HBM latency was exposed once per tile whatever the
// depth -- round 3 measured 2, 3 and 4 slots equal).  Depth A/B with the counted waits
// (profiles/r04/ab_tail_prefetch.txt): PA = 2 / 4 / 6 at 1-32 chains 0.077-0.078 / 0.085 /
// 0.089-0.090 ms per evaluation, at 256 chains 0.235 / 0.247 / 0.255 ms; bench --chains 512
// seeds 0-2 1.013M / 1.092M / 0.877M at PA = 2 vs 1.003M / 1.081M / 0.867M at 4: the deeper
// rings cost more in LDS-DMA issue and barrier waits than they hide.  LDS at PA = 2: 4 A slots
// x 14 KB + 3 label slots + 32 KB of residual slots = 91 KB, one workgroup per CU.
#ifndef NMX_X3_ROLE_PA
#define NMX_X3_ROLE_PA 2
#endif
constexpr int X3_ROLE_PA = NMX_X3_ROLE_PA;

// A-ring slots of the tail form: tiles k - 1 (GEMM2 of the B waves, transposed reads of the
// GEMM1 image), k + 1 (GEMM1 of the A waves) and k + PA landing
template <int PA>
constexpr int x3_roles_aslots() { return PA + 2; }

// A-part pieces a tail-form slot holds: with H the compact image (the last k-block's plane
// pieces left out: x3_gemm2_tr_load<..., true> takes those columns from the combined pieces), so
// the tail launches stream 11 + 1 KB per 32-row tile for covtype -- 218 MB of X per launch, which
// the 256 MB Infinity Cache keeps across a run's back-to-back tail launches (14 + 1 KB, 272 MB,
// did not fit)
template <int KB, int H>
constexpr int x3_roles_na() { return H ? 3 * (KB - 1) + 2 : 3 * KB; }

template <int KB, int DT, int H, int PA>
inline size_t x3_roles_lds_bytes() {
  constexpr int NA = x3_roles_na<KB, H>();
  // A ring, the label ring (one 1-KB piece per tile, PA + 1 slots), the residual ring
  return (size_t)(x3_roles_aslots<PA>() * NA + (PA + 1)) * 1024 + (size_t)2 * 4 * 4096;
}

// ---- narrow tail: launches over at most 32 listed chains ----------------------------------
// The common case of a NUTS run's straggler phase is one chain tile (<= 32 chains).  The role
// split above then keeps two SIMDs busy (the tile's A and B waves), its per-tile critical path
// GEMM1 + epilogue on one wave and both GEMM2 column halves plus the residual split on another,
// one barrier per tile (0.78 us a tile).  Here the one chain tile runs as a three-stage pipeline
// over tile pairs, one barrier per pair:
//   role A, waves 2 and 3 (SIMDs 2, 3): the tiles of a split alternately -- GEMM1 of tile
//     2k+2+a hand-interleaved with the epilogue of tile 2k+a, exactly x3_a_tile -- residual R and
//     U term to LDS (iteration k);
//   split, waves 4 and 5 (SIMDs 0, 1): the residual of tile 2(k-1)+j split into its three bf16
//     terms (iteration k), beside the role-B wave of their SIMD, which is MFMA-bound;
//   role B, waves 0 and 1 (SIMDs 0, 1): GEMM2 for one 32-column half dt each, over every tile in
//     tile order (pair k-2 in iteration k), wave 0 also adds the tiles' U terms in tile order;
//   every LDS-DMA on waves 4-7, two thirds on 6 and 7 (s_memtime stamps of an experiment build:
//     a 1-KB piece costs its issuing wave ~160-330 cycles, on the A / B waves the critical path).
// Every accumulator sees x3_item's products in x3_item's order, the split is split3 of the same
// values: bitwise the results of the other forms.  Compact image (H) only.  LDS (159 KB): images
// of five tile pairs (k-2 in GEMM2, k-1 and k kept for it, k+1 in GEMM1, k+2 landing), labels of
// two, residuals + terms and split residuals + terms of two pairs each.
template <int KB, int H>
inline size_t x3_narrow_lds_bytes() {
  constexpr int NA = x3_roles_na<KB, H>();
  return (size_t)(10 * NA + 4) * 1024 + 2 * 2 * (4096 + 512) + 2 * 2 * (6144 + 512);
}

// role B's operands of one tile, issued without a wait: the transposed X^T reads of column half
// DTI, the split residual (terms t of k-steps s at (3 s + t) KB) and (TERM) the tile's U term
template <int KB, int DT, bool CMP, int DTI, bool TERM>
__device__ __forceinline__ void x3_narrow_b_issue(const char* slot, const char* sbase, const char* tbase,
                                                  bf16x8 (&fb)[3][2], bf16x8 (&r)[2][3], double& term) {
  x3_tr_load_dt<KB, DT, CMP, DTI>(slot, fb);
  const unsigned sa = (unsigned)(size_t)((__attribute__((address_space(3))) const char*)sbase);
  asm volatile(
      "ds_read_b128 %0, %6\n\t"
      "ds_read_b128 %1, %6 offset:1024\n\t"
      "ds_read_b128 %2, %6 offset:2048\n\t"
      "ds_read_b128 %3, %6 offset:3072\n\t"
      "ds_read_b128 %4, %6 offset:4096\n\t"
      "ds_read_b128 %5, %6 offset:5120"
      : "=&v"(r[0][0]), "=&v"(r[0][1]), "=&v"(r[0][2]), "=&v"(r[1][0]), "=&v"(r[1][1]), "=&v"(r[1][2])
      : "v"(sa)
      : "memory");
  if constexpr (TERM) {
    const unsigned ta = (unsigned)(size_t)((__attribute__((address_space(3))) const char*)tbase);
    asm volatile("ds_read_b64 %0, %1" : "=&v"(term) : "v"(ta) : "memory");
  }
}
// wait for them (N: LDS operations issued after them that may stay in flight, <= 15); the empty
// asm makes every later use depend on the wait
template <int N = 0>
__device__ __forceinline__ void x3_narrow_b_wait(bf16x8 (&fb)[3][2], bf16x8 (&r)[2][3], double& term) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int pl = 0; pl < 3; ++pl)
#pragma unroll
    for (int sidx = 0; sidx < 2; ++sidx) asm volatile("" : "+v"(fb[pl][sidx]), "+v"(r[sidx][pl]));
  asm volatile("" : "+v"(term));
}
// the tile's 12 GEMM2 MFMAs of one column half, in x3_gemm2's order
__device__ __forceinline__ void x3_narrow_b_mma(const bf16x8 (&fb)[3][2], const bf16x8 (&r)[2][3], f32x16& g) {
#pragma unroll
  for (int sidx = 0; sidx < 2; ++sidx) {
    const bf16x8 b1 = fb[0][sidx], b2 = fb[1][sidx], b3 = fb[2][sidx];
    const bf16x8 r1 = r[sidx][0], r2 = r[sidx][1], r3 = r[sidx][2];
    g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b3, r1, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r2, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r3, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, r1, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r2, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, r1, g, 0, 0, 0);
  }
}

template <int KB, int DT, int H>
__device__ __forceinline__ void x3_narrow(const char* __restrict__ Xq, int64_t ntiles, int D, int S, int split,
                                          const nmx_eval_batch& ev, float* __restrict__ gpart,
                                          double* __restrict__ pepart, char* lds) {
  constexpr int NP = 3 * KB + 2 * H + 6 * DT + 1, NA = x3_roles_na<KB, H>();
  constexpr bool CMP = H != 0;
  constexpr int NIMG = 10, NLAB = 4;  // tile slots: 5 image pairs, 2 label pairs
  constexpr int NQ = 2 * NA + 2;      // DMA pieces of a pair: the images of two tiles, their labels
  static_assert(DT == 2 && H == 1 && X3_ROLE_WAVES == 8, "narrow tail: compact image, two column halves, 8 waves");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, l31 = lane & 31;
  const int ldc = ev.ldc;
  const int pos = l31;  // the chain tile 0 (ldc >= 64)
  const int c = nmx_eval_chain(ev, pos);
  const int64_t per = (ntiles + S - 1) / S;
  const int64_t t0 = min((int64_t)split * per, ntiles);
  const int64_t t1 = min(t0 + per, ntiles);
  const int nt = (int)(t1 - t0);
  const int npairs = (nt + 1) / 2;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Xq + (size_t)t0 * NP * 1024), 0, (int)((size_t)nt * NP * 1024), 0x00020000);
  char* iring = lds;                         // [tile % NIMG][NA KB]
  char* lring = iring + NIMG * NA * 1024;    // [tile % NLAB][1 KB]
  char* rring = lring + NLAB * 1024;         // [pair parity][j][4 KB] residuals
  char* tring = rring + 2 * 2 * 4096;        // [pair parity][j][512 B] their U terms
  char* sring = tring + 2 * 2 * 512;         // [pair parity][j][6 KB] split residuals
  char* uring = sring + 2 * 2 * 6144;        // [pair parity][j][512 B] their U terms
  // DMA pair p = the images of tile pair p + 1 and the labels of pair p; its piece q (images: q
  // = j NA + il for tile j of the pair and slot position il; labels: q = 2 NA + j) is issued by
  // wave owner(q).  Iteration k needs pair k, issued in iteration k - 1 (all of it: the barrier
  // waits vmcnt(0)).
  auto issue_q = [&](int p, int q) {
    if (q < 2 * NA) {
      const int j = q / NA, il = q % NA, tile = 2 * (p + 1) + j;
      if (tile < nt) {
        const int i = il < 3 * (KB - 1) ? (il / (KB - 1)) * KB + il % (KB - 1) : 3 * KB + (il - 3 * (KB - 1));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xrs, (__attribute__((address_space(3))) void*)(iring + (tile % NIMG) * NA * 1024 + il * 1024), 16,
            lane * 16, (unsigned)((tile * NP + i) * 1024), 0, 0);
      }
    } else {
      const int tile = 2 * p + (q - 2 * NA);
      if (tile < nt)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xrs, (__attribute__((address_space(3))) void*)(lring + (tile % NLAB) * 1024), 16, lane * 16,
            (unsigned)((tile * NP + NP - 1) * 1024), 0, 0);
    }
  };
  // pieces q < 16 go to waves 6 and 7 (SIMDs 2, 3, beside the A waves), the rest to the split
  // waves 4 and 5 (stamps: a wave issuing LDS-DMA stalls ~160-330 cycles a piece, ~1000 cycles
  // for even one piece on the A / B waves, whose reads and MFMAs then start late: measured
  // slower, 0.069 vs 0.058 ms per 1-32-chain evaluation)
  auto owner = [&](int q) { return q < 16 ? 6 + (q & 1) : 4 + (q & 1); };
  auto issue_pair = [&](int p) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (owner(q) == w) issue_q(p, q);
  };
  static_assert(NQ == 24, "the owner table covers 24 pieces a pair");
  const bool roleA = w == 2 || w == 3;
  // a tile's index within a pair is w & 1 for the A, split and B waves alike (w - 2 / w - 4 here
  // let the compiler merge the A and split waves' LDS addresses with a form valid for one only)
  const int a = w & 1;
  bf16x8 z1[KB], z2[KB], z3[KB];
  if (roleA) {
    const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc((void*)ev.z, 0, D * ldc * 4, 0x00020000);
    x3_load_z<KB, H>(zrs, c, h, ldc, z1, z2, z3);
  }
  f32x16 g;
#pragma unroll
  for (int r = 0; r < 16; ++r) g[r] = 0.0f;
  double pe = 0.0;
  if (nt > 0) {
    // the images of pair 0
#pragma unroll
    for (int q = 0; q < 2 * NA; ++q)
      if (owner(q) == w) issue_q(-1, q);
    x3_roles_barrier();  // the images of pair 0 are in
    issue_pair(0);
    f32x16 accA, accB;
    if (roleA) accA = x3_gemm1<KB, H, CMP>(reinterpret_cast<const bf16x8*>(iring + (a % NIMG) * NA * 1024) + lane, z1,
                                           z2, z3);
    auto iter = [&](int k, const f32x16& acc, f32x16& nxt) {
      x3_roles_barrier();  // DMA pair k landed; R(k - 1), SR(k - 2) written; pair k - 3's slots read
      issue_pair(k + 1);
      if (roleA) {
        const int i = 2 * k + a;
        if (k < npairs && i < nt) {
          f32x4 y4[4];
          x3_labels(lring + (i % NLAB) * 1024, h, y4);
          x3_labels_wait(y4);
          // GEMM1 of this wave's next tile i + 2 (a stale slot past the last tile: computed, never used)
          const bf16x8* fa = reinterpret_cast<const bf16x8*>(iring + ((i + 2) % NIMG) * NA * 1024) + lane;
          float res[16];
          float lin = 0.0f;
          float prod[2] = {1.0f, 1.0f};
          x3_a_tile<KB, H, CMP>(fa, z1, z2, z3, acc, y4, nxt, res, lin, prod);
          const double term = x3_epi_term(lin, prod);
          x3_res_store(rring + ((k & 1) * 2 + a) * 4096 + lane * 16, res);
          const unsigned ta =
              (unsigned)(size_t)((__attribute__((address_space(3))) char*)(tring + ((k & 1) * 2 + a) * 512)) + lane * 8;
          asm volatile("ds_write_b64 %0, %1" ::"v"(ta), "v"(term) : "memory");
        }
      } else if (w == 4 || w == 5) {
        const int j = w & 1, i = 2 * (k - 1) + j, par = (k - 1) & 1;
        if (k >= 1 && k <= npairs && i < nt) {  // split R(i): the residual's three bf16 terms per k-step
          float res[16];
          x3_res_load(rring + (par * 2 + j) * 4096 + lane * 16, res);
          const unsigned ta =
              (unsigned)(size_t)((__attribute__((address_space(3))) char*)(tring + (par * 2 + j) * 512)) + lane * 8;
          double term;
          asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(term) : "v"(ta) : "memory");
          bf16x8 r[2][3];
#pragma unroll
          for (int sidx = 0; sidx < 2; ++sidx) {
            float v[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] = res[8 * sidx + jj];
            split3(v, r[sidx][0], r[sidx][1], r[sidx][2]);
          }
          const unsigned sa =
              (unsigned)(size_t)((__attribute__((address_space(3))) char*)(sring + (par * 2 + j) * 6144)) + lane * 16;
          asm volatile(
              "ds_write_b128 %0, %1\n\t"
              "ds_write_b128 %0, %2 offset:1024\n\t"
              "ds_write_b128 %0, %3 offset:2048\n\t"
              "ds_write_b128 %0, %4 offset:3072\n\t"
              "ds_write_b128 %0, %5 offset:4096\n\t"
              "ds_write_b128 %0, %6 offset:5120" ::"v"(sa),
              "v"(r[0][0]), "v"(r[0][1]), "v"(r[0][2]), "v"(r[1][0]), "v"(r[1][1]), "v"(r[1][2])
              : "memory");
          const unsigned ua =
              (unsigned)(size_t)((__attribute__((address_space(3))) char*)(uring + (par * 2 + j) * 512)) + lane * 8;
          asm volatile("ds_write_b64 %0, %1" ::"v"(ua), "v"(term) : "memory");
        }
      } else if (w < 2 && k >= 2) {
        const int i0 = 2 * (k - 2), par = k & 1;  // (k - 2) & 1
        const bool two = i0 + 1 < nt;
        bf16x8 fb0[3][2], fb1[3][2], r0[2][3], r1[2][3];
        double u0 = 0.0, u1 = 0.0;
        // both tiles' operands at once (a missing second tile's slots are valid LDS: its MFMAs
        // run on whatever they hold and are dropped)
        if (w == 0) {
          x3_narrow_b_issue<KB, DT, CMP, 0, true>(iring + (i0 % NIMG) * NA * 1024,
                                                  sring + (par * 2) * 6144 + lane * 16,
                                                  uring + (par * 2) * 512 + lane * 8, fb0, r0, u0);
          x3_narrow_b_issue<KB, DT, CMP, 0, true>(iring + ((i0 + 1) % NIMG) * NA * 1024,
                                                  sring + (par * 2 + 1) * 6144 + lane * 16,
                                                  uring + (par * 2 + 1) * 512 + lane * 8, fb1, r1, u1);
        } else {
          x3_narrow_b_issue<KB, DT, CMP, 1, false>(iring + (i0 % NIMG) * NA * 1024,
                                                   sring + (par * 2) * 6144 + lane * 16, nullptr, fb0, r0, u0);
          x3_narrow_b_issue<KB, DT, CMP, 1, false>(iring + ((i0 + 1) % NIMG) * NA * 1024,
                                                   sring + (par * 2 + 1) * 6144 + lane * 16, nullptr, fb1, r1, u1);
        }
        // the first tile's operands (the oldest of the 37-38 reads), then its MFMAs while the
        // second tile's reads land
        x3_narrow_b_wait<15>(fb0, r0, u0);
        x3_narrow_b_mma(fb0, r0, g);
        x3_narrow_b_wait<0>(fb1, r1, u1);
        f32x16 g1 = g;
        x3_narrow_b_mma(fb1, r1, g1);
#pragma unroll
        for (int r = 0; r < 16; ++r) g[r] = two ? g1[r] : g[r];
        if (w == 0) {
          pe += u0;
          if (two) pe += u1;
        }
      }
    };
    for (int k = 0; k <= npairs + 1; k += 2) {
      iter(k, accA, accB);
      if (k + 1 <= npairs + 1) iter(k + 1, accB, accA);
    }
  }
  if (w >= 2 || pos >= ldc) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (d < D) gpart[((size_t)split * D + d) * ldc + pos] = g[r];
  }
  if (w == 0) {
    const double p = pe + __shfl_xor(pe, 32);
    if (h == 0) pepart[(size_t)split * ldc + pos] = p;
  }
}

template <int KB, int DT, int H, int PA>
__global__ __launch_bounds__(64 * X3_ROLE_WAVES, 1) void k_logreg_x3_roles(const char* __restrict__ Xq,
                                                                         int64_t ntiles, int D, int S, int Gt,
                                                                         nmx_eval_batch ev, float* __restrict__ gpart,
                                                                         double* __restrict__ pepart) {
  // the A ring holds the tile's GEMM1 image (with H the compact one: x3_roles_na), from which the
  // B waves also read GEMM2's X^T operand
  constexpr int NP = 3 * KB + 2 * H + 6 * DT + 1, NA = x3_roles_na<KB, H>();
  constexpr bool CMP = H != 0;
  static_assert(KB == 4, "role-split tail form: D in (48, 64]");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int b = blockIdx.x;
  const int qb = b >> 3;
  const int ct = qb % Gt;
  const int npos = ev.active_idx ? *ev.active_count : ev.ldc;
  if (ct * 128 >= npos) return;
  const int split = (qb / Gt) * 8 + (b & 7);
  if (npos <= 32) {  // one chain tile: the narrow form (ct = 0 here)
    if constexpr (DT == 2 && H == 1) {
      x3_narrow<KB, DT, H>(Xq, ntiles, D, S, split, ev, gpart, pepart, lds);
      return;
    }
  }
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool roleA = w < 4;
  // chain tile of the group: A waves 0-3 own tiles 0-3; B waves 4-7 own tiles 2, 3, 0, 1, so
  // with waves dealt to SIMDs w mod 4 the two waves of tile 0 / 1 (the tail's usual 1-2 active
  // tiles) sit on different SIMDs and their MFMA streams run in parallel
  const int t = roleA ? w : ((w + 2) & 3);
  const int h = lane >> 5;
  const int l31 = lane & 31;
  const int ldc = ev.ldc;
  const int pos = (ct * 4 + t) * 32 + l31;
  const int c = pos < ldc ? nmx_eval_chain(ev, pos) : -1;
  const bool active = __any(c >= 0);  // wave-uniform, equal for the A and B waves of a tile
  if (!__syncthreads_or(active)) return;

  const int64_t per = (ntiles + S - 1) / S;
  const int64_t t0 = min((int64_t)split * per, ntiles);
  const int64_t t1 = min(t0 + per, ntiles);
  const int nt = (int)(t1 - t0);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Xq + (size_t)t0 * NP * 1024), 0, (int)((size_t)nt * NP * 1024), 0x00020000);
  // The tail launch streams each tile's GEMM1 image (compact with H) and its labels only, and the
  // B waves take GEMM2's X^T operand from that image by transposed LDS reads (x3_gemm2_tr_load),
  // so the B pieces (half the packed bytes) stay in HBM.
  constexpr int PB = PA + 1, PAS = x3_roles_aslots<PA>();
  char* aring = lds;
  char* bring = lds + PAS * NA * 1024;  // labels: [slot][1 KB]
  char* rring = bring + PB * 1024;      // [slot][tile][4 KB]
  auto issue_a = [&](int k) {
    char* dst = aring + (k % PAS) * NA * 1024;
#pragma unroll
    for (int j = 0; j < (NA + X3_ROLE_WAVES - 1) / X3_ROLE_WAVES; ++j) {
      const int il = w + X3_ROLE_WAVES * j;  // slot position; i = the tile's piece
      const int i = !CMP ? il
                         : (il < 3 * (KB - 1) ? (il / (KB - 1)) * KB + il % (KB - 1) : 3 * KB + (il - 3 * (KB - 1)));
      if (il < NA)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + il * 1024), 16,
                                                 lane * 16, (unsigned)((k * NP + i) * 1024), 0, 0);
    }
  };
  auto issue_b = [&](int k) {  // the label piece (the last of the tile)
    if (w == X3_ROLE_WAVES - 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(bring + (k % PB) * 1024),
                                               16, lane * 16, (unsigned)((k * NP + NP - 1) * 1024), 0, 0);
  };
  char* const rmine = rring + t * 4096 + lane * 16;  // + slot * 4 * 4096
  // LDS-DMA pair p = (A(p + 1), labels(p)): pair p is issued in the prologue (p < PA - 1) or in
  // iteration p - PA + 1; iteration k needs pair k, so this wave's DMAs of pairs k + 1 ..
  // k + PA - 2 may stay in flight at its barrier
  const int na_w = (w < NA - X3_ROLE_WAVES ? 2 : 1) + (NA > 2 * X3_ROLE_WAVES ? 1 : 0);
  static_assert(NA <= 2 * X3_ROLE_WAVES, "issue_a: at most two pieces per wave");
  auto pair_ops = [&](int p) { return (p + 1 < nt ? na_w : 0) + (w == X3_ROLE_WAVES - 1 && p < nt ? 1 : 0); };
  auto in_flight = [&](int k) {
    int n = 0;
#pragma unroll
    for (int p = 1; p <= X3_ROLE_PA - 2; ++p) n += pair_ops(k + p);
    return n;
  };

  if (roleA) {
    // ---- role A: GEMM1 + epilogue, hands R(k) to its B wave --------------------------------
    const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc((void*)ev.z, 0, D * ldc * 4, 0x00020000);
    bf16x8 z1[KB], z2[KB], z3[KB];
    x3_load_z<KB, H>(zrs, c, h, ldc, z1, z2, z3);
    double pe = 0.0;
    if (nt > 0) {
      issue_a(0);
      x3_roles_barrier();  // A(0) is in
      for (int p = 0; p < PA - 1; ++p) {  // pairs (A(p + 1), labels(p)), in the loop's order
        if (p + 1 < nt) issue_a(p + 1);
        if (p < nt) issue_b(p);
      }
      f32x16 accA, accB;
      if (active) accA = x3_gemm1<KB, H, CMP>(reinterpret_cast<const bf16x8*>(aring) + lane, z1, z2, z3);
      auto stepA = [&](int k, const f32x16& acc, f32x16& nxt) {
        x3_roles_barrier_rt(in_flight(k));  // A(k+1), B(k) landed; R slot k&1 was read by B in iteration k-1
        if (k + PA < nt) issue_a(k + PA);
        if (k + PA - 1 < nt) issue_b(k + PA - 1);
        if (!active) return;
        f32x4 y4[4];
        x3_labels(bring + (k % PB) * 1024, h, y4);
        x3_labels_wait(y4);
        const bf16x8* fa = reinterpret_cast<const bf16x8*>(aring + ((k + 1) % PAS) * NA * 1024) + lane;
        float res[16];
        float lin = 0.0f;
        float prod[2] = {1.0f, 1.0f};
        x3_a_tile<KB, H, CMP>(fa, z1, z2, z3, acc, y4, nxt, res, lin, prod);
        x3_epi_finish(lin, prod, pe);
        x3_res_store(rmine + (k & 1) * 4 * 4096, res);
      };
      for (int k = 0; k < nt; k += 2) {
        stepA(k, accA, accB);
        if (k + 1 < nt) stepA(k + 1, accB, accA);
      }
      x3_roles_barrier();  // R(nt-1) handed over
    }
    if (!active || pos >= ldc) return;
    const double p = pe + __shfl_xor(pe, 32);
    if (h == 0) pepart[(size_t)split * ldc + pos] = p;
  } else {
    // ---- role B: split R(k-1) + GEMM2(k-1) --------------------------------------------------
    f32x16 g[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) g[dt][r] = 0.0f;
    auto gemm2 = [&](int k) {  // GEMM2 of tile k
      bf16x8 fb[3][DT][2];
      x3_gemm2_tr_load<KB, DT, CMP>(aring + (k % PAS) * NA * 1024, fb);
      float res[16];
      x3_res_load(rmine + (k & 1) * 4 * 4096, res);  // (waits for every LDS read, the above too)
      x3_tr_wait<DT>(fb);
      x3_gemm2_regs<DT>(fb, res, g);
    };
    if (nt > 0) {
      issue_a(0);
      x3_roles_barrier();
      for (int p = 0; p < PA - 1; ++p) {
        if (p + 1 < nt) issue_a(p + 1);
        if (p < nt) issue_b(p);
      }
      for (int k = 0; k < nt; ++k) {
        x3_roles_barrier_rt(in_flight(k));
        if (k + PA < nt) issue_a(k + PA);
        if (k + PA - 1 < nt) issue_b(k + PA - 1);
        if (active && k > 0) gemm2(k - 1);
      }
      x3_roles_barrier();
      if (active) gemm2(nt - 1);
    }
    if (!active || pos >= ldc) return;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = 32 * dt + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (d < D) gpart[((size_t)split * D + d) * ldc + pos] = g[dt][r];
      }
  }
}

// Sum of slots sp0 .. sp1-1 at stride st (in slot order; FIN_BATCH loads issued ahead of their
// adds; 64 measured equal at 332 VGPRs, profiles/r03/ab_finalize.txt)
#ifndef NMX_FIN_BATCH
#define NMX_FIN_BATCH 32
#endif
template <class T>
__device__ __forceinline__ T sum_slots(const T* __restrict__ p, size_t st, int sp0, int sp1) {
  constexpr int B = NMX_FIN_BATCH;
  T s = 0;
  int sp = sp0;
  for (; sp + B <= sp1; sp += B) {
    T v[B];
#pragma unroll
    for (int j = 0; j < B; ++j) v[j] = __builtin_nontemporal_load(p + (size_t)(sp + j) * st);
#pragma unroll
    for (int j = 0; j < B; ++j) s += v[j];
  }
  for (; sp < sp1; ++sp) s += p[(size_t)sp * st];
  return s;
}

// One workgroup per (64 batch positions, coordinate d or the U row d = D).  Wave w sums the
// slots [w S / W, (w + 1) S / W) in order, then the W wave sums are added in wave order: a
// fixed order that depends on S (a function of n_rows) only, and W independent load streams
// per output, so the small launches of a NUTS tail are not one long dependent chain of loads.
// wcol: U gains the per-chain linear term w . b; pe_shift removes the log(2) terms of the zero
// rows that pad the split-bf16 tiles.  W = 4 (8 and 16 measured slower)
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
  // the U row's z loads (wave 0) go out before the slot sums: one dependent round less
  // (clamped rows, masked after: a load under `k < D` compiled to 55 branches, each with its own
  // vmcnt(0) wait -- one dependent round per coordinate, ~14 us of a tail launch's finalize)
  float zf[64];
  if (d == D && w == 0 && c >= 0) {
#pragma unroll
    for (int k = 0; k < 64; ++k) zf[k] = ev.z[(size_t)(k < D ? k : D - 1) * ldc + c];
#pragma unroll
    for (int k = 0; k < 64; ++k) zf[k] = k < D ? zf[k] : 0.0f;
  }
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
    ev.grad[idx] = ev.z[idx] - s;  // the partials hold X^T (y - sigmoid(l)) (x3_epi_pair)
  } else {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < FIN_WAVES; ++i) s += part[i][lane];
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

// Launches over at most this many 128-chain groups (a NUTS run's tail: one workgroup per split
// and CU) run the role-split form k_logreg_x3_roles (bitwise equal): 0.083 vs 0.105 ms per
// evaluation at 16-64 chains, incl. the finalize.
#ifndef NMX_X3_TAIL_TILES
#define NMX_X3_TAIL_TILES 2
#endif
constexpr int X3_TAIL_TILES = NMX_X3_TAIL_TILES;

int check_ev(const nmx_eval_batch* ev) {
  if (!ev || !ev->z || !ev->grad || !ev->pe) return nmx_fail(NMX_ERR_INVALID, "eval batch has NULL pointers");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains || ev->ldc % 64)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  return NMX_OK;
}

}  // namespace

extern "C" int nmx_logreg_num_splits(int64_t n_rows) { return x3_num_splits(n_rows); }


// packed buffer: w[64] (k_logreg_colsums) | split-bf16 tiles (k_logreg_pack_x3)
inline size_t x3_offset() { return (COLTERM_BYTES + 255) / 256 * 256; }

extern "C" size_t nmx_logreg_packed_bytes(int64_t n_rows, int dim) {
  if (n_rows <= 0 || dim <= 0) return 0;
  return x3_offset() + (size_t)x3_ntiles(n_rows) * x3_np(dim) * 1024;
}

extern "C" int nmx_logreg_pack(const float* X, const float* y, int64_t n_rows, int dim, void* packed,
                               void* stream) {
  if (!X || !y || !packed) return nmx_fail(NMX_ERR_INVALID, "logreg_pack: NULL pointer");
  if (n_rows <= 0 || dim <= 0 || dim > 64)
    return nmx_fail(NMX_ERR_INVALID, "logreg_pack: need n_rows > 0 and 0 < dim <= 64 (got %lld, %d)",
                    (long long)n_rows, dim);
  hipLaunchKernelGGL(k_logreg_colsums, dim3(dim), dim3(CS_THREADS), 0, (hipStream_t)stream, X, y, n_rows, dim,
                     (double*)packed);
  if (int st = nmx_check_launch("k_logreg_colsums")) return st;
  const int64_t nt = x3_ntiles(n_rows);
  const int64_t nthreads = nt * x3_np(dim) * 64;
  hipLaunchKernelGGL(k_logreg_pack_x3, dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, X,
                     y, n_rows, dim, x3_kb(dim), x3_dt(dim), x3_h(dim), nt, (bf16x8*)((char*)packed + x3_offset()));
  return nmx_check_launch("k_logreg_pack_x3");
}

extern "C" size_t nmx_logreg_workspace_bytes(int64_t n_rows, int dim, int num_chains) {
  const size_t ldc = (size_t)(num_chains + 63) / 64 * 64;
  const size_t S = x3_num_splits(n_rows);
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
  const int S = x3_num_splits(n_rows);
  float* gpart = (float*)workspace;
  double* pepart = (double*)((char*)workspace + ((size_t)S * dim * ev->ldc * sizeof(float) + 255) / 256 * 256);
  const int64_t nt = x3_ntiles(n_rows);
  const int KB = x3_kb(dim);
  const int H = x3_h(dim);
  const char* Xq = (const char*)packed + x3_offset();
  const int nb = std::min(ev->num_chains, ev->ldc);  // batch positions that can hold a chain
  const int Gt = (nb + 127) / 128;
  const dim3 grid(Gt * S), blk(256);
  if (KB == 4 && Gt <= X3_TAIL_TILES) {
    // the role-split form, or (compact image) the narrow one (<= 32 listed chains, decided in the
    // kernel): LDS for either
    const size_t lds = H ? std::max(x3_roles_lds_bytes<4, 2, 1, X3_ROLE_PA>(), x3_narrow_lds_bytes<4, 1>())
                         : x3_roles_lds_bytes<4, 2, 0, X3_ROLE_PA>();
    const void* fn = H ? (const void*)k_logreg_x3_roles<4, 2, 1, X3_ROLE_PA>
                       : (const void*)k_logreg_x3_roles<4, 2, 0, X3_ROLE_PA>;
    if (int st = nmx_lds_limit(fn, lds, s, "k_logreg_x3_roles")) return st;
    if (H)
      hipLaunchKernelGGL((k_logreg_x3_roles<4, 2, 1, X3_ROLE_PA>), grid, dim3(64 * X3_ROLE_WAVES), lds, s, Xq, nt,
                         dim, S, Gt, *ev, gpart, pepart);
    else
      hipLaunchKernelGGL((k_logreg_x3_roles<4, 2, 0, X3_ROLE_PA>), grid, dim3(64 * X3_ROLE_WAVES), lds, s, Xq, nt,
                         dim, S, Gt, *ev, gpart, pepart);
  }
  else if (KB == 4 && H)
    hipLaunchKernelGGL((k_logreg_x3<4, 2, 1, 3, 0>), grid, blk, (x3_lds_bytes<4, 2, 1>()), s, Xq, nt, dim, S, Gt,
                       *ev, gpart, pepart);
  else if (KB == 4)
    hipLaunchKernelGGL((k_logreg_x3<4, 2, 0, 3, 0>), grid, blk, (x3_lds_bytes<4, 2, 0>()), s, Xq, nt, dim, S, Gt,
                       *ev, gpart, pepart);
  else if (KB == 3)
    hipLaunchKernelGGL((k_logreg_x3<3, 2, 0, 3, 0>), grid, blk, (x3_lds_bytes<3, 2, 0>()), s, Xq, nt, dim, S, Gt,
                       *ev, gpart, pepart);
  else if (KB == 2)
    hipLaunchKernelGGL((k_logreg_x3<2, 1, 0, 3, 0>), grid, blk, (x3_lds_bytes<2, 1, 0>()), s, Xq, nt, dim, S, Gt,
                       *ev, gpart, pepart);
  else
    hipLaunchKernelGGL((k_logreg_x3<1, 1, 0, 3, 0>), grid, blk, (x3_lds_bytes<1, 1, 0>()), s, Xq, nt, dim, S, Gt,
                       *ev, gpart, pepart);
  if (int st = nmx_check_launch("k_logreg_x3")) return st;
  const double* wcol = (const double*)packed;
  const double shift = -(double)(nt * X3_ROWS - n_rows) * 0.6931471805599453;
  hipLaunchKernelGGL(k_logreg_finalize, dim3((nb + 63) / 64, dim + 1), dim3(64 * FIN_WAVES), 0, s, gpart, pepart, S,
                     dim, *ev, wcol, shift);
  return nmx_check_launch("k_logreg_finalize");
}
