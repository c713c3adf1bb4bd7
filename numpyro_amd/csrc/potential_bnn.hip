// Bayesian neural network of examples/bnn.py:43-74 (D_X -> H -> H -> 1, tanh):
//   w1 [Dx,H], w2 [H,H], w3 [H,1] ~ N(0,1), prec_obs ~ Gamma(3,1),
//   Y ~ N(tanh(tanh(X w1) w2) w3, 1/sqrt(prec_obs)),
// z = (log prec_obs, w1, w2, w3) row-major (ravel_pytree of the sorted sites).
//
// U and dU per chain with the hand-derived adjoint (oracle
// BNN.pe_grad).  One workgroup (8 waves) owns one evaluated chain: its weights, both
// activation layers and the adjoints live in LDS (N=100, H=69: 78 KB, two workgroups per
// CU).  The three N x H x H products -- h1 W2 (forward), h1^T ga2 (grad W2) and ga2 W2^T
// (back to layer 1), ~2.9 MFLOP of the ~3 per chain-evaluation -- run on the matrix cores as
// 32 x 32 output tiles of v_mfma_f32_32x32x2_f32 (f32 operands, f32 accumulation in k order:
// bitwise the sequential FMA chain), the tiles of a product spread over the waves, operands
// read from LDS with the padding rows / columns masked to zero.  gfx950's f32 matrix peak
// equals its f32 vector peak (157 TF/s), so the gain over register-blocked FMA loops is the
// freed VALU (measured 0.30 vs 0.34 ms at 2048 chains, scripts/ab_bnn.py); the rest of a
// chain's evaluation is latency-bound serial phases (tanh layers, reductions, 20 KB of
// parameters in and gradient out).  Round 4: 16 x 16 tiles (v_mfma_f32_16x16x4_f32, less padding,
// even over the waves) and the serial sums unrolled (their loads issued ahead, same order).  The chain-major columns of the
// evaluated chains are first transposed to rows (k_cols_to_rows, 64x64 LDS tiles, both
// sides coalesced) so each workgroup reads its chain's 20 KB parameter vector and writes
// its gradient contiguously; k_rows_to_cols scatters the gradients back.
#include <math.h>

#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

constexpr int THREADS = 512;
constexpr int NWAVES = THREADS / 64;

// One 16 x 16 output tile of v_mfma_f32_16x16x4_f32: lane l supplies A(l & 15, 4s + (l >> 4)) and
// B(4s + (l >> 4), l & 15); register r of lane l holds row 4 (l >> 4) + r, column l & 15.  The
// same f32 products accumulated in k order as the 32 x 32 form, on tiles that fit N = 100 and
// H = 69 with less padding (7 x 5 tiles of 16 vs 4 x 3 of 32: 0.77 of the MACs useful vs 0.56)
// and spread evenly over the 8 waves (35 / 25 tiles instead of 12 / 9).
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <class FA, class FB>
__device__ __forceinline__ f32x4 mfma_tile16(int K, FA fa, FB fb) {
  const int lane = threadIdx.x & 63, l15 = lane & 15, kq = lane >> 4;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 6
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + kq;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa(l15, k), fb(k, l15), acc, 0, 0, 0);
  }
  return acc;
}
__device__ __forceinline__ int tile_row16(int r) { return 4 * ((threadIdx.x & 63) >> 4) + r; }


struct BnnDims {
  int N, Dx, H;
  int o_w1, o_w2, o_w3;  // offsets of the sites in z
};

// Sum over the workgroup in a fixed order: the 8 waves' values per lane in wave order, then the
// 64 lanes by a butterfly (the serial 64-step loop of thread 0 it replaces was ~1.5 us per sum)
__device__ __forceinline__ float block_sum256(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  float t = 0.0f;
  if (threadIdx.x < 64) {
#pragma unroll
    for (int w = 0; w < THREADS / 64; ++w) t += red[w * 64 + threadIdx.x];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
    if (threadIdx.x == 0) red[0] = t;
  }
  __syncthreads();
  t = red[0];
  __syncthreads();
  return t;
}

// Column <-> row transposes of the listed chains: rows[p][d] = cols[d][chain(p)] (and back),
// 64 x 64 tiles through LDS so both sides are coalesced.  They let k_bnn read and write
// each chain's D-vector contiguously instead of one cache line per coordinate.
__global__ __launch_bounds__(256) void k_cols_to_rows(const float* __restrict__ cols, int D, nmx_eval_batch ev,
                                                      float* __restrict__ rows) {
  __shared__ float tile[64][65];
  const int p0 = blockIdx.y * 64, d0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, p0 + lane);
  if (!__syncthreads_or(c >= 0)) return;
  for (int dd = wv; dd < 64; dd += 4) {
    const int d = d0 + dd;
    tile[dd][lane] = (c >= 0 && d < D) ? cols[(size_t)d * ev.ldc + c] : 0.0f;
  }
  __syncthreads();
  for (int pp = wv; pp < 64; pp += 4) {
    const int d = d0 + lane;
    if (d < D && nmx_eval_chain(ev, p0 + pp) >= 0) rows[(size_t)(p0 + pp) * D + d] = tile[lane][pp];
  }
}

__global__ __launch_bounds__(256) void k_rows_to_cols(const float* __restrict__ rows, int D, nmx_eval_batch ev,
                                                      float* __restrict__ cols) {
  __shared__ float tile[64][65];
  const int p0 = blockIdx.y * 64, d0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = nmx_eval_chain(ev, p0 + lane);
  if (!__syncthreads_or(c >= 0)) return;
  for (int pp = wv; pp < 64; pp += 4) {
    const int d = d0 + lane;
    tile[pp][lane] = (d < D && p0 + pp < ev.ldc) ? rows[(size_t)(p0 + pp) * D + d] : 0.0f;
  }
  __syncthreads();
  for (int dd = wv; dd < 64; dd += 4) {
    const int d = d0 + dd;
    if (c >= 0 && d < D) cols[(size_t)d * ev.ldc + c] = tile[lane][dd];
  }
}


// zr / gr: the evaluated chains' positions and gradients as rows [position][D].
__global__ __launch_bounds__(THREADS) void k_bnn(const float* __restrict__ X, const float* __restrict__ Y, BnnDims dm,
                                               nmx_eval_batch ev, const float* __restrict__ zr,
                                               float* __restrict__ gr, int D) {
  extern __shared__ float sm[];
  const int N = dm.N, Dx = dm.Dx, H = dm.H;
  // XCD-aware position: blocks b, b+8, b+16, ... (one XCD) take consecutive positions
  const int nb = gridDim.x;
  const int b = blockIdx.x;
  const int per = (nb + 7) / 8;
  const int pos = (b % 8) * per + b / 8;
  if (pos >= nb) return;
  const int c = nmx_eval_chain(ev, pos);
  if (c < 0) return;
  const int t = threadIdx.x;

  float* W1 = sm;                  // Dx*H
  float* W2 = W1 + Dx * H;         // H*H
  float* w3 = W2 + H * H;          // H
  float* Xs = w3 + H;              // N*Dx
  float* Ys = Xs + N * Dx;         // N
  float* h1 = Ys + N;              // N*H   (later: ga1)
  float* h2 = h1 + N * H;          // N*H   (later: ga2)
  float* gy = h2 + N * H;          // N     dU/dyhat
  float* red = gy + N;             // THREADS

  const float* z = zr + (size_t)pos * D;  // this chain's row
  float* g = gr + (size_t)pos * D;
  const float u = z[0];
  const float p = expf(u);
  float wsq = 0.0f;
  // unrolled so that a thread's loads are in flight together (a rolled loop waits on each)
#pragma unroll 4
  for (int i = t; i < Dx * H; i += THREADS) {
    const float v = z[dm.o_w1 + i];
    W1[i] = v;
    wsq += v * v;
  }
#pragma unroll 20
  for (int i = t; i < H * H; i += THREADS) {
    const float v = z[dm.o_w2 + i];
    W2[i] = v;
    wsq += v * v;
  }
  for (int i = t; i < H; i += THREADS) {
    const float v = z[dm.o_w3 + i];
    w3[i] = v;
    wsq += v * v;
  }
#pragma unroll 4
  for (int i = t; i < N * Dx; i += THREADS) Xs[i] = X[i];
  for (int i = t; i < N; i += THREADS) Ys[i] = Y[i];
  __syncthreads();

  // h1 = tanh(X W1)
  for (int e = t; e < N * H; e += THREADS) {
    const int n = e / H, j = e % H;
    float a = 0.0f;
    for (int k = 0; k < Dx; ++k) a += Xs[n * Dx + k] * W1[k * H + j];
    h1[e] = tanhf(a);
  }
  __syncthreads();

  // h2 = tanh(h1 W2): tiles over (n, j), K = i
  const int wv = t >> 6;
  const int l15 = t & 15;
  const int mtn = (N + 15) / 16, mth = (H + 15) / 16;
  for (int tile = wv; tile < mtn * mth; tile += NWAVES) {
    const int n0 = (tile / mth) * 16, j0 = (tile % mth) * 16;
    const f32x4 acc = mfma_tile16(
        H, [&](int m, int k) { return (n0 + m < N && k < H) ? h1[(n0 + m) * H + k] : 0.0f; },
        [&](int k, int c) { return (k < H && j0 + c < H) ? W2[k * H + j0 + c] : 0.0f; });
    const int j = j0 + l15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + tile_row16(r);
      if (n < N && j < H) h2[n * H + j] = tanhf(acc[r]);
    }
  }
  __syncthreads();

  // yhat = h2 w3; residual; dU/dyhat = -p (Y - yhat)
  float esq = 0.0f;
  for (int n = t; n < N; n += THREADS) {
    float yh = 0.0f;
    // sequential in j (the sum's order), unrolled so the LDS reads are issued ahead of the FMA chain
#pragma unroll 16
    for (int j = 0; j < H; ++j) yh += h2[n * H + j] * w3[j];
    const float e = Ys[n] - yh;
    esq += e * e;
    gy[n] = -p * e;
  }
  __syncthreads();

  // grad w3 = w3 + h2^T gy
  for (int j = t; j < H; j += THREADS) {
    float s = 0.0f;
#pragma unroll 16
    for (int n = 0; n < N; ++n) s += h2[n * H + j] * gy[n];
    g[dm.o_w3 + j] = w3[j] + s;
  }
  __syncthreads();
  // ga2 = (gy w3^T) * (1 - h2^2)   (in place of h2)
  for (int e = t; e < N * H; e += THREADS) {
    const int n = e / H, j = e % H;
    const float v = h2[e];
    h2[e] = gy[n] * w3[j] * (1.0f - v * v);
  }
  __syncthreads();

  // grad W2 = W2 + h1^T ga2: tiles over (i, j), K = n
  for (int tile = wv; tile < mth * mth; tile += NWAVES) {
    const int i0 = (tile / mth) * 16, j0 = (tile % mth) * 16;
    const f32x4 acc = mfma_tile16(
        N, [&](int m, int k) { return (k < N && i0 + m < H) ? h1[k * H + i0 + m] : 0.0f; },
        [&](int k, int c) { return (k < N && j0 + c < H) ? h2[k * H + j0 + c] : 0.0f; });
    const int j = j0 + l15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + tile_row16(r);
      if (i < H && j < H) g[dm.o_w2 + i * H + j] = W2[i * H + j] + acc[r];
    }
  }
  __syncthreads();

  // ga1 = (ga2 W2^T) * (1 - h1^2): tiles over (n, i), K = j, in place of h1 (a tile reads h1
  // only at its own elements; grad W2 above finished reading h1 at the barrier)
  for (int tile = wv; tile < mtn * mth; tile += NWAVES) {
    const int n0 = (tile / mth) * 16, i0 = (tile % mth) * 16;
    const f32x4 acc = mfma_tile16(
        H, [&](int m, int k) { return (n0 + m < N && k < H) ? h2[(n0 + m) * H + k] : 0.0f; },
        [&](int k, int c) { return (k < H && i0 + c < H) ? W2[(i0 + c) * H + k] : 0.0f; });
    const int i = i0 + l15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + tile_row16(r);
      if (n < N && i < H) {
        float* hp = &h1[n * H + i];
        const float hv = *hp;
        *hp = acc[r] * (1.0f - hv * hv);
      }
    }
  }
  __syncthreads();

  // grad W1 = W1 + X^T ga1
  for (int e = t; e < Dx * H; e += THREADS) {
    const int k = e / H, j = e % H;
    float s = 0.0f;
#pragma unroll 16
    for (int n = 0; n < N; ++n) s += Xs[n * Dx + k] * h1[n * H + j];
    g[dm.o_w1 + e] = W1[e] + s;
  }
  const float esq_t = block_sum256(esq, red);
  const float wsq_t = block_sum256(wsq, red);
  if (t == 0) {
    const float Nf = (float)N;
    const float nw = (float)(Dx * H + H * H + H);
    const float LOG_2PI = 1.8378770664093453f;
    float lp = -0.5f * wsq_t - 0.5f * nw * LOG_2PI;           // N(0,1) priors
    lp += 2.0f * u - p - 0.6931471805599453f + u;              // Gamma(3,1) at p (lgamma(3)=log 2) + log|J|
    lp += Nf * (0.5f * u - 0.5f * LOG_2PI) - 0.5f * p * esq_t;  // Normal(yhat, p^-1/2)
    ev.pe[c] = -lp;
    g[0] = -(3.0f - p + 0.5f * Nf - 0.5f * p * esq_t);
  }
}

// ---------------------------------------------------------------------------------------
// k_bnn_c3: the same evaluation for BASELINE config 3's shape (N = 100, Dx = 3, H = 69), with the
// three N x H x H products register-blocked.  In k_bnn every v_mfma_f32_16x16x4_f32 read both of
// its operands from LDS behind bounds checks (two reads per 32-cycle MFMA, 2-4-way bank conflicts
// at the H = 69 row stride): the products ran at MFMA-busy 0.27, bound by the LDS traffic
// (DESIGN.md, round 4).  Here:
//  * a wave computes up to 2 x 2 sub-tiles of 16 x 16 per unit, so one A and one B read feed two
//    MFMAs each (half the LDS reads per MFMA), with the whole K loop unrolled on immediate LDS
//    offsets (no address arithmetic, no bounds checks inside it);
//  * the 4 k-lanes of a step take k = 16 kq + s (s < 16; the remainder of K in groups of
//    (K - 64) / 4 after it), which puts the four lane groups of every operand read 16 banks
//    apart: with W2 stored at row stride 73 every read of the three products is conflict-free for
//    the first 64 k (2-way in the remainder; scripts/bnn_bank_pattern.py checks the pattern);
//  * K overruns are exact zeros: W2 carries three zero rows (P1's K = 72 > 69) and three zero
//    columns (P3's), and the products' other operand there reads finite values of the next row
//    (h2[0..2] are zeroed before P1 for the last row of h1); output rows / columns beyond N / H
//    read clamped rows and are never stored;
//  * units balanced over the 8 waves (largest share 5 sub-tiles of 35, 4 of 25).
// Every product is an f32 MFMA accumulation in a fixed k order (not k_bnn's order: rounding-level
// differences, tests/test_gpu_potentials.py compares both against the float64 oracle).
constexpr int C3_N = 100, C3_DX = 3, C3_H = 69;
constexpr int C3_W2S = 73;  // W2 row stride in LDS (72 rows: 69 + 3 zero rows; columns 69..72 zero)
constexpr int C3_W2R = 72;

// k index of lane group kq at step s of a K-loop over K (K % 4 == 0, K >= 64)
template <int K>
__device__ constexpr int c3_k(int kq, int s) {
  return s < 16 ? 16 * kq + s : 64 + ((K - 64) / 4) * kq + (s - 16);
}

// One unit: NA x NB sub-tiles (rows 16 (ra + a), cols 16 (cb + b)) of out = A . B with
// A(m, k) = As[m * AMS + k * AKS], B(k, n) = Bs[k * BKS + n * BNS]; rows / cols clamped to
// mmax / nmax (their outputs are not stored).  acc[a][b] register r of lane l: row
// 4 (l >> 4) + r, column l & 15 of sub-tile (a, b).
template <int K, int AMS, int AKS, int BKS, int BNS, int NA, int NB>
__device__ __forceinline__ void c3_unit(const float* As, const float* Bs, int ra, int cb, int mmax, int nmax,
                                        f32x4 (&acc)[2][2]) {
  static_assert(K % 4 == 0 && K >= 64, "c3_unit: K");
  const int lane = threadIdx.x & 63, l15 = lane & 15, kq = lane >> 4;
  const float* pa[NA];
  const float* pb[NB];
  const float* qa[NA];
  const float* qb[NB];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int m = min(16 * (ra + a) + l15, mmax);
    pa[a] = As + m * AMS + (16 * kq) * AKS;                    // main steps: k = 16 kq + s
    qa[a] = As + m * AMS + (64 + ((K - 64) / 4) * kq) * AKS;   // remainder
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int n = min(16 * (cb + b) + l15, nmax);
    pb[b] = Bs + (16 * kq) * BKS + n * BNS;
    qb[b] = Bs + (64 + ((K - 64) / 4) * kq) * BKS + n * BNS;
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int s = 0; s < K / 4; ++s) {
    float av[NA], bv[NB];
#pragma unroll
    for (int a = 0; a < NA; ++a) av[a] = s < 16 ? pa[a][s * AKS] : qa[a][(s - 16) * AKS];
#pragma unroll
    for (int b = 0; b < NB; ++b) bv[b] = s < 16 ? pb[b][s * BKS] : qb[b][(s - 16) * BKS];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
}

// units per wave: {row sub-tile, col sub-tile, NA, NB}, up to 2 per wave; NA = 0 ends the list
struct C3Unit {
  signed char ra, cb, na, nb;
};
// N x H outputs (7 x 5 sub-tiles, 35): six 2x2 units, four edge pairs, three singles; wave shares
// 5,5,5,4,4,4,4,4
__constant__ C3Unit c3_units_nh[8][2] = {
    {{0, 0, 2, 2}, {6, 2, 1, 1}}, {{0, 2, 2, 2}, {6, 3, 1, 1}}, {{2, 0, 2, 2}, {6, 4, 1, 1}},
    {{2, 2, 2, 2}, {0, 0, 0, 0}}, {{4, 0, 2, 2}, {0, 0, 0, 0}}, {{4, 2, 2, 2}, {0, 0, 0, 0}},
    {{0, 4, 2, 1}, {2, 4, 2, 1}}, {{4, 4, 2, 1}, {6, 0, 1, 2}}};
// H x H outputs (5 x 5 sub-tiles, 25): four 2x2, four edge pairs, one single; shares 4,4,4,4,3,2,2,2
__constant__ C3Unit c3_units_hh[8][2] = {
    {{0, 0, 2, 2}, {0, 0, 0, 0}}, {{0, 2, 2, 2}, {0, 0, 0, 0}}, {{2, 0, 2, 2}, {0, 0, 0, 0}},
    {{2, 2, 2, 2}, {0, 0, 0, 0}}, {{0, 4, 2, 1}, {4, 4, 1, 1}}, {{2, 4, 2, 1}, {0, 0, 0, 0}},
    {{4, 0, 1, 2}, {0, 0, 0, 0}}, {{4, 2, 1, 2}, {0, 0, 0, 0}}};

template <int K, int AMS, int AKS, int BKS, int BNS, class Store>
__device__ __forceinline__ void c3_product(const C3Unit (&units)[8][2], const float* As, const float* Bs, int mmax,
                                           int nmax, Store store) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const C3Unit un = units[wv][u];
    if (un.na == 0) break;
    f32x4 acc[2][2];
    if (un.na == 2 && un.nb == 2) c3_unit<K, AMS, AKS, BKS, BNS, 2, 2>(As, Bs, un.ra, un.cb, mmax, nmax, acc);
    else if (un.na == 2) c3_unit<K, AMS, AKS, BKS, BNS, 2, 1>(As, Bs, un.ra, un.cb, mmax, nmax, acc);
    else if (un.nb == 2) c3_unit<K, AMS, AKS, BKS, BNS, 1, 2>(As, Bs, un.ra, un.cb, mmax, nmax, acc);
    else c3_unit<K, AMS, AKS, BKS, BNS, 1, 1>(As, Bs, un.ra, un.cb, mmax, nmax, acc);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (a >= un.na || b >= un.nb) continue;
        const int col = 16 * (un.cb + b) + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) store(16 * (un.ra + a) + 4 * (lane >> 4) + r, col, acc[a][b][r]);
      }
  }
}

__global__ __launch_bounds__(THREADS, 2) void k_bnn_c3(const float* __restrict__ X, const float* __restrict__ Y,
                                                      BnnDims dm, nmx_eval_batch ev, const float* __restrict__ zr,
                                                      float* __restrict__ gr, int D) {
  constexpr int N = C3_N, Dx = C3_DX, H = C3_H;
  extern __shared__ float sm[];
  const int nb = gridDim.x;
  const int b = blockIdx.x;
  const int per = (nb + 7) / 8;
  const int pos = (b % 8) * per + b / 8;
  if (pos >= nb) return;
  const int c = nmx_eval_chain(ev, pos);
  if (c < 0) return;
  const int t = threadIdx.x;

  float* W1 = sm;                     // Dx*H
  float* W2 = W1 + Dx * H;            // C3_W2R x C3_W2S (zero rows / columns >= H)
  float* w3 = W2 + C3_W2R * C3_W2S;   // H
  float* Xs = w3 + H;                 // N*Dx
  float* Ys = Xs + N * Dx;            // N
  float* h1 = Ys + N;                 // N*H   (later: ga1)
  float* h2 = h1 + N * H;             // N*H   (later: ga2)
  float* gy = h2 + N * H;             // N     dU/dyhat
  float* red = gy + N;                // THREADS

  const float* z = zr + (size_t)pos * D;
  float* g = gr + (size_t)pos * D;
  const float u = z[0];
  const float p = expf(u);
  float wsq = 0.0f;
#pragma unroll
  for (int i = t; i < Dx * H; i += THREADS) {
    const float v = z[dm.o_w1 + i];
    W1[i] = v;
    wsq += v * v;
  }
#pragma unroll 10
  for (int i = t; i < H * H; i += THREADS) {
    const float v = z[dm.o_w2 + i];
    W2[(i / H) * C3_W2S + i % H] = v;
    wsq += v * v;
  }
  for (int i = t; i < C3_W2R * (C3_W2S - H); i += THREADS) W2[(i / (C3_W2S - H)) * C3_W2S + H + i % (C3_W2S - H)] = 0.0f;
  for (int i = t; i < (C3_W2R - H) * H; i += THREADS) W2[(H + i / H) * C3_W2S + i % H] = 0.0f;
  if (t < H) {
    const float v = z[dm.o_w3 + t];
    w3[t] = v;
    wsq += v * v;
  }
  for (int i = t; i < N * Dx; i += THREADS) Xs[i] = X[i];
  if (t < N) Ys[t] = Y[t];
  __syncthreads();

  // h1 = tanh(X W1); h2[0..2] zeroed (P1's K overrun of the last h1 row reads them)
  for (int e = t; e < N * H; e += THREADS) {
    const int n = e / H, j = e % H;
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < Dx; ++k) a += Xs[n * Dx + k] * W1[k * H + j];
    h1[e] = tanhf(a);
  }
  if (t < 3) h2[t] = 0.0f;
  __syncthreads();

  // P1: h2 = tanh(h1 W2)   (K = H padded to 72 by W2's zero rows)
  c3_product<72, H, 1, C3_W2S, 1>(c3_units_nh, h1, W2, N - 1, H - 1, [&](int n, int j, float v) {
    if (n < N && j < H) h2[n * H + j] = tanhf(v);
  });
  __syncthreads();

  // yhat = h2 w3; residual; dU/dyhat = -p (Y - yhat)
  float esq = 0.0f;
  if (t < N) {
    float yh = 0.0f;
#pragma unroll 23
    for (int j = 0; j < H; ++j) yh += h2[t * H + j] * w3[j];
    const float e = Ys[t] - yh;
    esq = e * e;
    gy[t] = -p * e;
  }
  __syncthreads();

  // grad w3 = w3 + h2^T gy
  if (t < H) {
    float sacc = 0.0f;
#pragma unroll 20
    for (int n = 0; n < N; ++n) sacc += h2[n * H + t] * gy[n];
    g[dm.o_w3 + t] = w3[t] + sacc;
  }
  __syncthreads();
  // ga2 = (gy w3^T) * (1 - h2^2)   (in place of h2)
  for (int e = t; e < N * H; e += THREADS) {
    const int n = e / H, j = e % H;
    const float v = h2[e];
    h2[e] = gy[n] * w3[j] * (1.0f - v * v);
  }
  __syncthreads();

  // P2: grad W2 = W2 + h1^T ga2   (K = N = 100)
  c3_product<N, 1, H, H, 1>(c3_units_hh, h1, h2, H - 1, H - 1, [&](int i, int j, float v) {
    if (i < H && j < H) g[dm.o_w2 + i * H + j] = W2[i * C3_W2S + j] + v;
  });
  __syncthreads();

  // P3: ga1 = (ga2 W2^T) * (1 - h1^2), in place of h1 (P3 reads ga2 and W2 only; an output
  // element is read and written by its own lane)   (K = H padded to 72 by W2's zero columns)
  c3_product<72, H, 1, 1, C3_W2S>(c3_units_nh, h2, W2, N - 1, H - 1, [&](int n, int i, float v) {
    if (n < N && i < H) {
      float* hp = &h1[n * H + i];
      const float hv = *hp;
      *hp = v * (1.0f - hv * hv);
    }
  });
  __syncthreads();

  // grad W1 = W1 + X^T ga1
  for (int e = t; e < Dx * H; e += THREADS) {
    const int k = e / H, j = e % H;
    float sacc = 0.0f;
#pragma unroll 20
    for (int n = 0; n < N; ++n) sacc += Xs[n * Dx + k] * h1[n * H + j];
    g[dm.o_w1 + e] = W1[e] + sacc;
  }
  const float esq_t = block_sum256(esq, red);
  const float wsq_t = block_sum256(wsq, red);
  if (t == 0) {
    const float Nf = (float)N;
    const float nw = (float)(Dx * H + H * H + H);
    const float LOG_2PI = 1.8378770664093453f;
    float lp = -0.5f * wsq_t - 0.5f * nw * LOG_2PI;
    lp += 2.0f * u - p - 0.6931471805599453f + u;
    lp += Nf * (0.5f * u - 0.5f * LOG_2PI) - 0.5f * p * esq_t;
    ev.pe[c] = -lp;
    g[0] = -(3.0f - p + 0.5f * Nf - 0.5f * p * esq_t);
  }
}

size_t lds_bytes_c3() {
  return sizeof(float) * ((size_t)C3_DX * C3_H + (size_t)C3_W2R * C3_W2S + C3_H + (size_t)C3_N * C3_DX + C3_N +
                          2 * (size_t)C3_N * C3_H + C3_N + THREADS);
}
bool is_c3(int N, int Dx, int H) {
#ifdef NMX_BNN_GENERIC
  return false;  // (experiments: the generic kernel at config 3's shape)
#endif
  return N == C3_N && Dx == C3_DX && H == C3_H;
}

size_t lds_bytes(int N, int Dx, int H) {
  return sizeof(float) * ((size_t)Dx * H + (size_t)H * H + H + (size_t)N * Dx + N + 2 * (size_t)N * H + N + THREADS);
}

}  // namespace


extern "C" size_t nmx_pe_bnn_workspace_bytes(int Dx, int H, int num_chains) {
  const size_t D = 1 + (size_t)Dx * H + (size_t)H * H + H;
  const size_t ldc = (size_t)(num_chains + 63) / 64 * 64;
  return 2 * ldc * D * sizeof(float);
}

extern "C" int nmx_pe_bnn(const float* X, const float* Y, int N, int Dx, int H, const nmx_eval_batch* ev,
                          void* workspace, void* stream) {
  if (!ev || !ev->z || !ev->grad || !ev->pe || !X || !Y) return nmx_fail(NMX_ERR_INVALID, "bnn: NULL operand");
  if (N <= 0 || Dx <= 0 || H <= 0) return nmx_fail(NMX_ERR_INVALID, "bnn: bad sizes");
  if (!workspace) return nmx_fail(NMX_ERR_INVALID, "bnn: NULL workspace (nmx_pe_bnn_workspace_bytes)");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains || ev->ldc % 64)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  const bool c3 = is_c3(N, Dx, H);
  const size_t lds = c3 ? lds_bytes_c3() : lds_bytes(N, Dx, H);
  if (lds > 160 * 1024)
    return nmx_fail(NMX_ERR_UNSUPPORTED, "bnn: N=%d, H=%d needs %zu bytes of LDS (> 160 KiB)", N, H, lds);
  BnnDims dm{N, Dx, H, 1, 1 + Dx * H, 1 + Dx * H + H * H};
  const void* fn = c3 ? (const void*)k_bnn_c3 : (const void*)k_bnn;
  if (const int st = nmx_lds_limit(fn, lds, (hipStream_t)stream, "bnn")) return st;
  const int D = 1 + Dx * H + H * H + H;
  float* zr = (float*)workspace;
  float* gr = zr + (size_t)ev->ldc * D;
  hipStream_t s = (hipStream_t)stream;
  const dim3 tgrid((D + 63) / 64, ev->ldc / 64);
  hipLaunchKernelGGL(k_cols_to_rows, tgrid, dim3(256), 0, s, ev->z, D, *ev, zr);
  if (c3) hipLaunchKernelGGL(k_bnn_c3, dim3(ev->ldc), dim3(THREADS), lds, s, X, Y, dm, *ev, zr, gr, D);
  else hipLaunchKernelGGL(k_bnn, dim3(ev->ldc), dim3(THREADS), lds, s, X, Y, dm, *ev, zr, gr, D);
  hipLaunchKernelGGL(k_rows_to_cols, tgrid, dim3(256), 0, s, gr, D, *ev, ev->grad);
  return nmx_check_launch("k_bnn");
}

extern "C" int nmx_pe_bnn_rows(const float* X, const float* Y, int N, int Dx, int H, const nmx_eval_batch* ev,
                               const float* z_rows, float* g_rows, void* stream) {
  if (!ev || !ev->pe || !X || !Y || !z_rows || !g_rows) return nmx_fail(NMX_ERR_INVALID, "bnn_rows: NULL operand");
  if (N <= 0 || Dx <= 0 || H <= 0) return nmx_fail(NMX_ERR_INVALID, "bnn_rows: bad sizes");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains || ev->ldc % 64)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  const bool c3 = is_c3(N, Dx, H);
  const size_t lds = c3 ? lds_bytes_c3() : lds_bytes(N, Dx, H);
  if (lds > 160 * 1024)
    return nmx_fail(NMX_ERR_UNSUPPORTED, "bnn: N=%d, H=%d needs %zu bytes of LDS (> 160 KiB)", N, H, lds);
  BnnDims dm{N, Dx, H, 1, 1 + Dx * H, 1 + Dx * H + H * H};
  const void* fn = c3 ? (const void*)k_bnn_c3 : (const void*)k_bnn;
  if (const int st = nmx_lds_limit(fn, lds, (hipStream_t)stream, "bnn")) return st;
  const int D = 1 + Dx * H + H * H + H;
  if (c3)
    hipLaunchKernelGGL(k_bnn_c3, dim3(ev->ldc), dim3(THREADS), lds, (hipStream_t)stream, X, Y, dm, *ev, z_rows,
                       g_rows, D);
  else
    hipLaunchKernelGGL(k_bnn, dim3(ev->ldc), dim3(THREADS), lds, (hipStream_t)stream, X, Y, dm, *ev, z_rows,
                       g_rows, D);
  return nmx_check_launch("k_bnn");
}
