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
  const size_t lds = lds_bytes(N, Dx, H);
  if (lds > 160 * 1024)
    return nmx_fail(NMX_ERR_UNSUPPORTED, "bnn: N=%d, H=%d needs %zu bytes of LDS (> 160 KiB)", N, H, lds);
  BnnDims dm{N, Dx, H, 1, 1 + Dx * H, 1 + Dx * H + H * H};
  if (const int st = nmx_lds_limit((const void*)k_bnn, lds, (hipStream_t)stream, "bnn")) return st;
  const int D = 1 + Dx * H + H * H + H;
  float* zr = (float*)workspace;
  float* gr = zr + (size_t)ev->ldc * D;
  hipStream_t s = (hipStream_t)stream;
  const dim3 tgrid((D + 63) / 64, ev->ldc / 64);
  hipLaunchKernelGGL(k_cols_to_rows, tgrid, dim3(256), 0, s, ev->z, D, *ev, zr);
  hipLaunchKernelGGL(k_bnn, dim3(ev->ldc), dim3(THREADS), lds, s, X, Y, dm, *ev, zr, gr, D);
  hipLaunchKernelGGL(k_rows_to_cols, tgrid, dim3(256), 0, s, gr, D, *ev, ev->grad);
  return nmx_check_launch("k_bnn");
}

extern "C" int nmx_pe_bnn_rows(const float* X, const float* Y, int N, int Dx, int H, const nmx_eval_batch* ev,
                               const float* z_rows, float* g_rows, void* stream) {
  if (!ev || !ev->pe || !X || !Y || !z_rows || !g_rows) return nmx_fail(NMX_ERR_INVALID, "bnn_rows: NULL operand");
  if (N <= 0 || Dx <= 0 || H <= 0) return nmx_fail(NMX_ERR_INVALID, "bnn_rows: bad sizes");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains || ev->ldc % 64)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  const size_t lds = lds_bytes(N, Dx, H);
  if (lds > 160 * 1024)
    return nmx_fail(NMX_ERR_UNSUPPORTED, "bnn: N=%d, H=%d needs %zu bytes of LDS (> 160 KiB)", N, H, lds);
  BnnDims dm{N, Dx, H, 1, 1 + Dx * H, 1 + Dx * H + H * H};
  if (const int st = nmx_lds_limit((const void*)k_bnn, lds, (hipStream_t)stream, "bnn")) return st;
  const int D = 1 + Dx * H + H * H + H;
  hipLaunchKernelGGL(k_bnn, dim3(ev->ldc), dim3(THREADS), lds, (hipStream_t)stream, X, Y, dm, *ev, z_rows, g_rows, D);
  return nmx_check_launch("k_bnn");
}
