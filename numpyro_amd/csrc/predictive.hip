// Posterior predictive draws of the observed sites of the fused models
// (numpyro/infer/util.py:888-1090 Predictive; _predictive :803-885 runs the model with the
// latent sites substituted from each posterior sample and samples the rest).  One kernel per
// model draws every observed site for every posterior sample on the device.
//
// Randomness: Philox4x32-10 keyed by the seed (nmx_common.h), counter = (sample index, site
// id, NMX_EV_PREDICT << 24 | element index, attempt) -- a draw depends only on (seed,
// sample, element), not on the launch shape.  The reference draws from jax.random under
// split keys; that stream is not reproduced (PRNG parity unpinned), the
// distributions are (tests/test_gpu_predictive.py).
#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

constexpr uint32_t NMX_EV_PREDICT = 7u;

__device__ __forceinline__ nmx_u4 pred_rng(uint64_t seed, int s, int site, int64_t idx, uint32_t sub) {
  return nmx_rng(seed, (uint32_t)s, (uint32_t)site, NMX_EV_PREDICT, (uint32_t)idx, sub);
}

// covtype (examples/covtype.py:66-71): obs ~ Bernoulli(logits = data . coefs).  Block =
// 256 rows of one sample; the sample's coefficients in LDS.
__global__ __launch_bounds__(256) void k_predict_logreg(const float* __restrict__ X, int64_t N, int D,
                                                        const float* __restrict__ coefs, uint64_t seed,
                                                        int32_t* __restrict__ out) {
  __shared__ float w[64];
  const int s = blockIdx.y;
  if (threadIdx.x < D) w[threadIdx.x] = coefs[(size_t)s * D + threadIdx.x];
  __syncthreads();
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* x = X + n * D;
  float l = 0.0f;
  for (int d = 0; d < D; ++d) l = __builtin_fmaf(x[d], w[d], l);
  const float p = 1.0f / (1.0f + expf(-l));  // expit (BernoulliLogits.probs)
  const nmx_u4 r = pred_rng(seed, s, 0, n, 0);
  out[(size_t)s * N + n] = nmx_u01(r.x) < p ? 1 : 0;  // random.bernoulli: U < p
}

// Normal(loc, scale) with per-sample loc [S][J] and per-element scale [J] (eight schools:
// obs ~ Normal(theta, sigma), README.md:47-55).
__global__ void k_predict_normal(const float* __restrict__ loc, const float* __restrict__ scale, int J, int S,
                                 uint64_t seed, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)S * J) return;
  const int s = (int)(i / J), j = (int)(i % J);
  const nmx_u4 r = pred_rng(seed, s, 0, j, 0);
  float z, unused;
  nmx_box_muller(r.x, r.y, z, unused);
  out[i] = loc[i] + scale[j] * z;
}

// BNN (examples/bnn.py:43-74): Y ~ Normal(tanh(tanh(X w1) w2) w3, 1 / sqrt(prec_obs)).
// One 256-thread workgroup per sample: weights and both activation layers in LDS.
// Sample layout (sorted sites): prec_obs, w1 [Dx][H], w2 [H][H], w3 [H][Dy].
__global__ __launch_bounds__(256) void k_predict_bnn(const float* __restrict__ X, int N, int Dx, int H, int Dy,
                                                     const float* __restrict__ samples, int D, uint64_t seed,
                                                     float* __restrict__ out) {
  extern __shared__ float sm[];
  const int s = blockIdx.x;
  const float* smp = samples + (size_t)s * D;
  float* w1 = sm;
  float* w2 = w1 + Dx * H;
  float* w3 = w2 + H * H;
  float* z1 = w3 + H * Dy;
  float* z2 = z1 + N * H;
  for (int i = threadIdx.x; i < Dx * H + H * H + H * Dy; i += blockDim.x) w1[i] = smp[1 + i];
  __syncthreads();
  for (int i = threadIdx.x; i < N * H; i += blockDim.x) {
    const int n = i / H, h = i % H;
    float a = 0.0f;
    for (int k = 0; k < Dx; ++k) a = __builtin_fmaf(X[n * Dx + k], w1[k * H + h], a);
    z1[i] = tanhf(a);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N * H; i += blockDim.x) {
    const int n = i / H, h = i % H;
    float a = 0.0f;
    for (int k = 0; k < H; ++k) a = __builtin_fmaf(z1[n * H + k], w2[k * H + h], a);
    z2[i] = tanhf(a);
  }
  __syncthreads();
  const float sigma = 1.0f / sqrtf(smp[0]);
  for (int i = threadIdx.x; i < N * Dy; i += blockDim.x) {
    const int n = i / Dy, y = i % Dy;
    float a = 0.0f;
    for (int k = 0; k < H; ++k) a = __builtin_fmaf(z2[n * H + k], w3[k * Dy + y], a);
    const nmx_u4 r = pred_rng(seed, s, 0, i, 0);
    float z, unused;
    nmx_box_muller(r.x, r.y, z, unused);
    out[(size_t)s * N * Dy + i] = a + sigma * z;
  }
}

size_t bnn_lds_bytes(int N, int Dx, int H, int Dy) {
  return sizeof(float) * ((size_t)Dx * H + (size_t)H * H + (size_t)H * Dy + 2 * (size_t)N * H);
}

}  // namespace

extern "C" int nmx_predict_logreg(const float* X, int64_t n_rows, int dim, const float* coefs, int num_samples,
                                  uint64_t seed, int32_t* out, void* stream) {
  if (!X || !coefs || !out) return nmx_fail(NMX_ERR_INVALID, "predict_logreg: NULL pointer");
  if (n_rows <= 0 || dim <= 0 || dim > 64 || num_samples <= 0 || num_samples > 65535)
    return nmx_fail(NMX_ERR_INVALID, "predict_logreg: need n_rows > 0, 0 < dim <= 64, 0 < samples < 65536");
  if (n_rows > 0x00FFFFFF) return nmx_fail(NMX_ERR_INVALID, "predict_logreg: at most 2^24 rows per call");
  const dim3 grid((unsigned)((n_rows + 255) / 256), num_samples);
  hipLaunchKernelGGL(k_predict_logreg, grid, dim3(256), 0, (hipStream_t)stream, X, n_rows, dim, coefs, seed, out);
  return nmx_check_launch("k_predict_logreg");
}

extern "C" int nmx_predict_normal(const float* loc, const float* scale, int n, int num_samples, uint64_t seed,
                                  float* out, void* stream) {
  if (!loc || !scale || !out) return nmx_fail(NMX_ERR_INVALID, "predict_normal: NULL pointer");
  if (n <= 0 || n > 0x00FFFFFF || num_samples <= 0)
    return nmx_fail(NMX_ERR_INVALID, "predict_normal: need 0 < n < 2^24 and num_samples > 0");
  const int64_t total = (int64_t)n * num_samples;
  hipLaunchKernelGGL(k_predict_normal, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, loc,
                     scale, n, num_samples, seed, out);
  return nmx_check_launch("k_predict_normal");
}

extern "C" int nmx_predict_bnn(const float* X, int n, int dx, int dh, int dy, const float* samples, int num_samples,
                               uint64_t seed, float* out, void* stream) {
  if (!X || !samples || !out) return nmx_fail(NMX_ERR_INVALID, "predict_bnn: NULL pointer");
  if (n <= 0 || dx <= 0 || dh <= 0 || dy <= 0 || num_samples <= 0 || (int64_t)n * dy > 0x00FFFFFF)
    return nmx_fail(NMX_ERR_INVALID, "predict_bnn: bad sizes");
  const size_t lds = bnn_lds_bytes(n, dx, dh, dy);
  if (lds > 160 * 1024)
    return nmx_fail(NMX_ERR_INVALID, "predict_bnn: weights + activations need %zu B of LDS (> 160 KB)", lds);
  if (const int st = nmx_lds_limit((const void*)k_predict_bnn, 160 * 1024, (hipStream_t)stream, "predict_bnn"))
    return st;
  const int D = 1 + dx * dh + dh * dh + dh * dy;
  hipLaunchKernelGGL(k_predict_bnn, dim3(num_samples), dim3(256), lds, (hipStream_t)stream, X, n, dx, dh, dy, samples,
                     D, seed, out);
  return nmx_check_launch("k_predict_bnn");
}
