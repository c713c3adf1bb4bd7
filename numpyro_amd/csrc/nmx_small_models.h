// Per-chain potential + gradient of the small-D models, shared by their launched kernels
// (potential_small.hip) and the persistent NUTS kernel (nuts.hip, k_nuts_persistent): the
// same device code, so both schedules draw bitwise the same samples.
#pragma once
#include <math.h>

#include "nmx_common.h"

// Normal.log_prob (numpyro/distributions/continuous.py:2200-2204) negated, as U terms.
__device__ __forceinline__ float nmx_nlpN(float x, float loc, float scale) {
  const float v = (x - loc) / scale;
  return 0.5f * v * v + logf(2.5066282746310002f * scale);
}

// U = 0.5 sum_d prec_d (z_d - mu_d)^2 (test/infer/test_mcmc.py:28-72 target)
struct NmxDiagNormal {
  const float* mu;
  const float* prec;
  int D;
  __device__ __forceinline__ void operator()(const nmx_eval_batch& ev, int c) const {
    float u = 0.0f;
    for (int d = 0; d < D; ++d) {
      const size_t idx = (size_t)d * ev.ldc + c;
      const float dz = ev.z[idx] - mu[d];
      const float g = dz * prec[d];
      u += 0.5f * dz * g;
      ev.grad[idx] = g;
    }
    ev.pe[c] = u;
  }
};

// Eight schools (README.md:47-55), z = (mu, u = log tau, theta[J]); SURVEY.md Appendix A, C0.
struct NmxEightSchools {
  const float* y;
  const float* sigma;
  int J;
  __device__ __forceinline__ void operator()(const nmx_eval_batch& ev, int c) const {
    const int ldc = ev.ldc;
    const float mu = ev.z[c];
    const float u = ev.z[(size_t)ldc + c];
    const float tau = expf(u);
    const float tau2 = tau * tau;
    float U = nmx_nlpN(mu, 0.0f, 5.0f);
    // HalfCauchy(5).log_prob = -log(pi) - log(5) - log1p((x/5)^2) + log(2)  (continuous.py:720-722)
    const float x5 = tau / 5.0f;
    U += 1.1447298858494002f + 1.6094379124341003f + log1pf(x5 * x5) - 0.6931471805599453f;
    U -= u;  // ExpTransform log|J|
    float g_mu = mu / 25.0f;
    float g_u = (2.0f * tau2 / 25.0f) / (1.0f + tau2 / 25.0f) - 1.0f;
    for (int jj = 0; jj < J; ++jj) {
      const size_t idx = (size_t)(2 + jj) * ldc + c;
      const float th = ev.z[idx];
      const float dt = th - mu;
      U += nmx_nlpN(th, mu, tau) + nmx_nlpN(y[jj], th, sigma[jj]);
      g_mu -= dt / tau2;
      g_u -= dt * dt / tau2 - 1.0f;
      ev.grad[idx] = dt / tau2 + (th - y[jj]) / (sigma[jj] * sigma[jj]);
    }
    ev.grad[c] = g_mu;
    ev.grad[(size_t)ldc + c] = g_u;
    ev.pe[c] = U;
  }
};
