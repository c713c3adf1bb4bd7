// Potentials of small-D models: one thread per chain, coordinates loop in registers.
#include <math.h>

#include "nmx_api_internal.h"
#include "nmx_common.h"

namespace {

__global__ void k_diag_normal(const float* mu, const float* prec, int D, nmx_eval_batch ev) {
  const int c = nmx_eval_chain(ev, blockIdx.x * blockDim.x + threadIdx.x);
  if (c < 0) return;
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

// Normal.log_prob (numpyro/distributions/continuous.py:2200-2204) negated, as U terms.
__device__ __forceinline__ float nlpN(float x, float loc, float scale) {
  const float v = (x - loc) / scale;
  return 0.5f * v * v + logf(2.5066282746310002f * scale);
}

// z = (mu, u = log tau, theta[J]); SURVEY.md Appendix A, C0.
__global__ void k_eight_schools(const float* y, const float* sigma, int J, nmx_eval_batch ev) {
  const int c = nmx_eval_chain(ev, blockIdx.x * blockDim.x + threadIdx.x);
  if (c < 0) return;
  const int ldc = ev.ldc;
  const float mu = ev.z[c];
  const float u = ev.z[(size_t)ldc + c];
  const float tau = expf(u);
  const float tau2 = tau * tau;
  float U = nlpN(mu, 0.0f, 5.0f);
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
    U += nlpN(th, mu, tau) + nlpN(y[jj], th, sigma[jj]);
    g_mu -= dt / tau2;
    g_u -= dt * dt / tau2 - 1.0f;
    ev.grad[idx] = dt / tau2 + (th - y[jj]) / (sigma[jj] * sigma[jj]);
  }
  ev.grad[c] = g_mu;
  ev.grad[(size_t)ldc + c] = g_u;
  ev.pe[c] = U;
}

int check_ev(const nmx_eval_batch* ev) {
  if (!ev || !ev->z || !ev->grad || !ev->pe) return nmx_fail(NMX_ERR_INVALID, "eval batch has NULL pointers");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  return NMX_OK;
}

}  // namespace

extern "C" int nmx_pe_diag_normal(const float* mu, const float* prec, int dim, const nmx_eval_batch* ev,
                                  void* stream) {
  if (int st = check_ev(ev)) return st;
  if (!mu || !prec || dim <= 0) return nmx_fail(NMX_ERR_INVALID, "bad diag_normal parameters");
  hipLaunchKernelGGL(k_diag_normal, dim3((ev->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     mu, prec, dim, *ev);
  return nmx_check_launch("k_diag_normal");
}

extern "C" int nmx_pe_eight_schools(const float* y, const float* sigma, int J, const nmx_eval_batch* ev,
                                    void* stream) {
  if (int st = check_ev(ev)) return st;
  if (!y || !sigma || J <= 0) return nmx_fail(NMX_ERR_INVALID, "bad eight_schools data");
  hipLaunchKernelGGL(k_eight_schools, dim3((ev->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     y, sigma, J, *ev);
  return nmx_check_launch("k_eight_schools");
}
