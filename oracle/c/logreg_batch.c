/* ORACLE (test infrastructure only: bench.py's cpu_baseline leg) -- batched CPU restatement
 * of the covtype logistic-regression potential and its gradient for B chains at once,
 * OpenMP over row blocks.  The product (numpyro_amd/) never links this.
 *
 * Model: examples/covtype.py:66-71 (coefs ~ Normal(0, 1)^D, obs ~ Bernoulli(logits = X coefs)).
 *   U(z)    = sum_n [max(l_n, 0) + log1p(exp(-|l_n|)) - l_n y_n] + 0.5 |z|^2 + D/2 log(2 pi)
 *             (BernoulliLogits.log_prob = -binary_cross_entropy_with_logits,
 *              numpyro/distributions/discrete.py:137-139, distributions/util.py:295-298;
 *              Normal.log_prob continuous.py:2200-2204)
 *   grad U  = X^T (sigmoid(l) - y) + z
 * Same arithmetic as oracle/potentials.py LogisticRegression.pe_grad in float32, evaluated
 * for a batch of chains so that the two contractions are GEMMs (one X row block in cache
 * serves every chain), which is the fair multi-core CPU form of the reference's vmapped
 * potential (CPU side 2).
 *
 * Layout: X [N][D] row-major f32, y [N] f32, Zt [D][B] (chain-minor, so the inner loops run
 * over chains and vectorise), outputs pe [B] (double accumulation per thread, f32 result),
 * Gt [D][B].
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define RB 64 /* rows per block */

int nmx_cpu_threads(void) { return omp_get_max_threads(); }

void nmx_cpu_logreg_pe_grad(const float* X, const float* y, long N, int D, const float* Zt, int B,
                            float* pe, float* Gt) {
  const int T = omp_get_max_threads();
  double* pe_part = (double*)calloc((size_t)T * B, sizeof(double));
  float* g_part = (float*)calloc((size_t)T * D * B, sizeof(float));
#pragma omp parallel
  {
    const int tid = omp_get_thread_num();
    double* pp = pe_part + (size_t)tid * B;
    float* gp = g_part + (size_t)tid * D * B;
    float* L = (float*)malloc(sizeof(float) * RB * B);
    float* ub = (float*)malloc(sizeof(float) * B);
#pragma omp for schedule(static)
    for (long r0 = 0; r0 < N; r0 += RB) {
      const int nr = (int)((N - r0) < RB ? (N - r0) : RB);
      for (int b = 0; b < B; ++b) ub[b] = 0.0f;
      for (int r = 0; r < nr; ++r) {
        /* logits L[r][b] = sum_d X[r][d] Zt[d][b] */
        float* l = L + (size_t)r * B;
        const float* x = X + (size_t)(r0 + r) * D;
        for (int b = 0; b < B; ++b) l[b] = 0.0f;
        for (int d = 0; d < D; ++d) {
          const float xv = x[d];
          const float* z = Zt + (size_t)d * B;
#pragma omp simd
          for (int b = 0; b < B; ++b) l[b] += xv * z[b];
        }
        /* epilogue: BCE-with-logits into U, residual sigmoid(l) - y in place */
        const float yv = y[r0 + r];
#pragma omp simd
        for (int b = 0; b < B; ++b) {
          const float lv = l[b];
          const float e = expf(-fabsf(lv));
          ub[b] += fmaxf(lv, 0.0f) + log1pf(e) - lv * yv;
          const float sig = lv >= 0.0f ? 1.0f / (1.0f + e) : e / (1.0f + e);
          l[b] = sig - yv;
        }
      }
      for (int b = 0; b < B; ++b) pp[b] += (double)ub[b];
      /* gradient G[d][b] += X[r][d] R[r][b] */
      for (int r = 0; r < nr; ++r) {
        const float* x = X + (size_t)(r0 + r) * D;
        const float* rr = L + (size_t)r * B;
        for (int d = 0; d < D; ++d) {
          const float xv = x[d];
          float* g = gp + (size_t)d * B;
#pragma omp simd
          for (int b = 0; b < B; ++b) g[b] += xv * rr[b];
        }
      }
    }
    free(L);
    free(ub);
  }
  /* fixed-order reduction over threads, then the prior terms */
  const double half_log_2pi = 0.91893853320467274178;
  for (int b = 0; b < B; ++b) {
    double u = 0.0;
    for (int t = 0; t < T; ++t) u += pe_part[(size_t)t * B + b];
    double zz = 0.0;
    for (int d = 0; d < D; ++d) zz += (double)Zt[(size_t)d * B + b] * Zt[(size_t)d * B + b];
    pe[b] = (float)(u + 0.5 * zz + D * half_log_2pi);
  }
  for (int d = 0; d < D; ++d)
    for (int b = 0; b < B; ++b) {
      float g = Zt[(size_t)d * B + b];
      for (int t = 0; t < T; ++t) g += g_part[((size_t)t * D + d) * B + b];
      Gt[(size_t)d * B + b] = g;
    }
  free(pe_part);
  free(g_part);
}
