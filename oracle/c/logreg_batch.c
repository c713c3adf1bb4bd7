/* ORACLE (test infrastructure only: bench.py's cpu_baseline leg) -- batched CPU restatement
 * of the covtype logistic-regression potential and its gradient for B chains at once,
 * OpenMP over row blocks, register-blocked AVX-512 GEMMs.  The product (numpyro_amd/) never
 * links this.
 *
 * Model: examples/covtype.py:66-71 (coefs ~ Normal(0, 1)^D, obs ~ Bernoulli(logits = X coefs)).
 *   U(z)    = sum_n [max(l_n, 0) + log1p(exp(-|l_n|)) - l_n y_n] + 0.5 |z|^2 + D/2 log(2 pi)
 *             (BernoulliLogits.log_prob = -binary_cross_entropy_with_logits,
 *              numpyro/distributions/discrete.py:137-139, distributions/util.py:295-298;
 *              Normal.log_prob continuous.py:2200-2204)
 *   grad U  = X^T (sigmoid(l) - y) + z
 * Same arithmetic as oracle/potentials.py LogisticRegression.pe_grad in float32, evaluated
 * for a batch of chains so that the two contractions are GEMMs (one X row block in cache
 * serves every chain): the fair multi-core CPU form of the reference's vmapped potential
 * (CPU side 2).
 *
 * Work split: a thread takes blocks of RB = 8 rows.  Per block and per chunk of 32 chains:
 *   GEMM1  L[8][32] = X[8 rows][D] . Z[D][32]   -- 16 zmm accumulators, one broadcast of
 *          X[r][d] and two Z loads per 16 FMAs;
 *   epilogue on L (vectorised exp / log1p over the 256 logits): U partials and the residual
 *          R = sigmoid(l) - y;
 *   GEMM2  G[d][32] += sum_r X[r][d] R[r][32]  -- R held in 16 zmm over the d loop, G (the
 *          thread's [D][Bp] partial, L1-resident) loaded and stored once per d.
 * Per-thread partials are reduced in a fixed thread order (U in double).
 *
 * Layout: X [N][D] row-major f32, y [N] f32, Zt [D][B] (chain-minor), outputs pe [B],
 * Gt [D][B].  B is padded internally to a multiple of 32 chains.
 */
#include <immintrin.h>
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#define RB 8  /* rows per block */
#define CB 32 /* chains per register block (two zmm) */

int nmx_cpu_threads(void) { return omp_get_max_threads(); }

static inline void gemm1(const float* x /* [RB][D] */, int D, const float* z /* Zp + b0, stride Bp */,
                         int Bp, float* L /* [RB][CB] */) {
  __m512 a[RB][2];
  for (int r = 0; r < RB; ++r) a[r][0] = a[r][1] = _mm512_setzero_ps();
  for (int d = 0; d < D; ++d) {
    const __m512 z0 = _mm512_loadu_ps(z + (size_t)d * Bp);
    const __m512 z1 = _mm512_loadu_ps(z + (size_t)d * Bp + 16);
    for (int r = 0; r < RB; ++r) {
      const __m512 xb = _mm512_set1_ps(x[(size_t)r * D + d]);
      a[r][0] = _mm512_fmadd_ps(xb, z0, a[r][0]);
      a[r][1] = _mm512_fmadd_ps(xb, z1, a[r][1]);
    }
  }
  for (int r = 0; r < RB; ++r) {
    _mm512_storeu_ps(L + r * CB, a[r][0]);
    _mm512_storeu_ps(L + r * CB + 16, a[r][1]);
  }
}

static inline void gemm2(const float* x /* [RB][D] */, int D, const float* R /* [RB][CB] */,
                         float* g /* partial + b0, stride Bp */, int Bp) {
  __m512 rr[RB][2];
  for (int r = 0; r < RB; ++r) {
    rr[r][0] = _mm512_loadu_ps(R + r * CB);
    rr[r][1] = _mm512_loadu_ps(R + r * CB + 16);
  }
  for (int d = 0; d < D; ++d) {
    float* gd = g + (size_t)d * Bp;
    __m512 g0 = _mm512_loadu_ps(gd), g1 = _mm512_loadu_ps(gd + 16);
    for (int r = 0; r < RB; ++r) {
      const __m512 xb = _mm512_set1_ps(x[(size_t)r * D + d]);
      g0 = _mm512_fmadd_ps(xb, rr[r][0], g0);
      g1 = _mm512_fmadd_ps(xb, rr[r][1], g1);
    }
    _mm512_storeu_ps(gd, g0);
    _mm512_storeu_ps(gd + 16, g1);
  }
}

void nmx_cpu_logreg_pe_grad(const float* X, const float* y, long N, int D, const float* Zt, int B,
                            float* pe, float* Gt) {
  const int T = omp_get_max_threads();
  const int Bp = (B + CB - 1) / CB * CB;
  float* Zp = (float*)calloc((size_t)D * Bp, sizeof(float));
  for (int d = 0; d < D; ++d) memcpy(Zp + (size_t)d * Bp, Zt + (size_t)d * B, sizeof(float) * B);
  double* pe_part = (double*)calloc((size_t)T * Bp, sizeof(double));
  float* g_part = (float*)calloc((size_t)T * D * Bp, sizeof(float));
  const long nblk = (N + RB - 1) / RB;
#pragma omp parallel
  {
    const int tid = omp_get_thread_num();
    double* pp = pe_part + (size_t)tid * Bp;
    float* gp = g_part + (size_t)tid * D * Bp;
    float L[RB * CB], ub[CB];
    float* xt = (float*)calloc((size_t)RB * D, sizeof(float)); /* zero-padded tail block */
    float yt[RB];
#pragma omp for schedule(static)
    for (long blk = 0; blk < nblk; ++blk) {
      const long r0 = blk * RB;
      const int nr = (int)((N - r0) < RB ? (N - r0) : RB);
      const float* x = X + (size_t)r0 * D;
      const float* yb = y + r0;
      if (nr < RB) {
        memset(xt, 0, sizeof(float) * RB * D);
        memcpy(xt, x, sizeof(float) * nr * D);
        for (int r = 0; r < RB; ++r) yt[r] = r < nr ? yb[r] : 0.0f;
        x = xt;
        yb = yt;
      }
      for (int b0 = 0; b0 < Bp; b0 += CB) {
        gemm1(x, D, Zp + b0, Bp, L);
        for (int b = 0; b < CB; ++b) ub[b] = 0.0f;
        for (int r = 0; r < nr; ++r) {
          const float yv = yb[r];
          float* l = L + r * CB;
#pragma omp simd
          for (int b = 0; b < CB; ++b) {
            const float lv = l[b];
            const float e = expf(-fabsf(lv));
            ub[b] += fmaxf(lv, 0.0f) + log1pf(e) - lv * yv;
            const float sig = lv >= 0.0f ? 1.0f / (1.0f + e) : e / (1.0f + e);
            l[b] = sig - yv;
          }
        }
        for (int r = nr; r < RB; ++r)
          for (int b = 0; b < CB; ++b) L[r * CB + b] = 0.0f;
        for (int b = 0; b < CB; ++b) pp[b0 + b] += (double)ub[b];
        gemm2(x, D, L, gp + b0, Bp);
      }
    }
    free(xt);
  }
  /* fixed-order reduction over threads, then the prior terms */
  const double half_log_2pi = 0.91893853320467274178;
  for (int b = 0; b < B; ++b) {
    double u = 0.0;
    for (int t = 0; t < T; ++t) u += pe_part[(size_t)t * Bp + b];
    double zz = 0.0;
    for (int d = 0; d < D; ++d) zz += (double)Zt[(size_t)d * B + b] * Zt[(size_t)d * B + b];
    pe[b] = (float)(u + 0.5 * zz + D * half_log_2pi);
  }
  for (int d = 0; d < D; ++d)
    for (int b = 0; b < B; ++b) {
      float g = Zt[(size_t)d * B + b];
      for (int t = 0; t < T; ++t) g += g_part[((size_t)t * D + d) * Bp + b];
      Gt[(size_t)d * B + b] = g;
    }
  free(Zp);
  free(pe_part);
  free(g_part);
}
