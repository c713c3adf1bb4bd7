/* ORACLE (test infrastructure only: bench.py's cpu_baseline legs and tests/) -- C restatement of
 * numpyro's NUTS sample kernel for many chains on the CPU cores, with the benchmark models'
 * potentials in C: the CPU side of SURVEY.md §8d ("the build's own C++ CPU restatement of the same
 * lockstep NUTS and the same fused potentials, OpenMP over chains").  The product (numpyro_amd/)
 * never links this.
 *
 * Sampler (sampling phase: fixed step size, diagonal inverse mass; dense mass runs as identity-mass
 * NUTS on whitened coordinates w, z = mu + T w, exactly as the device does):
 *   numpyro/infer/hmc.py:459-530 sample_kernel (momentum hmc.py:92-110: r = mass_matrix_sqrt * eps),
 *   numpyro/infer/hmc_util.py:1088-1180 build_tree, :984-1085 _iterative_build_subtree,
 *   :851-894 _build_basetree, :767-848 _combine_tree (:749-764 the two transition kernels),
 *   :941-981 checkpoints and the iterative U-turn check, :710-746 _is_turning,
 *   :262-311 velocity_verlet, :1183-1220 the Euclidean kinetic energy;
 * statement by statement as oracle/hmc_ref.py restates them, on the same Philox4x32-10 stream
 * (oracle/philox.py, csrc/nmx_common.h): counter (global chain id, transition, event << 24 | index,
 * sub), so a chain here takes the device's and the NumPy oracle's trajectory up to float32
 * rounding (tests/test_cpu_nuts.py).  Reductions (kinetic energy, U-turn dots) accumulate in double.
 *
 * Schedule: every chain is a state machine advanced leaf by leaf (per-chain asynchronous, like the
 * device engine: a chain whose tree ends starts its next transition at once); each round evaluates
 * the potential of every chain with a leaf in flight in ONE batched call -- covtype's two GEMMs over
 * the full data (logreg_batch.c, register-blocked AVX-512), the whitening GEMMs, or one chain per
 * OpenMP thread for the elementwise models -- then advances every chain (OpenMP over chains).
 * Compiled without -ffast-math (oracle/build.py FILE_FLAGS): the NaN -> +inf energy rule and the
 * float32 operation order of the sampler arithmetic are kept.
 *
 * Models (numpyro_amd/potentials.py; oracle/potentials.py float64 forms pinned against scipy):
 *   1 covtype logistic regression (examples/covtype.py:66-71)
 *   2 funnel, centred (examples/funnel.py:44-46)
 *   3 stochastic volatility (examples/stochastic_volatility.py:57-65)
 *   4 BNN (examples/bnn.py:43-74)
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* logreg_batch.c (linked: liblogreg_batch.so, built with -ffast-math for its vector exp / log1p;
 * this file keeps IEEE semantics so NaN energies map to +inf as the reference does) */
void nmx_cpu_logreg_pe_grad(const float* X, const float* y, long N, int D, const float* Zt, int B, float* pe,
                            float* Gt);
int nmx_cpu_threads(void);

#define NMX_PI 3.14159265358979323846

#define LOG_2PI 1.8378770664093453
#define MAXD 12

typedef struct {
  int model; /* 1 covtype, 2 funnel, 3 SV, 4 BNN */
  int dim;
  const float* X; /* covtype: X [N][D], y [N]; BNN: X [N][Dx], Y [N] */
  const float* y;
  long n;
  int bnn_dx, bnn_h;
  const float* r2; /* SV: squared returns [T] */
  const float* wT; /* dense mass: whitening T [D][D] row-major (NULL: none), mu [D] */
  const float* wmu;
} nmx_cpu_model;

/* ------------------------------------------------------------------------------- Philox */
static inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
enum { EV_MOMENTUM = 1, EV_DIRECTION = 2, EV_BIASED = 3, EV_LEAF = 4 };
static inline void rng(uint64_t seed, uint32_t chain, uint32_t it, uint32_t ev, uint32_t idx, uint32_t sub,
                       uint32_t out[4]) {
  out[0] = chain;
  out[1] = it;
  out[2] = (ev << 24) | (idx & 0x00FFFFFFu);
  out[3] = sub;
  philox4x32_10(out, (uint32_t)seed, (uint32_t)(seed >> 32));
}
static inline float u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }
static inline float u01_open0(uint32_t x) { return ((float)(x >> 8) + 1.0f) * 5.9604644775390625e-08f; }
static inline float uniform(uint64_t seed, uint32_t ch, uint32_t it, uint32_t ev, uint32_t idx, uint32_t sub) {
  uint32_t o[4];
  rng(seed, ch, it, ev, idx, sub, o);
  return u01(o[0]);
}
static inline void box_muller(uint32_t a, uint32_t b, float* x, float* y) {
  const double u1 = (double)u01_open0(a), u2 = (double)u01(b);
  const double rad = sqrt(-2.0 * log(u1)), ang = 2.0 * NMX_PI * u2;
  *x = (float)(rad * cos(ang));
  *y = (float)(rad * sin(ang));
}

/* ----------------------------------------------------------------------------- potentials */
static double digamma(double x) {
  double r = 0.0;
  while (x < 6.0) {
    r -= 1.0 / x;
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  return r + log(x) - 0.5 / x - f * (1.0 / 12 - f * (1.0 / 120 - f * (1.0 / 252 - f * (1.0 / 240 - f / 132))));
}

static void pe_funnel(int D, const float* z, float* pe, float* g) {
  const int K = D - 1;
  const float y = z[K], e = expf(-y);
  double xx = 0.0;
#pragma omp simd reduction(+ : xx)
  for (int i = 0; i < K; ++i) xx += (double)z[i] * z[i];
  for (int i = 0; i < K; ++i) g[i] = z[i] * e;
  g[K] = (float)(y / 9.0 + 0.5 * K - 0.5 * e * xx);
  *pe = (float)(y * (double)y / 18.0 + log(3.0) + 0.5 * LOG_2PI + 0.5 * e * xx + K * (0.5 * y + 0.5 * LOG_2PI));
}

static void pe_sv(const float* r2, int T, const float* z, float* pe, float* g) {
  const double a = z[0], b = z[T + 1], nu = exp(a), sigma = exp(b), s2 = sigma * sigma;
  const float* s = z + 1;
  double dd = 0.0, l1q = 0.0, qq = 0.0, ss = 0.0;
  for (int t = 0; t < T; ++t) {
    const float d = s[t] - (t ? s[t - 1] : 0.0f);
    const float dn = t + 1 < T ? s[t + 1] - s[t] : 0.0f;
    const float q = (float)(r2[t] * expf(-2.0f * s[t]) / nu);
    const float qr = q / (1.0f + q);
    dd += (double)d * d;
    l1q += log1pf(q);
    qq += qr;
    ss += s[t];
    g[1 + t] = -(float)(-(d - dn) / s2 + (nu + 1.0) * qr - 1.0);
  }
  const double lg = lgamma(0.5 * nu) - lgamma(0.5 * (nu + 1.0));
  double lp = log(50.0) - 50.0 * sigma + b - 0.5 * dd / s2 - T * b - 0.5 * T * LOG_2PI;
  lp += log(0.1) - 0.1 * nu + a - 0.5 * (nu + 1.0) * l1q - ss - T * (0.5 * a + 0.5 * log(NMX_PI) + lg);
  const double gb = -50.0 * sigma + 1.0 + dd / s2 - T;
  const double dg = digamma(0.5 * (nu + 1.0)) - digamma(0.5 * nu);
  const double ga = nu * (-0.1 - 0.5 * l1q + 0.5 * (nu + 1.0) / nu * qq + T * (-0.5 / nu + 0.5 * dg)) + 1.0;
  g[0] = (float)-ga;
  g[T + 1] = (float)-gb;
  *pe = (float)-lp;
}

/* BNN: z = (u, w1 [Dx][H], w2 [H][H], w3 [H]); work: h1, h2, ga [N][H] */
static void pe_bnn(const nmx_cpu_model* m, const float* z, float* pe, float* g, float* work) {
  const int N = (int)m->n, Dx = m->bnn_dx, H = m->bnn_h, D = m->dim;
  const float* X = m->X;
  const float* Y = m->y;
  const float u = z[0], *w1 = z + 1, *w2 = w1 + Dx * H, *w3 = w2 + H * H;
  float *h1 = work, *h2 = h1 + (size_t)N * H, *ga = h2 + (size_t)N * H, *e = ga + (size_t)N * H;
  const double p = exp((double)u);
  for (int n = 0; n < N; ++n) {
    float* a = h1 + (size_t)n * H;
    for (int k = 0; k < H; ++k) a[k] = 0.0f;
    for (int i = 0; i < Dx; ++i)
      for (int k = 0; k < H; ++k) a[k] += X[n * Dx + i] * w1[i * H + k];
    for (int k = 0; k < H; ++k) a[k] = tanhf(a[k]);
  }
  double ee = 0.0;
  for (int n = 0; n < N; ++n) {
    const float* a1 = h1 + (size_t)n * H;
    float* a2 = h2 + (size_t)n * H;
    for (int k = 0; k < H; ++k) a2[k] = 0.0f;
    for (int i = 0; i < H; ++i)
      for (int k = 0; k < H; ++k) a2[k] += a1[i] * w2[i * H + k];
    float yh = 0.0f;
    for (int k = 0; k < H; ++k) {
      a2[k] = tanhf(a2[k]);
      yh += a2[k] * w3[k];
    }
    e[n] = Y[n] - yh;
    ee += (double)e[n] * e[n];
  }
  double ww = 0.0;
  for (int i = 1; i < D; ++i) ww += (double)z[i] * z[i];
  const double lp = -0.5 * ww - 0.5 * (D - 1) * LOG_2PI + 2.0 * u - p - lgamma(3.0) + u - 0.5 * p * ee +
                    0.5 * N * u - 0.5 * N * LOG_2PI;
  float *g1 = g + 1, *g2 = g1 + Dx * H, *g3 = g2 + H * H;
  for (int k = 0; k < H; ++k) g3[k] = w3[k];
  for (int i = 0; i < H * H; ++i) g2[i] = w2[i];
  for (int i = 0; i < Dx * H; ++i) g1[i] = w1[i];
  for (int n = 0; n < N; ++n) {
    const float gy = (float)(-p * e[n]);
    const float* a2 = h2 + (size_t)n * H;
    float* gn = ga + (size_t)n * H;
    for (int k = 0; k < H; ++k) {
      g3[k] += a2[k] * gy;
      gn[k] = gy * w3[k] * (1.0f - a2[k] * a2[k]); /* g_a2 */
    }
  }
  for (int n = 0; n < N; ++n) {
    const float* a1 = h1 + (size_t)n * H;
    const float* gn = ga + (size_t)n * H;
    for (int i = 0; i < H; ++i)
      for (int k = 0; k < H; ++k) g2[i * H + k] += a1[i] * gn[k];
  }
  for (int n = 0; n < N; ++n) { /* g_a1 = (g_a2 w2^T) (1 - h1^2), then gw1 += X^T g_a1 */
    const float* a1 = h1 + (size_t)n * H;
    const float* gn = ga + (size_t)n * H;
    for (int i = 0; i < H; ++i) {
      float s = 0.0f;
      for (int k = 0; k < H; ++k) s += gn[k] * w2[i * H + k];
      s *= 1.0f - a1[i] * a1[i];
      for (int x = 0; x < Dx; ++x) g1[x * H + i] += X[n * Dx + x] * s;
    }
  }
  g[0] = (float)-(3.0 - p + 0.5 * N - 0.5 * p * ee);
  *pe = (float)-lp;
}

/* Z [B][D] -> pe [B], G [B][D] (model coordinates); work: per-thread scratch */
typedef struct {
  float* zt; /* covtype: [D][B] transposes */
  float* gt;
  float* work; /* BNN: [threads][4 N H] */
  size_t work_per;
  float* zm; /* dense: model-space positions / gradients [B][D] */
  float* gm;
} Scratch;

static void model_pe_grad(const nmx_cpu_model* m, int B, const float* Z, float* pe, float* G, Scratch* sc) {
  const int D = m->dim;
  if (m->model == 1) {
    for (int b = 0; b < B; ++b)
      for (int d = 0; d < D; ++d) sc->zt[(size_t)d * B + b] = Z[(size_t)b * D + d];
    nmx_cpu_logreg_pe_grad(m->X, m->y, m->n, D, sc->zt, B, pe, sc->gt);
    for (int b = 0; b < B; ++b)
      for (int d = 0; d < D; ++d) G[(size_t)b * D + d] = sc->gt[(size_t)d * B + b];
    return;
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int b = 0; b < B; ++b) {
    const float* z = Z + (size_t)b * D;
    float* g = G + (size_t)b * D;
    if (m->model == 2) pe_funnel(D, z, pe + b, g);
    else if (m->model == 3) pe_sv(m->r2, D - 2, z, pe + b, g);
    else pe_bnn(m, z, pe + b, g, sc->work + (size_t)omp_get_thread_num() * sc->work_per);
  }
}

/* dense mass: U_w(w) = U(mu + T w), grad_w = T^T grad_z (numpyro_amd/dense.py whitening) */
static void pe_grad(const nmx_cpu_model* m, int B, const float* W, float* pe, float* G, Scratch* sc) {
  if (!m->wT) {
    model_pe_grad(m, B, W, pe, G, sc);
    return;
  }
  const int D = m->dim;
  const float* T = m->wT;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < D; ++i) {
    const float* t = T + (size_t)i * D;
    for (int b = 0; b < B; ++b) {
      const float* w = W + (size_t)b * D;
      float s = 0.0f;
#pragma omp simd reduction(+ : s)
      for (int k = 0; k < D; ++k) s += t[k] * w[k];
      sc->zm[(size_t)b * D + i] = m->wmu[i] + s;
    }
  }
  model_pe_grad(m, B, sc->zm, pe, sc->gm, sc);
#pragma omp parallel
  {
    const int nt = omp_get_num_threads(), id = omp_get_thread_num();
    const int k0 = (int)((long)D * id / nt), k1 = (int)((long)D * (id + 1) / nt);
    for (int b = 0; b < B; ++b) {
      float* gw = G + (size_t)b * D;
      for (int k = k0; k < k1; ++k) gw[k] = 0.0f;
      for (int i = 0; i < D; ++i) {
        const float gi = sc->gm[(size_t)b * D + i];
        const float* t = T + (size_t)i * D;
#pragma omp simd
        for (int k = k0; k < k1; ++k) gw[k] += gi * t[k];
      }
    }
  }
}

/* ------------------------------------------------------------------------------- sampler */
typedef struct {
  int D, c;
  uint32_t gch; /* global chain id (Philox) */
  float step;
  const float *im, *msq;
  /* current sample */
  float *z, *g;
  float pe;
  int it, done_t; /* RNG transition index, transitions completed */
  int active;
  /* transition */
  float E0;
  float *tlr, *tlz, *tlg, *trr, *trz, *trg; /* tree ends (left, right) */
  float *tpz, *tpg;
  float tp_pe, tp_e, tw, tacc;
  int tn, tdepth, tturn, tdiv;
  float* trs;
  /* subtree */
  int j, right, sn, smax, sdiv, sturn;
  float sw, sacc, sp_pe, sp_e;
  float *spz, *spg, *srs;
  /* leaf in flight: moving end l* -> new leaf n* */
  float *lz, *lr, *lg, *nz, *nr, *ng, *rh;
  float half, st;
  float *ckr, *ckrs; /* [MAXD][D] */
  int maxd;
  float* trace; /* this chain's records [T][L][8] (NULL: off), the device's layout (nmx_trace_field) */
  int trace_T, trace_L;
} Chain;

/* Reductions in double, vectorised (omp simd reduction: the partial sums' order is the compiler's,
 * as in any float32 implementation of a dot product) */
static inline float kinetic(const float* im, const float* r, int D) { /* 0.5 (M^-1 r) . r */
  double s = 0.0;
#pragma omp simd reduction(+ : s)
  for (int i = 0; i < D; ++i) s += (double)(im[i] * r[i]) * r[i];
  return (float)(0.5 * s);
}
static int is_turning(const float* im, const float* rl, const float* rr, const float* rs, const float* ck_rs_or_null,
                      const float* ck_r_or_null, int D) {
  /* _is_turning(im, r_left, r_right, r_sum'), r_sum' = r_sum (- ck_rs + ck_r for a checkpoint) */
  double la = 0.0, ra = 0.0;
  if (ck_rs_or_null) {
#pragma omp simd reduction(+ : la, ra)
    for (int i = 0; i < D; ++i) {
      const float s = (rs[i] - ck_rs_or_null[i] + ck_r_or_null[i]) - (rl[i] + rr[i]) / 2.0f;
      la += (double)(im[i] * rl[i]) * s;
      ra += (double)(im[i] * rr[i]) * s;
    }
  } else {
#pragma omp simd reduction(+ : la, ra)
    for (int i = 0; i < D; ++i) {
      const float s = rs[i] - (rl[i] + rr[i]) / 2.0f;
      la += (double)(im[i] * rl[i]) * s;
      ra += (double)(im[i] * rr[i]) * s;
    }
  }
  return (la <= 0.0) || (ra <= 0.0);
}
static float turn_dots_min(const float* im, const float* rl, const float* rr, const float* rs, const float* ck_rs,
                           const float* ck_r, int D) { /* min(left, right) angle: the trace's U-turn dot */
  double la = 0.0, ra = 0.0;
#pragma omp simd reduction(+ : la, ra)
  for (int i = 0; i < D; ++i) {
    const float s = (ck_rs ? rs[i] - ck_rs[i] + ck_r[i] : rs[i]) - (rl[i] + rr[i]) / 2.0f;
    la += (double)(im[i] * rl[i]) * s;
    ra += (double)(im[i] * rr[i]) * s;
  }
  return (float)(la < ra ? la : ra);
}
static inline float logaddexpf_(float a, float b) {
  const float m = fmaxf(a, b);
  if (isinf(m) && m < 0) return m;
  return (float)(m + log1p(exp(-(double)fabsf(a - b))));
}
static inline int popc(unsigned x) { return __builtin_popcount(x); }
static void ckpt_idxs(int n, int* lo, int* hi) { /* hmc_util.py:941-958 */
  *hi = popc((unsigned)n >> 1);
  const int ns = popc((unsigned)((~n & (n + 1)) - 1));
  *lo = *hi - ns + 1;
}

static void copyv(float* d, const float* s, int D) { memcpy(d, s, sizeof(float) * (size_t)D); }

/* leapfrog first half from the moving end l*: r_half, z_new (the potential is evaluated next) */
static void leaf_begin(Chain* ch) {
  const int D = ch->D;
  ch->st = ch->right ? ch->step : -ch->step;
  ch->half = 0.5f * ch->st;
  for (int i = 0; i < D; ++i) {
    ch->rh[i] = ch->lr[i] - ch->half * ch->lg[i];
    ch->nz[i] = ch->lz[i] + ch->st * (ch->im[i] * ch->rh[i]);
  }
}

static void start_doubling(Chain* ch, uint64_t seed);
static void start_transition(Chain* ch, uint64_t seed) {
  const int D = ch->D;
  /* momentum: r = mass_matrix_sqrt * eps (hmc.py:92-110), eps from 4-wide Philox blocks */
  float* r = ch->tlr;
  for (int blk = 0; blk < (D + 3) / 4; ++blk) {
    uint32_t o[4];
    float n[4];
    rng(seed, ch->gch, (uint32_t)ch->it, EV_MOMENTUM, (uint32_t)blk, 0, o);
    box_muller(o[0], o[1], &n[0], &n[1]);
    box_muller(o[2], o[3], &n[2], &n[3]);
    for (int q = 0; q < 4 && 4 * blk + q < D; ++q) r[4 * blk + q] = ch->msq[4 * blk + q] * n[q];
  }
  ch->E0 = ch->pe + kinetic(ch->im, r, D);
  copyv(ch->trr, r, D);
  copyv(ch->trs, r, D);
  copyv(ch->tlz, ch->z, D);
  copyv(ch->tlg, ch->g, D);
  copyv(ch->trz, ch->z, D);
  copyv(ch->trg, ch->g, D);
  copyv(ch->tpz, ch->z, D);
  copyv(ch->tpg, ch->g, D);
  ch->tp_pe = ch->pe;
  ch->tp_e = ch->E0;
  ch->tw = 0.0f;
  ch->tacc = 0.0f;
  ch->tn = 0;
  ch->tdepth = 0;
  ch->tturn = 0;
  ch->tdiv = 0;
  start_doubling(ch, seed);
}

/* build_tree loop condition (:1155-1157); a new doubling (_double_tree :907-938) or the end */
static void start_doubling(Chain* ch, uint64_t seed) {
  const int D = ch->D;
  if (ch->tdepth < ch->maxd && !ch->tturn && !ch->tdiv) {
    ch->j = ch->tdepth;
    ch->right = uniform(seed, ch->gch, (uint32_t)ch->it, EV_DIRECTION, (uint32_t)ch->j, 0) < 0.5f;
    ch->sn = 0;
    ch->smax = 1 << ch->j;
    ch->sturn = 0;
    ch->sdiv = 0;
    /* the first leaf grows from the tree's end in this direction (_get_leaf :897-904) */
    copyv(ch->lz, ch->right ? ch->trz : ch->tlz, D);
    copyv(ch->lr, ch->right ? ch->trr : ch->tlr, D);
    copyv(ch->lg, ch->right ? ch->trg : ch->tlg, D);
    leaf_begin(ch);
    return;
  }
  ch->active = 0; /* transition ends: the proposal is the sample (_nuts_next :416-455) */
}

/* the evaluated leaf: second half step, _build_basetree, the subtree combine, checkpoints and the
 * iterative U-turn check; at the subtree's end the biased tree combine.  Returns 1 when the
 * chain's transition has ended. */
static int leaf_end(Chain* ch, float pe_new, float max_de, uint64_t seed) {
  const int D = ch->D;
  for (int i = 0; i < D; ++i) ch->nr[i] = ch->rh[i] - ch->half * ch->ng[i];
  const float e_new = pe_new + kinetic(ch->im, ch->nr, D);
  float de = e_new - ch->E0;
  if (isnan(de)) de = INFINITY;
  const float w = -de;
  const int div = de > max_de;
  const float acc = fminf(expf(-de), 1.0f);
  const int k = ch->sn;
  float p_leaf = -1.0f;
  int take = 1;
  if (k == 0) { /* new_tree = new_leaf */
    copyv(ch->srs, ch->nr, D);
    copyv(ch->spz, ch->nz, D);
    copyv(ch->spg, ch->ng, D);
    ch->sp_pe = pe_new;
    ch->sp_e = e_new;
    ch->sw = w;
    ch->sacc = acc;
  } else { /* _combine_tree(..., biased_transition=False) (:767-848, :749-753) */
    for (int i = 0; i < D; ++i) ch->srs[i] += ch->nr[i];
    const float p = 1.0f / (1.0f + expf(-(w - ch->sw)));
    const float u = uniform(seed, ch->gch, (uint32_t)ch->it, EV_LEAF, (uint32_t)ch->j, (uint32_t)k);
    p_leaf = p;
    take = u < p;
    if (u < p) {
      copyv(ch->spz, ch->nz, D);
      copyv(ch->spg, ch->ng, D);
      ch->sp_pe = pe_new;
      ch->sp_e = e_new;
    }
    ch->sw = logaddexpf_(ch->sw, w);
    ch->sacc += acc;
  }
  ch->sdiv = div;
  ch->sn = k + 1;
  int lo, hi;
  ckpt_idxs(k, &lo, &hi);
  if (k % 2 == 0) {
    copyv(ch->ckr + (size_t)hi * D, ch->nr, D);
    copyv(ch->ckrs + (size_t)hi * D, ch->srs, D);
  }
  int turning = 0; /* _is_iterative_turning (:961-981): idx_max down to idx_min */
  for (int i = hi; i >= lo && !turning; --i)
    turning = is_turning(ch->im, ch->ckr + (size_t)i * D, ch->nr, ch->srs, ch->ckrs + (size_t)i * D,
                         ch->ckr + (size_t)i * D, D);
  float* R = NULL; /* decision trace (every checkpoint dot of the leaf, like the device and the oracle) */
  const int leaf_n = ch->tn + k;
  if (ch->trace && ch->done_t < ch->trace_T && leaf_n < ch->trace_L) {
    R = ch->trace + ((size_t)ch->done_t * ch->trace_L + leaf_n) * 8;
    float dmin = INFINITY;
    for (int i = lo; i <= hi; ++i) {
      const float d = turn_dots_min(ch->im, ch->ckr + (size_t)i * D, ch->nr, ch->srs, ch->ckrs + (size_t)i * D,
                                    ch->ckr + (size_t)i * D, D);
      dmin = d < dmin ? d : dmin;
    }
    R[0] = de;
    R[1] = p_leaf;
    R[2] = dmin;
    R[3] = -1.0f;
    R[4] = INFINITY;
    R[5] = (float)((take ? 1 : 0) | (turning ? 2 : 0) | (div ? 4 : 0));
    R[6] = pe_new;
    R[7] = (float)leaf_n;
  }
  /* the new leaf is the subtree's moving end */
  float* t;
  t = ch->lz, ch->lz = ch->nz, ch->nz = t;
  t = ch->lr, ch->lr = ch->nr, ch->nr = t;
  t = ch->lg, ch->lg = ch->ng, ch->ng = t;
  if (ch->sn < ch->smax && !turning && !ch->sdiv) {
    leaf_begin(ch);
    return 0;
  }
  ch->sturn = turning;
  const int full = ch->sn == ch->smax && !turning && !ch->sdiv;
  /* _combine_tree(tree, subtree, biased_transition=True) (:756-764, :795-799) */
  if (ch->right) {
    copyv(ch->trz, ch->lz, D);
    copyv(ch->trr, ch->lr, D);
    copyv(ch->trg, ch->lg, D);
  } else {
    copyv(ch->tlz, ch->lz, D);
    copyv(ch->tlr, ch->lr, D);
    copyv(ch->tlg, ch->lg, D);
  }
  for (int i = 0; i < D; ++i) ch->trs[i] += ch->srs[i];
  float pb = expf(ch->sw - ch->tw);
  pb = isnan(pb) ? pb : fminf(pb, 1.0f);
  const float pb_raw = pb;
  if (ch->sturn || ch->sdiv) pb = 0.0f;
  const int tturn = ch->sturn || is_turning(ch->im, ch->tlr, ch->trr, ch->trs, NULL, NULL, D);
  const float u = uniform(seed, ch->gch, (uint32_t)ch->it, EV_BIASED, (uint32_t)ch->j, 0);
  if (R) {
    R[3] = pb_raw;
    if (full) R[4] = turn_dots_min(ch->im, ch->tlr, ch->trr, ch->trs, NULL, NULL, D);
    const int done = ch->tdepth + 1 >= ch->maxd || tturn || ch->sdiv;
    R[5] = (float)((int)R[5] | 8 | (u < pb ? 16 : 0) | (tturn ? 32 : 0) | (done ? 64 : 0));
  }
  if (u < pb) {
    copyv(ch->tpz, ch->spz, D);
    copyv(ch->tpg, ch->spg, D);
    ch->tp_pe = ch->sp_pe;
    ch->tp_e = ch->sp_e;
  }
  ch->tw = logaddexpf_(ch->tw, ch->sw);
  ch->tdepth += 1;
  ch->tturn = tturn;
  ch->tdiv = ch->sdiv;
  ch->tacc += ch->sacc;
  ch->tn += ch->sn;
  start_doubling(ch, seed);
  return !ch->active;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* Run C chains from the given sampling state until each has completed `num_transitions`
 * transitions, or -- once it has completed `min_transitions` -- until `seconds` have elapsed.
 * out_num_steps [C][num_transitions] (tree sizes, -1 past a chain's last), out_z
 * [C][num_transitions][D] (draws in the sampler's coordinates, NULL: not kept), out_done [C],
 * stats [4]: leapfrogs (potential evaluations), wall seconds, seconds inside the potential,
 * batched potential calls; out_trace [C][num_transitions][2^max_tree_depth][8] (NULL: off; the
 * caller fills it with NaN) the per-leaf decision records in the device trace's layout
 * (include/numpyro_amd.h enum nmx_trace_field / nmx_trace_flag; oracle/parity.py).  Returns 0, or -1 on a bad argument / allocation failure. */
int nmx_cpu_nuts_run(const nmx_cpu_model* m, int C, const float* z0, const float* g0, const float* pe0,
                     const float* step, const float* inv_mass, const float* mass_sqrt, uint64_t seed, int it0,
                     long chain_offset, int max_tree_depth, float max_delta_energy, int num_transitions,
                     int min_transitions, double seconds, int* out_num_steps, float* out_z, int* out_done,
                     double* stats, float* out_trace) {
  if (!m || C <= 0 || m->dim <= 0 || max_tree_depth < 1 || max_tree_depth > MAXD || num_transitions < 1) return -1;
  const int D = m->dim;
  const size_t vec = (size_t)D;
  const int NV = 28; /* D-vectors per chain */
  float* pool = (float*)calloc((size_t)C * (NV + 2 * MAXD) * vec, sizeof(float));
  Chain* ch = (Chain*)calloc((size_t)C, sizeof(Chain));
  float* Zb = (float*)malloc(sizeof(float) * (size_t)C * vec);
  float* Gb = (float*)malloc(sizeof(float) * (size_t)C * vec);
  float* Pb = (float*)malloc(sizeof(float) * (size_t)C);
  int* idx = (int*)malloc(sizeof(int) * (size_t)C);
  Scratch sc = {0};
  sc.zt = (float*)malloc(sizeof(float) * (size_t)C * vec);
  sc.gt = (float*)malloc(sizeof(float) * (size_t)C * vec);
  if (m->model == 4) {
    sc.work_per = (size_t)4 * m->n * m->bnn_h + 64;
    sc.work = (float*)malloc(sizeof(float) * sc.work_per * (size_t)omp_get_max_threads());
  }
  if (m->wT) {
    sc.zm = (float*)malloc(sizeof(float) * (size_t)C * vec);
    sc.gm = (float*)malloc(sizeof(float) * (size_t)C * vec);
  }
  if (!pool || !ch || !Zb || !Gb || !Pb || !idx || !sc.zt || !sc.gt || (m->model == 4 && !sc.work) ||
      (m->wT && (!sc.zm || !sc.gm))) {
    free(pool), free(ch), free(Zb), free(Gb), free(Pb), free(idx), free(sc.zt), free(sc.gt), free(sc.work);
    free(sc.zm), free(sc.gm);
    return -1;
  }
  for (int c = 0; c < C; ++c) {
    Chain* h = ch + c;
    float* p = pool + (size_t)c * (NV + 2 * MAXD) * vec;
    float** slots[] = {&h->z, &h->g, &h->tlr, &h->tlz, &h->tlg, &h->trr, &h->trz, &h->trg, &h->tpz, &h->tpg,
                       &h->trs, &h->spz, &h->spg, &h->srs, &h->lz, &h->lr, &h->lg, &h->nz, &h->nr, &h->ng,
                       &h->rh};
    for (size_t s = 0; s < sizeof(slots) / sizeof(slots[0]); ++s) *slots[s] = p + s * vec;
    h->ckr = p + (size_t)NV * vec;
    h->ckrs = h->ckr + (size_t)MAXD * vec;
    h->D = D;
    h->c = c;
    h->gch = (uint32_t)(chain_offset + c);
    h->step = step[c];
    h->im = inv_mass + (size_t)c * vec;
    h->msq = mass_sqrt + (size_t)c * vec;
    copyv(h->z, z0 + (size_t)c * vec, D);
    copyv(h->g, g0 + (size_t)c * vec, D);
    h->pe = pe0[c];
    h->it = it0;
    h->maxd = max_tree_depth;
    if (out_trace) {
      h->trace_T = num_transitions;
      h->trace_L = 1 << max_tree_depth;
      h->trace = out_trace + (size_t)c * num_transitions * h->trace_L * 8;
    }
    h->active = 1;
    start_transition(h, seed);
  }
  for (int c = 0; c < C; ++c)
    for (int t = 0; t < num_transitions; ++t) out_num_steps[(size_t)c * num_transitions + t] = -1;
  const double t0 = now_s();
  double pot = 0.0, leap = 0.0, calls = 0.0;
  int running = C;
  if (m->model != 1 && !m->wT) {
    /* per-chain potentials (funnel, SV, BNN with a diagonal mass): no batch to form, so each thread
     * runs its own chains (c = tid, tid + nthreads, ...) leaf by leaf, round robin, with no
     * barrier per leaf -- the batched loop below paid three fork / joins and waited for the slowest
     * chain every round.  Each chain's arithmetic is the same (bitwise the same draws); the
     * potential seconds are the threads' mean. */
    const int nth = omp_get_max_threads();
#pragma omp parallel reduction(+ : pot, leap, calls)
    {
      const int tid = omp_get_thread_num(), nt = omp_get_num_threads();
      float* work = sc.work ? sc.work + (size_t)tid * sc.work_per : NULL;
      int live = 1;
      while (live) {
        live = 0;
        for (int c = tid; c < C; c += nt) {
          Chain* h = ch + c;
          if (!h->active) continue;
          const double p0 = now_s();
          float pe_new;
          if (m->model == 2) pe_funnel(D, h->nz, &pe_new, h->ng);
          else if (m->model == 3) pe_sv(m->r2, D - 2, h->nz, &pe_new, h->ng);
          else pe_bnn(m, h->nz, &pe_new, h->ng, work);
          const double p1 = now_s();
          pot += p1 - p0;
          leap += 1.0;
          calls += 1.0;
          if (min_transitions == 0 && p1 - t0 >= seconds) { /* a timing run: stop mid-transition */
            h->active = 0;
            continue;
          }
          live = 1;
          if (!leaf_end(h, pe_new, max_delta_energy, seed)) continue;
          copyv(h->z, h->tpz, D);
          copyv(h->g, h->tpg, D);
          h->pe = h->tp_pe;
          const int t = h->done_t;
          out_num_steps[(size_t)h->c * num_transitions + t] = h->tn;
          if (out_z) copyv(out_z + ((size_t)h->c * num_transitions + t) * vec, h->z, D);
          h->done_t = t + 1;
          h->it += 1;
          if (h->done_t < num_transitions && (h->done_t < min_transitions || p1 - t0 < seconds)) {
            h->active = 1;
            start_transition(h, seed);
          }
        }
      }
    }
    pot /= nth;
    running = 0;
  }
  while (running > 0) {
    int B = 0;
    for (int c = 0; c < C; ++c)
      if (ch[c].active) idx[B++] = c;
    if (B == 0) break;
#pragma omp parallel for schedule(static)
    for (int b = 0; b < B; ++b) copyv(Zb + (size_t)b * vec, ch[idx[b]].nz, D);
    const double p0 = now_s();
    pe_grad(m, B, Zb, Pb, Gb, &sc);
    pot += now_s() - p0;
    leap += B;
    calls += 1;
    const double elapsed = now_s() - t0;
    if (min_transitions == 0 && elapsed >= seconds) break; /* a timing run: stop mid-transition */
    /* one chain per chunk: with 32 chains on 16 threads, chunks of 4 left half the threads idle in
     * the tree logic (SV, scripts/sv_cpu_share.py on the GPU box: 1.37-1.42x leapfrog/s) */
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      Chain* h = ch + idx[b];
      copyv(h->ng, Gb + (size_t)b * vec, D);
      if (!leaf_end(h, Pb[b], max_delta_energy, seed)) continue;
      /* transition end: the tree's proposal is the new sample */
      copyv(h->z, h->tpz, D);
      copyv(h->g, h->tpg, D);
      h->pe = h->tp_pe;
      const int t = h->done_t;
      out_num_steps[(size_t)h->c * num_transitions + t] = h->tn;
      if (out_z) copyv(out_z + ((size_t)h->c * num_transitions + t) * vec, h->z, D);
      h->done_t = t + 1;
      h->it += 1;
      if (h->done_t < num_transitions && (h->done_t < min_transitions || elapsed < seconds)) {
        h->active = 1;
        start_transition(h, seed);
      }
    }
    running = 0;
    for (int c = 0; c < C; ++c) running += ch[c].active;
  }
  for (int c = 0; c < C; ++c) out_done[c] = ch[c].done_t;
  stats[0] = leap;
  stats[1] = now_s() - t0;
  stats[2] = pot;
  stats[3] = calls;
  free(pool), free(ch), free(Zb), free(Gb), free(Pb), free(idx), free(sc.zt), free(sc.gt), free(sc.work);
  free(sc.zm), free(sc.gm);
  return 0;
}
