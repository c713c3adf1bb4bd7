// Per-coordinate potential terms of the D-split (wide) models, shared by their standalone
// potential kernels (potential_wide.hip) and the fused leaf kernel of the wide NUTS step
// (nuts.hip, k_wide_leaf / k_wide_rs), so both compute every coordinate gradient with the same
// device code.  A model splits z into
//   * per-coordinate rows [lo, hi): gradient from the row, its stencil neighbours and the
//     model's global values; each row adds NSUM partial sums;
//   * NSCALAR global (scalar-site) rows, whose gradients and U need the full sums (fin).
// Gradients are hand-derived.
#pragma once
#include <math.h>

// NMX_SV_FAST (default): the SV row's q / (1 + q) by the hardware reciprocal and log1p(q) as
// log(u) q / (u - 1), u = 1 + q, from the hardware log2 -- a few ulp instead of the libm forms'
// ~1, 62 instead of 177 VALU instructions per row.  The persistent SV kernel is VALU-bound
// (profiles/r04/sv_persistent_pmc_and_bc.txt): 29.9M -> 35.6M leapfrog/s at 8192 chains, 14.1M ->
// 18.1M at 1024 (profiles/r04/ab_sv_row_math.txt).  Every schedule includes this header, so they
// stay bitwise equal to each other; against the float64 oracle the potential keeps its tolerance.
#ifndef NMX_SV_FAST
#define NMX_SV_FAST 1
#endif

#include "nmx_common.h"

// A double constant materialized at its use: the compiler otherwise hoists the 64-bit constants
// of a double polynomial out of the persistent kernel's leaf loop and, at 128 VGPRs, spills them
// to scratch -- and each reload in the serial section waited (vmcnt(0)) for every global store
// the wave still had in flight from its rows.
__device__ __forceinline__ double nmx_kd(double c) {
  asm volatile("" : "+s"(c));
  return c;
}

// log(y) for a finite y > 0 in double: y = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s),
// s = (m - 1) / (m + 1) (|s| <= 0.172: ten series terms), e ln 2 in two parts.  Within 2 ulp of
// libm over 1e-30..1e30 (tests/test_sv_fin_series.py restates it); replaces ocml's log, whose
// hoisted coefficients were the spilled constants above.
__device__ __forceinline__ double nmx_log_f64(double y) {
  int e = __builtin_amdgcn_frexp_exp(y);
  double m = __builtin_amdgcn_frexp_mant(y);  // [0.5, 1)
  if (m < nmx_kd(0.70710678118654752440)) {
    m *= 2.0;
    e -= 1;
  }
  const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
  double p = nmx_kd(1.0 / 21);
  p = nmx_kd(1.0 / 19) + s2 * p;
  p = nmx_kd(1.0 / 17) + s2 * p;
  p = nmx_kd(1.0 / 15) + s2 * p;
  p = nmx_kd(1.0 / 13) + s2 * p;
  p = nmx_kd(1.0 / 11) + s2 * p;
  p = nmx_kd(1.0 / 9) + s2 * p;
  p = nmx_kd(1.0 / 7) + s2 * p;
  p = nmx_kd(1.0 / 5) + s2 * p;
  p = nmx_kd(1.0 / 3) + s2 * p;
  const double ed = (double)e;
  return ed * nmx_kd(6.93147180369123816490e-01) + (2.0 * s + (2.0 * s * s2 * p + ed * nmx_kd(1.90821492927058770002e-10)));
}

// The StudentT normaliser's two differences at x = nu / 2 > 0, in double:
//   L = lgamma(x) - lgamma(x + 1/2),  Psi = digamma(x) - digamma(x + 1/2).
// The recurrence lgamma(x) = lgamma(x + 1) - log x (digamma: - 1/x) shifts x to X >= 8, keeping
// the shifts as one product ratio prod (x+k) / (x+k+1/2) and one fraction sum 1/2 / ((x+k)(x+k+1/2))
// (one log and one division for all of them); at X the Stirling series of both functions are
// differenced analytically: log(X + 1/2) = log X + log1p(1/(2X)), log1p by its atanh series (t <=
// 1/33: six terms).  Absolute error <= 2e-13 over x in [0.02, 60] against scipy's gammaln /
// digamma (tests/test_sv_fin_series.py restates the series) -- what the float64 lgamma / digamma pair gave, at one log
// instead of two lgammas, two digamma recurrences and their divisions: the SV leaf's serial
// section (wave 0) was 31% of the persistent kernel's leaf (profiles/r06/sv_phase_stamps.txt).
__device__ __forceinline__ void nmx_lgamma_digamma_half_diff(double x, double& L, double& Psi) {
  double X = x, pn = 1.0, pd = 1.0, num = 0.0, den = 1.0;
  while (X < 8.0) {
    const double h = X + 0.5, q = X * h;
    pn *= X;
    pd *= h;
    num = num * q + 0.5 * den;
    den *= q;
    X += 1.0;
  }
  // 1/X and 1/(X + 1/2) from one division, likewise pn/pd and num/den (double divisions are ~10
  // dependent instructions each)
  const double H = X + 0.5, rxh = 1.0 / (X * H), inv = H * rxh, invh = X * rxh;
  const double u = 0.5 * inv, t = u / (2.0 + u), t2 = t * t;
  const double l1p =
      2.0 * t * (1.0 + t2 * (1.0 / 3 + t2 * (1.0 / 5 + t2 * (1.0 / 7 + t2 * (1.0 / 9 + t2 * (1.0 / 11))))));
  // lgamma's Stirling tail 1/(12z) - 1/(360z^3) + ... and digamma's -1/(12z^2) + 1/(120z^4) - ...
  auto lser = [](double iz) {
    const double iz2 = iz * iz;
    return iz * (1.0 / 12 - iz2 * (1.0 / 360 - iz2 * (1.0 / 1260 - iz2 * (1.0 / 1680 - iz2 / 1188))));
  };
  auto pser = [](double iz) {
    const double iz2 = iz * iz;
    return iz2 * (1.0 / 12 - iz2 * (1.0 / 120 - iz2 * (1.0 / 252 - iz2 * (1.0 / 240 - iz2 / 132))));
  };
  const double rpd = 1.0 / (pd * den), r = pn * den * rpd;
  L = -0.5 * nmx_log_f64(X * r * r) - X * l1p + 0.5 + lser(inv) - lser(invh);
  Psi = -l1p - 0.5 * inv + 0.5 * invh - pser(inv) + pser(invh) - num * pd * rpd;
}

// expf(x) by the same reduction the compiler's expf uses (x log2 e in two parts, 2^frac by
// v_exp_f32, ldexp) without its overflow / underflow selects: bitwise expf's value for |x| <= 87
// (SV's -2 s), four VALU fewer per row; beyond that the value saturates the same way (ldexp), and
// a non-finite s gives NaN where expf gives inf -- either way the leaf's energy is not finite and
// the trajectory diverges.
__device__ __forceinline__ float nmx_expf_unchecked(float x) {
  const float l2e = __int_as_float(0x3fb8aa3b), l2e_lo = __int_as_float(0x32a5705f);
  float t = x * l2e;
  asm volatile("" : "+v"(t));  // t is the rounded product, as in expf (else (t - n) became fma(x, l2e, -n))
  const float n = __builtin_rintf(t);
  const float c = __builtin_fmaf(x, l2e_lo, __builtin_fmaf(x, l2e, -t));
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f((t - n) + c), (int)n);
}

// Stochastic volatility (examples/stochastic_volatility.py:57-65), z = (a = log nu, s[T],
// b = log sigma): rows 1..T are s_t (t = row - 1), scalar rows 0 (a) and T + 1 (b).
// Sums: sum d_t^2, sum log1p(q_t), sum q_t / (1 + q_t), sum s_t.
struct NmxWideSV {
  const float* ret;
  int T;
  static constexpr int NSUM = 4;
  static constexpr int NSCALAR = 2;
  struct Glob {
    float a, b, nu, inv_sig2, inv_nu;
  };
  NMX_HD int lo() const { return 1; }
  NMX_HD int hi() const { return T + 1; }
  NMX_HD int scalar_row(int i) const { return i == 0 ? 0 : T + 1; }
  __device__ __forceinline__ Glob globals(const float* z, int ldc, int c) const {
    Glob g;
    g.a = z[c];
    g.b = z[(size_t)(T + 1) * ldc + c];
    g.nu = expf(g.a);
    g.inv_sig2 = expf(-2.0f * g.b);
    g.inv_nu = 1.0f / g.nu;
    return g;
  }
  // the same from any layout: row r of the chain at byte offset off0 + r * stride4
  __device__ __forceinline__ Glob globals_at(const float* z, uint32_t off0, uint32_t stride4) const {
    Glob g;
    g.a = nmx_at(z, off0);
    g.b = nmx_at(z, off0 + (uint32_t)(T + 1) * stride4);
    g.nu = expf(g.a);
    g.inv_sig2 = expf(-2.0f * g.b);
    g.inv_nu = 1.0f / g.nu;
    return g;
  }
  // dU/ds_t of row d = 1 + t (GaussianRandomWalk stencil + StudentT(nu, 0, e^s) term)
  // (off: byte offset of the row; ldc4: the byte stride between rows -- 4 ldc in the
  // chain-minor layout, 4 in the chain-row layout of the persistent wide kernel).  row_load /
  // row_eval split row() into its loads and its arithmetic (the pipelined leaf, nuts.hip).
  struct RowIn {
    float s, sp, sn, r;
  };
  __device__ __forceinline__ void row_load(const float* z, uint32_t off, uint32_t ldc4, int d, RowIn& x) const {
    row_load_z(z, off, ldc4, d, x);
    row_load_data(d, x);
  }
  // the two halves of row_load: the positions (the LDS frontier in the persistent kernel) and the
  // data (HBM / L2), so a caller can batch the memory loads of several rows ahead of the rest
  __device__ __forceinline__ void row_load_z(const float* z, uint32_t off, uint32_t ldc4, int d, RowIn& x) const {
    const int t = d - 1;
    x.s = nmx_at(z, off);
    x.sp = t > 0 ? nmx_at(z, off - ldc4) : 0.0f;
    x.sn = t + 1 < T ? nmx_at(z, off + ldc4) : 0.0f;
  }
  // (a 32-bit byte offset from the SGPR base: ret[d - 1] took a 64-bit per-lane address, which the
  // persistent kernel hoisted per row and spilled)
  __device__ __forceinline__ void row_load_data(int d, RowIn& x) const { x.r = nmx_at(ret, (uint32_t)(d - 1) << 2); }
  __device__ __forceinline__ float row(const float* z, uint32_t off, uint32_t ldc4, int d, const Glob& g,
                                       float* sums) const {
    RowIn x;
    row_load(z, off, ldc4, d, x);
    return row_eval(x, d, g, sums);
  }
  __device__ __forceinline__ float row_eval(const RowIn& x, int d, const Glob& g, float* sums) const {
    const int t = d - 1;
    const float s = x.s, sp = x.sp, sn = x.sn;
    const float dd = s - sp;
    const float dn = t + 1 < T ? sn - s : 0.0f;
    const float r = x.r;
#if NMX_SV_FAST
    const float q = r * r * nmx_expf_unchecked(-2.0f * s) * g.inv_nu;
    const float u = 1.0f + q;
    const float qq = q * __builtin_amdgcn_rcpf(u);
    const float l1q = (u == 1.0f || !(u < INFINITY)) ? q
                                                     : __builtin_amdgcn_logf(u) * 0.6931471805599453f *
                                                           (q * __builtin_amdgcn_rcpf(u - 1.0f));
#else
    const float q = r * r * expf(-2.0f * s) * g.inv_nu;
    const float qq = q / (1.0f + q);
    const float l1q = log1pf(q);
#endif
    sums[0] += dd * dd;
    sums[1] += l1q;
    sums[2] += qq;
    sums[3] += s;
    // dU/ds_t = -( -(d_t - d_{t+1})/sigma^2 + (nu+1) q/(1+q) - 1 )
    return (dd - dn) * g.inv_sig2 - (g.nu + 1.0f) * qq + 1.0f;
  }
  // U and the gradients of the scalar rows (gs[0] = dU/da, gs[1] = dU/db), in double: the
  // StudentT normaliser enters as T x (lgamma(nu/2) - lgamma((nu+1)/2)) and dU/da as
  // T x (psi(nu/2) - psi((nu+1)/2)) -- differences of two O(1) values multiplied by T = 2517, and
  // dU/da is a small difference of O(T) terms.  In float32 their rounding moved dU/da by ~1e-4
  // relative and the draws 5-40x further from the float64 reference than a float32 NumPy
  // implementation's (round-5 parity calibration, tests/test_gpu_nuts.py fixed-step SV); in double
  // the scalar section costs a few hundred FP64 instructions per chain-leaf (wave 0 only).
  __device__ __forceinline__ float fin(const float* sums, const Glob& g, float* gs) const {
    const double a = g.a, b = g.b, nu = exp(a), Tf = (double)T;
    const double sig = exp(b), inv_sig2 = 1.0 / (sig * sig);
    const double s0 = sums[0], s1 = sums[1], s2 = sums[2], s3 = sums[3];
    double lg, dig;
    nmx_lgamma_digamma_half_diff(0.5 * nu, lg, dig);
    // log p
    double lp = 3.912023005428146 - 50.0 * sig + b;                 // Exponential(50) + log|J|
    lp += -0.5 * s0 * inv_sig2 - Tf * b - Tf * 0.9189385332046727;  // GaussianRandomWalk
    lp += -2.302585092994046 - 0.1 * nu + a;                        // Exponential(0.1) + log|J|
    lp += -0.5 * (nu + 1.0) * s1 - s3 - Tf * (0.5 * a + 0.5723649429247001 + lg);  // StudentT(nu, 0, e^s)
    const double ga = nu * (-0.1 - 0.5 * s1 - 0.5 * Tf * dig) + 0.5 * (nu + 1.0) * s2 - 0.5 * Tf + 1.0;
    const double gb = -50.0 * sig + 1.0 + s0 * inv_sig2 - Tf;
    gs[0] = (float)-ga;
    gs[1] = (float)-gb;
    return (float)-lp;
  }
};

// Centred funnel (examples/funnel.py:44-46), z = (x[K], y), K = dim - 1:
// U = y^2/18 + log(3 sqrt(2 pi)) + sum_i [x_i^2 e^-y / 2 + y/2 + log(2 pi)/2].
struct NmxWideFunnel {
  int dim;
  static constexpr int NSUM = 1;
  static constexpr int NSCALAR = 1;
  struct Glob {
    float y, e;
  };
  NMX_HD int lo() const { return 0; }
  NMX_HD int hi() const { return dim - 1; }
  NMX_HD int scalar_row(int) const { return dim - 1; }
  __device__ __forceinline__ Glob globals(const float* z, int ldc, int c) const {
    Glob g;
    g.y = z[(size_t)(dim - 1) * ldc + c];
    g.e = expf(-g.y);
    return g;
  }
  __device__ __forceinline__ Glob globals_at(const float* z, uint32_t off0, uint32_t stride4) const {
    Glob g;
    g.y = nmx_at(z, off0 + (uint32_t)(dim - 1) * stride4);
    g.e = expf(-g.y);
    return g;
  }
  struct RowIn {
    float x;
  };
  __device__ __forceinline__ void row_load(const float* z, uint32_t off, uint32_t, int, RowIn& in) const {
    in.x = nmx_at(z, off);
  }
  __device__ __forceinline__ void row_load_z(const float* z, uint32_t off, uint32_t, int, RowIn& in) const {
    in.x = nmx_at(z, off);
  }
  __device__ __forceinline__ void row_load_data(int, RowIn&) const {}
  __device__ __forceinline__ float row_eval(const RowIn& in, int, const Glob& g, float* sums) const {
    sums[0] += in.x * in.x;
    return in.x * g.e;
  }
  __device__ __forceinline__ float row(const float* z, uint32_t off, uint32_t ldc4, int d, const Glob& g,
                                       float* sums) const {
    RowIn in;
    row_load(z, off, ldc4, d, in);
    return row_eval(in, d, g, sums);
  }
  __device__ __forceinline__ float fin(const float* sums, const Glob& g, float* gs) const {
    const float K = (float)(dim - 1);
    gs[0] = g.y / 9.0f + 0.5f * K - 0.5f * g.e * sums[0];
    return g.y * g.y / 18.0f + 2.0175508218727822f + 0.5f * g.e * sums[0] + K * (0.5f * g.y + 0.9189385332046727f);
  }
};

// Non-centred funnel (examples/funnel.py:49, LocScaleReparam(0), numpyro/infer/reparam.py:
// 104-145), z = (x_decentered[K], y): U = y^2/18 + log(3 sqrt(2 pi)) + sum_i [x_i^2/2 +
// log(2 pi)/2]; dU/dx_i = x_i, dU/dy = y/9.
struct NmxWideFunnelNC {
  int dim;
  static constexpr int NSUM = 1;
  static constexpr int NSCALAR = 1;
  struct Glob {
    float y;
  };
  NMX_HD int lo() const { return 0; }
  NMX_HD int hi() const { return dim - 1; }
  NMX_HD int scalar_row(int) const { return dim - 1; }
  __device__ __forceinline__ Glob globals(const float* z, int ldc, int c) const {
    Glob g;
    g.y = z[(size_t)(dim - 1) * ldc + c];
    return g;
  }
  __device__ __forceinline__ Glob globals_at(const float* z, uint32_t off0, uint32_t stride4) const {
    Glob g;
    g.y = nmx_at(z, off0 + (uint32_t)(dim - 1) * stride4);
    return g;
  }
  struct RowIn {
    float x;
  };
  __device__ __forceinline__ void row_load(const float* z, uint32_t off, uint32_t, int, RowIn& in) const {
    in.x = nmx_at(z, off);
  }
  __device__ __forceinline__ void row_load_z(const float* z, uint32_t off, uint32_t, int, RowIn& in) const {
    in.x = nmx_at(z, off);
  }
  __device__ __forceinline__ void row_load_data(int, RowIn&) const {}
  __device__ __forceinline__ float row_eval(const RowIn& in, int, const Glob&, float* sums) const {
    sums[0] += in.x * in.x;
    return in.x;
  }
  __device__ __forceinline__ float row(const float* z, uint32_t off, uint32_t ldc4, int d, const Glob& g,
                                       float* sums) const {
    RowIn in;
    row_load(z, off, ldc4, d, in);
    return row_eval(in, d, g, sums);
  }
  __device__ __forceinline__ float fin(const float* sums, const Glob& g, float* gs) const {
    gs[0] = g.y / 9.0f;
    return g.y * g.y / 18.0f + 2.0175508218727822f + 0.5f * sums[0] + (float)(dim - 1) * 0.9189385332046727f;
  }
};
