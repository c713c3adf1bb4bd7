// Shared device helpers for the numpyro_amd HIP kernels (gfx950 / CDNA4, wave64).
//
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11). Every random draw of the
// sampler is a pure function of (seed, global chain id, MCMC iteration, event, index),
// so a chain's stream does not depend on which GPU runs it, on how many chains share
// the launch, or on whether chains advance in lockstep.  This replaces the nested
// jax.random.split tree of the reference (numpyro/infer/hmc.py:472-474,
// numpyro/infer/hmc_util.py:920,1005,1161-1162); see DESIGN.md "RNG streams".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/numpyro_amd.h"

#define NMX_HD __host__ __device__ __forceinline__

// Bounds / invariant checks of the debug build (numpyro_amd.build(debug=True), -DNMX_DEBUG;
// loaded with NUMPYRO_AMD_DEBUG=1): a failed check prints its location from the device (the
// tests scan the output) and the kernel continues -- no trap, so a bad index shows up as a
// message, not as a GPU fault.  Compiled out of the release library.
#ifdef NMX_DEBUG
#include <stdio.h>
#define NMX_DCHECK(cond)                                                                           \
  do {                                                                                             \
    if (!(cond)) printf("NMX_DCHECK failed %s:%d: %s (block %d thread %d)\n", __FILE__, __LINE__, #cond, \
                        (int)blockIdx.x, (int)threadIdx.x);                                        \
  } while (0)
#else
#define NMX_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

// RNG event tags (high byte of counter word 2).
enum nmx_rng_event : uint32_t {
  NMX_EV_MOMENTUM = 1u,   // momentum draw, word2 low bits = block of 4 coordinates
  NMX_EV_DIRECTION = 2u,  // doubling direction, word2 low bits = doubling index
  NMX_EV_BIASED = 3u,     // doubling-level (biased) transition
  NMX_EV_LEAF = 4u,       // leaf-level (uniform) transition, word3 = leaf index
  NMX_EV_INIT = 5u,       // init_to_uniform draw, word3 = attempt
  NMX_EV_ACCEPT = 6u,     // HMC Metropolis accept
  NMX_EV_HEURISTIC = 8u,  // find_reasonable_step_size momentum, word2 = block, word3 = attempt
};

struct nmx_u4 { uint32_t x, y, z, w; };

NMX_HD void nmx_mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

NMX_HD nmx_u4 nmx_philox4x32_10(nmx_u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0, lo0, hi1, lo1;
    nmx_mulhilo(0xD2511F53u, c.x, hi0, lo0);
    nmx_mulhilo(0xCD9E8D57u, c.z, hi1, lo1);
    nmx_u4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// One Philox block for a sampler event.
NMX_HD nmx_u4 nmx_rng(uint64_t seed, uint32_t chain, uint32_t iter, uint32_t event,
                      uint32_t idx, uint32_t sub) {
  nmx_u4 c;
  c.x = chain;
  c.y = iter;
  c.z = (event << 24) | (idx & 0x00FFFFFFu);
  c.w = sub;
  return nmx_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// uniform in [0, 1) with 24 random bits: exactly representable in fp32.
NMX_HD float nmx_u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }
// uniform in (0, 1]
NMX_HD float nmx_u01_open0(uint32_t x) { return ((float)(x >> 8) + 1.0f) * 5.9604644775390625e-08f; }

// Box-Muller pair from two words.
__device__ __forceinline__ void nmx_box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
  float u1 = nmx_u01_open0(a);
  float u2 = nmx_u01(b);
  float rad = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  n0 = rad * c;
  n1 = rad * s;
}

// Checkpoint index range of a leaf (numpyro/infer/hmc_util.py:941-958).
NMX_HD void nmx_leaf_idx_to_ckpt_idxs(int n, int& idx_min, int& idx_max) {
  idx_max = __builtin_popcount((unsigned)(n >> 1));
  int num_subtrees = __builtin_popcount((unsigned)((~n & (n + 1)) - 1));
  idx_min = idx_max - num_subtrees + 1;
}

// log(exp(a) + exp(b)) with the jnp.logaddexp conventions for infinities.
__device__ __forceinline__ float nmx_logaddexp(float a, float b) {
  float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  if (a == b) return a + 0.6931471805599453f;  // also handles +inf == +inf
  float d = -fabsf(a - b);
  return m + log1pf(expf(d));
}

__device__ __forceinline__ float nmx_sigmoid(float x) {
  // jax.scipy.special.expit
  return 1.0f / (1.0f + expf(-x));
}

// Chain evaluated at batch position `pos` of a potential launch, or -1.
// Element (d, c) of a chain-minor [D][ldc] field as a 32-bit byte offset.  Every field (and
// every checkpoint level) of the arena is < 4 GiB, so an access takes the SGPR-base + 32-bit
// VGPR-offset form of the global load / store and one offset register serves every field of a
// row (64-bit per-field addresses cost two VGPRs each and a 64-bit add per access).
__device__ __forceinline__ uint32_t nmx_row_off(int d, int ldc, int c) {
  return ((uint32_t)d * (uint32_t)ldc + (uint32_t)c) << 2;
}
template <class T>
__device__ __forceinline__ T& nmx_at(T* base, uint32_t off) {
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}
template <class T>
__device__ __forceinline__ const T& nmx_at(const T* base, uint32_t off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
}

__device__ __forceinline__ int nmx_eval_chain(const nmx_eval_batch& ev, int pos) {
  if (ev.active_idx) {
    if (pos >= *ev.active_count) return -1;
    const int c = ev.active_idx[pos];
    NMX_DCHECK(c >= 0 && c < ev.ldc && pos < ev.ldc);
    return c;
  }
  if (pos >= ev.num_chains) return -1;
  if (ev.phase && ev.phase[pos] < NMX_PH_LEAF) return -1;
  return pos;
}
