/*
 * numpyro_amd C-ABI: the drop-in boundary of the MI355X-native NUTS/HMC engine.
 *
 * The reference (fehiepsi/numpyro) has no native code: its hot path is Python traced by
 * JAX/XLA.  Each entry point below replaces one piece of that traced path; the comment
 * on each names the reference function (file:line under numpyro/) it stands in for.
 * INTEGRATION.md shows the ctypes binding a numpyro maintainer would add.
 *
 * Conventions
 *  - extern "C", plain pointers and sizes; no torch types.  All pointers are device
 *    pointers unless named host_*.  `stream` is a hipStream_t passed as void*.
 *  - Chain-major SoA: a per-chain vector field is stored [D][ldc] (ldc >= C, ldc % 64 == 0),
 *    so lanes of a wave read consecutive chains.  Per-chain scalars are [ldc].
 *  - The library never allocates on the hot path: callers allocate the arena / workspace
 *    whose size the *_bytes() queries return.
 *  - Return value: NMX_OK or an error code; nmx_last_error() has the message.  Numerical
 *    events (divergence, NaN energy) are data, never errors (hmc_util.py:870-874).
 */
#ifndef NUMPYRO_AMD_H
#define NUMPYRO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMX_VERSION 1

enum nmx_status {
  NMX_OK = 0,
  NMX_ERR_INVALID = 1,     /* API misuse: bad size, null pointer, unsupported combo */
  NMX_ERR_HIP = 2,         /* HIP runtime error (launch failure etc.) */
  NMX_ERR_UNSUPPORTED = 3, /* configuration not implemented */
};

int nmx_version(void);
const char* nmx_last_error(void);

/* ---- self tests (no reference counterpart; used by tests and smoke()) ---- */
/* Philox4x32-10 on device: ctr_key is n x {c0,c1,c2,c3,k0,k1}, out is n x 4 words. */
int nmx_selftest_philox(const uint32_t* ctr_key, uint32_t* out, int n, void* stream);
/* C[32][32] = A[32][K] * B[K][32] through v_mfma_f32_32x32x2_f32 (fragment-layout probe). */
int nmx_selftest_mfma(const float* A, const float* B, float* C, int K, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NUMPYRO_AMD_H */
