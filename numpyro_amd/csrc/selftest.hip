// Device self-tests used by tests/ and __graft_entry__.smoke(): Philox known-answer
// vectors and the gfx950 f32 MFMA fragment layout that the potential kernels rely on.
#include "nmx_common.h"
#include "nmx_api_internal.h"
#include "nmx_wide_models.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_philox_kat(const uint32_t* ctr_key, uint32_t* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* p = ctr_key + 6 * i;
  nmx_u4 c{p[0], p[1], p[2], p[3]};
  nmx_u4 r = nmx_philox4x32_10(c, p[4], p[5]);
  out[4 * i + 0] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

// One wave computes C[32][32] = A[32][K] * B[K][32] with v_mfma_f32_32x32x2_f32,
// using the operand maps documented in cdna_hip_programming.md §3:
//   A: lane l holds A[l&31][k0 + (l>>5)], B: lane l holds B[k0 + (l>>5)][l&31]
//   C: register r of lane l is C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
__global__ void k_mfma_probe(const float* A, const float* B, float* C, int K) {
  int l = threadIdx.x;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += 2) {
    float a = A[(l & 31) * K + k0 + (l >> 5)];
    float b = B[(k0 + (l >> 5)) * 32 + (l & 31)];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    C[row * 32 + (l & 31)] = acc[r];
  }
}

extern "C" int nmx_selftest_philox(const uint32_t* ctr_key, uint32_t* out, int n,
                                   void* stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (n <= 0) return nmx_fail(NMX_ERR_INVALID, "n must be positive");
  hipLaunchKernelGGL(k_philox_kat, dim3((n + 63) / 64), dim3(64), 0, stream, ctr_key, out, n);
  return nmx_check_launch("k_philox_kat");
}

extern "C" int nmx_selftest_mfma(const float* A, const float* B, float* C, int K,
                                 void* stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (K <= 0 || (K & 1)) return nmx_fail(NMX_ERR_INVALID, "K must be positive and even");
  hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, stream, A, B, C, K);
  return nmx_check_launch("k_mfma_probe");
}

// NMX_DCHECK(value == 0) in one thread: prints a failed check in the debug build, nothing in
// the release build (where the check is compiled out).  Returns 1 in the debug build.
__global__ void k_dcheck_probe(int value) { NMX_DCHECK(value == 0); }

extern "C" int nmx_selftest_dcheck(int value, void* stream) {
  hipLaunchKernelGGL(k_dcheck_probe, dim3(1), dim3(1), 0, (hipStream_t)stream, value);
  if (int st = nmx_check_launch("k_dcheck_probe")) return -st;
#ifdef NMX_DEBUG
  return 1;
#else
  return 0;
#endif
}

// nmx_expf_unchecked (the SV row's exp) against the device expf, element by element
__global__ void k_expf_probe(const float* x, float* fast, float* ref, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fast[i] = nmx_expf_unchecked(x[i]);
  ref[i] = expf(x[i]);
}

extern "C" int nmx_selftest_expf(const float* x, float* fast, float* ref, int n, void* stream) {
  if (n <= 0 || !x || !fast || !ref) return nmx_fail(NMX_ERR_INVALID, "expf probe: bad arguments");
  hipLaunchKernelGGL(k_expf_probe, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, fast, ref, n);
  return nmx_check_launch("k_expf_probe");
}
