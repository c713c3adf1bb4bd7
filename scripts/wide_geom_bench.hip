// Microbenchmark of the wide-step memory geometry (not part of the library): how fast can a
// kernel with k_wide_v2's shape (grid = 64-chain groups x 32-row slices, 4 waves per block,
// chain-major [D][ldc] rows of 256 B) stream NI input and NO output vectors, vs the same
// bytes as one flat float4 stream.  Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 scripts/wide_geom_bench.hip -o /tmp/wgb && /tmp/wgb 2519 1024
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int NI = 5, NO = 3;

// geometry of k_wide_v2: block = 64 chains x one slice of SW rows, wave w rows w, w+4, ...;
// RB rows per round (loads of RB rows, then their stores)
template <int RB>
__global__ __launch_bounds__(256) void k_geom(const float* const* in, float* const* out, int D, int ldc, int sw) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int d0 = blockIdx.y * sw, d1 = min(D, d0 + sw);
  for (int d = d0 + wv; d < d1; d += 4 * RB) {
    float x[RB][NI];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int i = 0; i < NI; ++i) x[r][i] = (d + 4 * r < d1) ? in[i][(size_t)(d + 4 * r) * ldc + c] : 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (d + 4 * r >= d1) break;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i) s += x[r][i];
#pragma unroll
      for (int o = 0; o < NO; ++o) out[o][(size_t)(d + 4 * r) * ldc + c] = s + o;
    }
  }
}

__global__ void k_flat(const float4* const* in, float4* const* out, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 s = in[0][i];
#pragma unroll
    for (int k = 1; k < NI; ++k) {
      float4 v = in[k][i];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) out[o][i] = s;
  }
}

int main(int argc, char** argv) {
  const int D = argc > 1 ? atoi(argv[1]) : 2519;
  const int C = argc > 2 ? atoi(argv[2]) : 1024;
  const int ldc = (C + 63) / 64 * 64;
  const size_t n = (size_t)D * ldc;
  float* bufs[NI + NO];
  for (int i = 0; i < NI + NO; ++i) {
    CHECK(hipMalloc(&bufs[i], n * 4));
    CHECK(hipMemset(bufs[i], 0, n * 4));
  }
  float** dptr;
  CHECK(hipMalloc(&dptr, sizeof(bufs)));
  CHECK(hipMemcpy(dptr, bufs, sizeof(bufs), hipMemcpyHostToDevice));
  const float* const* in = (const float* const*)dptr;
  float* const* out = dptr + NI;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const double bytes = (double)(NI + NO) * n * 4;
  auto report = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipEventRecord(a));
    const int reps = 50;
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    printf("%-28s D=%d C=%d  %8.1f us  %7.2f TB/s\n", name, D, C, us, bytes / (us * 1e-6) / 1e12);
  };
  for (int sw : {32, 64, 128}) {
    const dim3 grid(ldc / 64, (D + sw - 1) / sw);
    char nm[64];
    snprintf(nm, sizeof nm, "geom sw=%d rows/round=1", sw);
    report(nm, [&] { hipLaunchKernelGGL(k_geom<1>, grid, dim3(256), 0, 0, in, out, D, ldc, sw); });
    snprintf(nm, sizeof nm, "geom sw=%d rows/round=2", sw);
    report(nm, [&] { hipLaunchKernelGGL(k_geom<2>, grid, dim3(256), 0, 0, in, out, D, ldc, sw); });
    snprintf(nm, sizeof nm, "geom sw=%d rows/round=8", sw);
    report(nm, [&] { hipLaunchKernelGGL(k_geom<8>, grid, dim3(256), 0, 0, in, out, D, ldc, sw); });
  }
  report("flat float4", [&] {
    hipLaunchKernelGGL(k_flat, dim3(2048), dim3(256), 0, 0, (const float4* const*)in, (float4* const*)out, n / 4);
  });
  report("empty launch", [&] { hipLaunchKernelGGL(k_flat, dim3(1), dim3(64), 0, 0, (const float4* const*)in, (float4* const*)out, (size_t)0); });
  return 0;
}
