// Launch-overhead floor on the box: back-to-back launches of near-empty kernels shaped like the
// covtype tail launches (the fused step: 32 x 512 threads, 48 KB static LDS; the finalize: 56 x
// 256; the narrow tail: 256 x 512, 158 KB dynamic LDS), timed with hipEvents over 2000 launches.
// Each kernel writes one word per block so it is not elided.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void k_step_like(int* out) {
  __shared__ float lds[23 * 512 + 23 * 16];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (int)lds[5];
}
__global__ __launch_bounds__(256) void k_fin_like(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x + blockIdx.y * 64] = 1;
}
__global__ __launch_bounds__(512) void k_tail_like(int* out) {
  extern __shared__ char dl[];
  dl[threadIdx.x] = 1;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = dl[3];
}

template <class F>
float time_it(F f, int n) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) f();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < n; ++i) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.0f / n;
}

int main() {
  int* out;
  if (hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  (void)hipFuncSetAttribute((const void*)k_tail_like, hipFuncAttributeMaxDynamicSharedMemorySize, 161792);
  const int n = 2000;
  float t1 = time_it([&] { hipLaunchKernelGGL(k_step_like, dim3(32), dim3(512), 0, 0, out); }, n);
  float t2 = time_it([&] { hipLaunchKernelGGL(k_fin_like, dim3(1, 56), dim3(256), 0, 0, out); }, n);
  float t3 = time_it([&] { hipLaunchKernelGGL(k_tail_like, dim3(256), dim3(512), 161792, 0, out); }, n);
  float t4 = time_it([&] {
    hipLaunchKernelGGL(k_step_like, dim3(32), dim3(512), 0, 0, out);
    hipLaunchKernelGGL(k_tail_like, dim3(256), dim3(512), 161792, 0, out);
    hipLaunchKernelGGL(k_fin_like, dim3(1, 56), dim3(256), 0, 0, out);
  }, n);
  printf("us per launch: step-like %.2f  finalize-like %.2f  tail-like %.2f  triple %.2f\n", t1, t2, t3, t4);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
