// Kernel-boundary cost with real data hand-offs, shaped like a covtype tail launch: a producer
// (256 x 512 threads) writes a slab image of `bytes` (row splits x values x chains, f32), a
// reducer (56 x 256) sums the slabs of its value row in fixed order and writes one row, and a
// consumer (2 x 512) reads the reduced rows.  The producer's slab stores are plain or
// nontemporal; the question is whether a hand-off of freshly written lines costs more than the
// 1.8 us an empty kernel costs in the trace (the finalize's trace duration is ~8 us above its
// blocks' span).  Timed with hipEvents over 2000 triples; run under rocprofv3 --kernel-trace
// --stats for per-kernel durations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int S = 256, NV = 56;

template <bool NT>
__global__ __launch_bounds__(512) void k_produce(float* slab, int chains, int iter) {
  // one split per block: NV x chains values, thread t writes values t, t + 512, ...
  float* o = slab + (size_t)blockIdx.x * NV * chains;
  for (int i = threadIdx.x; i < NV * chains; i += 512) {
    float v = (float)(i + iter) * 1e-3f;
    if constexpr (NT) __builtin_nontemporal_store(v, o + i);
    else o[i] = v;
  }
}

__global__ __launch_bounds__(256) void k_reduce(const float* slab, float* rows, int chains) {
  // block (x, y): value row y, chains x*256 .. ; fixed-order sum over the S splits
  const int v = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= chains) return;
  float acc = 0.f;
#pragma unroll 8
  for (int s = 0; s < S; ++s) acc += slab[((size_t)s * NV + v) * chains + c];
  rows[(size_t)v * chains + c] = acc;
}

__global__ __launch_bounds__(512) void k_consume(const float* rows, float* out, int chains) {
  const int c = blockIdx.x * 16 + (threadIdx.x >> 5), l = threadIdx.x & 31;
  if (c >= chains) return;
  float acc = 0.f;
  for (int v = l; v < NV; v += 32) acc += rows[(size_t)v * chains + c];
  if (l == 0) out[c] = acc;
}

__global__ __launch_bounds__(512) void k_empty(float* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = 1.f;
}

template <class F>
static float time_it(F f, int n) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) f(i);
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < n; ++i) f(i);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.0f / n;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2000;
  float *slab, *rows, *out;
  const int cmax = 4096;
  if (hipMalloc(&slab, (size_t)S * NV * cmax * 4) != hipSuccess) return 1;
  if (hipMalloc(&rows, (size_t)NV * cmax * 4) != hipSuccess) return 1;
  if (hipMalloc(&out, cmax * 4) != hipSuccess) return 1;
  const int only = argc > 2 ? atoi(argv[2]) : 0;
  for (int chains : {32, 512, 4096}) {
    if (only && chains != only) continue;
    const int rb = (chains + 255) / 256, cb = (chains + 15) / 16;
    float te = time_it([&](int) {
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(512), 0, 0, out);
      hipLaunchKernelGGL(k_empty, dim3(56), dim3(256), 0, 0, out);
      hipLaunchKernelGGL(k_empty, dim3(cb), dim3(512), 0, 0, out);
    }, n);
    float tp = time_it([&](int i) {
      hipLaunchKernelGGL(k_produce<false>, dim3(S), dim3(512), 0, 0, slab, chains, i);
      hipLaunchKernelGGL(k_reduce, dim3(rb, NV), dim3(256), 0, 0, slab, rows, chains);
      hipLaunchKernelGGL(k_consume, dim3(cb), dim3(512), 0, 0, rows, out, chains);
    }, n);
    float tn = time_it([&](int i) {
      hipLaunchKernelGGL(k_produce<true>, dim3(S), dim3(512), 0, 0, slab, chains, i);
      hipLaunchKernelGGL(k_reduce, dim3(rb, NV), dim3(256), 0, 0, slab, rows, chains);
      hipLaunchKernelGGL(k_consume, dim3(cb), dim3(512), 0, 0, rows, out, chains);
    }, n);
    float tr = time_it([&](int) {
      hipLaunchKernelGGL(k_reduce, dim3(rb, NV), dim3(256), 0, 0, slab, rows, chains);
    }, n);
    printf("chains %4d slab %.2f MB: empty triple %.2f us, plain triple %.2f us, nontemporal triple %.2f us, "
           "reduce alone (warm slabs) %.2f us\n",
           chains, (double)S * NV * chains * 4 / 1e6, te, tp, tn, tr);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
