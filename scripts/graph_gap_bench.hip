// Microbenchmark (not part of the library): the per-launch cost of a chain of dependent kernels
// issued on one stream vs the same chain captured into a hipGraph and replayed -- the question
// behind "capture the NUTS launch loop in a graph" (launch loop).  Kernels of a fixed
// grid (G workgroups of 256 threads) spin for `iters` FMA rounds and store one float each; the
// per-launch time minus the kernel's own duration is the inter-kernel gap.
//   hipcc -O3 --offload-arch=gfx950 scripts/graph_gap_bench.hip -o /tmp/ggb && /tmp/ggb
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

__global__ __launch_bounds__(256) void k_work(float* p, int iters, float a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  float x = p[i];
  for (int k = 0; k < iters; ++k) x = fmaf(x, a, 0.5f);
  p[i] = x;
}

constexpr int BATCH = 16;   // launches per graph (the engine polls every 16 launches)
constexpr int ROUNDS = 64;  // graph replays per measurement

static float time_stream(hipStream_t s, float* p, int G, int iters, int n) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_work, dim3(G), dim3(256), 0, s, p, iters, 0.999f);
  CHECK(hipEventRecord(e1, s));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms * 1000.f / n;
}

static float time_graph(hipStream_t s, float* p, int G, int iters) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < BATCH; ++i) hipLaunchKernelGGL(k_work, dim3(G), dim3(256), 0, s, p, iters, 0.999f);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CHECK(hipGraphLaunch(ge, s));  // warm
  CHECK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, s));
  for (int r = 0; r < ROUNDS; ++r) CHECK(hipGraphLaunch(ge, s));
  CHECK(hipEventRecord(e1, s));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return ms * 1000.f / (ROUNDS * BATCH);
}

static float time_single(hipStream_t s, float* p, int G, int iters) {
  // one launch between two syncs, events around it: the kernel's own duration (+ event cost)
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float tot = 0.f;
  const int n = 32;
  for (int i = 0; i < n; ++i) {
    CHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_work, dim3(G), dim3(256), 0, s, p, iters, 0.999f);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return tot * 1000.f / n;
}

int main() {
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* p;
  const int GMAX = 4096;
  CHECK(hipMalloc(&p, (size_t)GMAX * 256 * sizeof(float)));
  CHECK(hipMemset(p, 0, (size_t)GMAX * 256 * sizeof(float)));
  printf("%6s %7s %10s %12s %11s\n", "grid", "iters", "single_us", "stream_us/l", "graph_us/l");
  const int grids[] = {32, 256, 2048};
  const int iterss[] = {0, 2000, 8000, 30000};
  for (int G : grids)
    for (int it : iterss) {
      time_stream(s, p, G, it, 64);  // warm
      const float t1 = time_single(s, p, G, it);
      const float ts = time_stream(s, p, G, it, ROUNDS * BATCH);
      const float tg = time_graph(s, p, G, it);
      printf("%6d %7d %10.2f %12.2f %11.2f\n", G, it, t1, ts, tg);
    }
  CHECK(hipFree(p));
  CHECK(hipStreamDestroy(s));
  return 0;
}
