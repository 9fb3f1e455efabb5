// Microbenchmark: per-kernel cost inside a captured HIP graph on this MI355X (dispatch floor), for
//  (a) an empty 1-block kernel, (b) an empty 1024-block kernel, (c) a 512-block kernel touching 8 MB,
//  (d) the same with 48 KB dynamic LDS.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_touch(const float4* __restrict__ in, float4* __restrict__ out, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = in[i];
}
__global__ void k_touch_lds(const float4* __restrict__ in, float4* __restrict__ out, int n) {
  extern __shared__ float s[];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = in[i];
  if (threadIdx.x == 0) s[0] = 1.f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename F>
double time_graph(hipStream_t st, int nk, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed);
  for (int i = 0; i < nk; ++i) launch(st);
  (void)hipStreamEndCapture(st, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 5; ++w) (void)hipGraphLaunch(ge, st);
  (void)hipStreamSynchronize(st);
  const int R = 50;
  auto t0 = std::chrono::high_resolution_clock::now();
  for (int r = 0; r < R; ++r) (void)hipGraphLaunch(ge, st);
  (void)hipStreamSynchronize(st);
  auto t1 = std::chrono::high_resolution_clock::now();
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / R / nk;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int n = (8 << 20) / 16, nbig = (64 << 20) / 16;
  float4 *a, *b;
  CK(hipMalloc(&a, nbig * 16));
  CK(hipMalloc(&b, nbig * 16));
  const int NK = 100;
  printf("empty 1 block      : %.2f us/kernel\n", time_graph(st, NK, [](hipStream_t s) { hipLaunchKernelGGL(k_empty, 1, 64, 0, s); }));
  printf("empty 1024 blocks  : %.2f us/kernel\n", time_graph(st, NK, [](hipStream_t s) { hipLaunchKernelGGL(k_empty, 1024, 256, 0, s); }));
  printf("copy 8MB 512 blocks: %.2f us/kernel\n", time_graph(st, NK, [&](hipStream_t s) { hipLaunchKernelGGL(k_touch, 512, 256, 0, s, a, b, n); }));
  printf("copy 8MB + 48KB LDS: %.2f us/kernel\n", time_graph(st, NK, [&](hipStream_t s) { hipLaunchKernelGGL(k_touch_lds, 512, 256, 48 * 1024, s, a, b, n); }));
  printf("copy 64KB 16 blocks: %.2f us/kernel\n", time_graph(st, NK, [&](hipStream_t s) { hipLaunchKernelGGL(k_touch, 16, 256, 0, s, a, b, 4096); }));
  for (int blocks : {2048, 4096, 8192}) {
    const double us = time_graph(st, NK, [&](hipStream_t s) { hipLaunchKernelGGL(k_touch, blocks, 256, 0, s, a, b, nbig); });
    printf("copy 64MB %5d blocks: %.2f us/kernel = %.0f GB/s (read+write)\n", blocks, us, 2.0 * 64 * 1048576 / us / 1e3);
  }
  return 0;
}
