// Read-bandwidth probe for the forward's first kernel (csrc/ym_misc.hip input_stats): a max-reduce over the fp32
// NCHW batch (8x3x640x640 = 39.3 MB), cold (a 512 MB write between launches evicts L2 and MALL), per layout of the
// reads.  Prints the average kernel time (HIP events around each launch) and the achieved GB/s.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/read_probe.hip -o tools/probe_bin/read_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));            \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline float red4(f32x4 v) { return fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])); }

__device__ inline void block_out(float m, float* out) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float wm[16];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)blockDim.x / 64; ++w) m = fmaxf(m, wm[w]);
    out[blockIdx.x] = m;
  }
}

// contiguous chunk per block, U loads in flight per lane
template <int U>
__global__ void chunk_max(const f32x4* x4, long n4, float* out) {
  const long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long lo = blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  float m = -INFINITY;
  long i = lo + threadIdx.x;
  const int bs = blockDim.x;
  for (; i + (U - 1) * bs < hi; i += U * bs) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x4[i + u * bs];
#pragma unroll
    for (int u = 0; u < U; ++u) m = fmaxf(m, red4(v[u]));
  }
  for (; i < hi; i += bs) m = fmaxf(m, red4(x4[i]));
  block_out(m, out);
}

// grid-stride, U loads per lane per trip
template <int U>
__global__ void stride_max(const f32x4* x4, long n4, float* out) {
  const long st = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  float m = -INFINITY;
  for (; i + (U - 1) * st < n4; i += U * st) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x4[i + u * st];
#pragma unroll
    for (int u = 0; u < U; ++u) m = fmaxf(m, red4(v[u]));
  }
  for (; i < n4; i += st) m = fmaxf(m, red4(x4[i]));
  block_out(m, out);
}

// exactly U float4 per lane, one trip (grid sized to the batch), nontemporal loads
template <int U>
__global__ void tile_max_nt(const f32x4* x4, long n4, float* out) {
  const long base = blockIdx.x * (long)blockDim.x * U + threadIdx.x;
  float m = -INFINITY;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + (long)u * blockDim.x;
    v[u] = i < n4 ? __builtin_nontemporal_load(x4 + i) : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) m = fmaxf(m, red4(v[u]));
  block_out(m, out);
}

template <int U>
__global__ void tile_max(const f32x4* x4, long n4, float* out) {
  const long base = blockIdx.x * (long)blockDim.x * U + threadIdx.x;
  float m = -INFINITY;
  f32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + (long)u * blockDim.x;
    v[u] = i < n4 ? x4[i] : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) m = fmaxf(m, red4(v[u]));
  block_out(m, out);
}

__global__ void scrub(f32x4* p, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    p[i] = f32x4{1, 2, 3, 4};
}

int main() {
  const long n = 8L * 3 * 640 * 640, n4 = n / 4;
  const long sn4 = (512L << 20) / 16;
  f32x4 *x, *s;
  float* out;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&s, sn4 * 16));
  CK(hipMalloc(&out, 1 << 20));
  std::vector<float> h(n);
  for (long i = 0; i < n; ++i) h[i] = (float)((i * 2654435761L) % 1000) * 0.001f;
  CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) -> int {
    float tot = 0, best = 1e9;
    const int iters = 40;
    for (int it = -3; it < iters; ++it) {
      hipLaunchKernelGGL(scrub, dim3(4096), dim3(256), 0, 0, s, sn4);
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (it >= 0) {
        tot += ms;
        best = ms < best ? ms : best;
      }
    }
    CK(hipGetLastError());
    const float us = tot / iters * 1000;
    printf("%-28s avg %7.2f us  best %7.2f us  %6.0f GB/s\n", name, us, best * 1000, n * 4 / (us * 1e3));
    return 0;
  };
#define RUNK(name, K, grid, blk) run(name, [&] { hipLaunchKernelGGL(K, dim3(grid), dim3(blk), 0, 0, x, n4, out); })
  RUNK("chunk8 1024x256", chunk_max<8>, 1024, 256);
  RUNK("chunk8 2048x256", chunk_max<8>, 2048, 256);
  RUNK("chunk4 4096x256", chunk_max<4>, 4096, 256);
  RUNK("stride4 2048x256", stride_max<4>, 2048, 256);
  RUNK("stride4 4096x256", stride_max<4>, 4096, 256);
  RUNK("stride2 8192x256", stride_max<2>, 8192, 256);
  RUNK("tile8 x256", tile_max<8>, (n4 + 2047) / 2048, 256);
  RUNK("tile4 x256", tile_max<4>, (n4 + 1023) / 1024, 256);
  RUNK("tile16 x256", tile_max<16>, (n4 + 4095) / 4096, 256);
  RUNK("tile8 nt x256", tile_max_nt<8>, (n4 + 2047) / 2048, 256);
  RUNK("tile4 x512", tile_max<4>, (n4 + 2047) / 2048, 512);
  RUNK("tile8 x1024", tile_max<8>, (n4 + 8191) / 8192, 1024);
  // warm (no scrub): what L2/MALL-resident reads give
  float ms;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(tile_max<8>, dim3((n4 + 2047) / 2048), dim3(256), 0, 0, x, n4, out);
  CK(hipEventRecord(e0, 0));
  for (int w = 0; w < 40; ++w) hipLaunchKernelGGL(tile_max<8>, dim3((n4 + 2047) / 2048), dim3(256), 0, 0, x, n4, out);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s avg %7.2f us (back-to-back, warm)\n", "tile8 x256 warm", ms * 1000 / 40);
  return 0;
}
