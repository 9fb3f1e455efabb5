// Probe: what bounds input_stats (csrc/ym_misc.hip), the forward's first kernel — 21.5 us for the 39 MB yolo11s
// B=8 batch (1.8 TB/s, profiles/r06a_s_b8_x3_kernel_stats.csv).  Variants of the same max reduction, each timed
// alone with HIP events after a 1 GB memset flush (the batch is not L2/MALL-resident when a forward starts):
//   grid x block x float4-loads-per-lane-and-round, with or without the last-block ticket.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_input_stats.hip -o tools/probe_input_stats && ./tools/probe_input_stats
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int f2ord(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}

template <int BS, int U, bool TICKET, int G = 1>
__global__ __launch_bounds__(BS) void stats(const float* __restrict__ x, long n, int* part, int* ticket, int* out) {
  const int tid = threadIdx.x;
  const long n4 = n >> 2;
  const long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long lo = blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  float m = -INFINITY;
  for (long i = lo + tid; lo < hi && i - tid < hi; i += U * BS) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * BS;
      v[u] = x4[j < hi ? j : hi - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) m = fmaxf(m, fmaxf(fmaxf(v[u][0], v[u][1]), fmaxf(v[u][2], v[u][3])));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float wm[BS / 64];
  __shared__ int last;
  if ((tid & 63) == 0) wm[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < BS / 64; ++w) m = fmaxf(m, wm[w]);
    m = fmaxf(m, wm[0]);
    __hip_atomic_store(part + blockIdx.x, f2ord(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (TICKET) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (G == 1) {
        const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == (int)gridDim.x - 1;
      } else {  // two-level: group tickets 256 B apart (blocks b % G), the last of each group takes the top ticket
        const int g = blockIdx.x % G, ng = ((int)gridDim.x - g + G - 1) / G;
        const int t = __hip_atomic_fetch_add(ticket + 64 * (1 + g), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 0;
        if (t == ng - 1) {
          __hip_atomic_store(ticket + 64 * (1 + g), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const int u = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last = u == G - 1;
        }
      }
    } else {
      last = 0;
    }
  }
  __syncthreads();
  if (!last) return;
  int r = f2ord(-INFINITY);
  for (int b = tid; b < (int)gridDim.x; b += BS) r = max(r, __hip_atomic_load(part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) r = max(r, __shfl_xor(r, o));
  __shared__ int wr[BS / 64];
  if ((tid & 63) == 0) wr[tid >> 6] = r;
  __syncthreads();
  if (tid == 0) {
    int q = wr[0];
    for (int w = 1; w < BS / 64; ++w) q = max(q, wr[w]);
    *out = q;
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

#define CK(e)                                                          \
  do {                                                                 \
    hipError_t r_ = (e);                                               \
    if (r_ != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_)); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

template <int BS, int U, bool TICKET, int G = 1>
int run(const char* name, int grid, const float* x, long n, int* part, int* ticket, int* out, char* flush, size_t fb,
        float expect) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < 40; ++it) {
    CK(hipMemsetAsync(flush, it & 255, fb, 0));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((stats<BS, U, TICKET, G>), dim3(grid), dim3(BS), 0, 0, x, n, part, ticket, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 5) ts.push_back(ms * 1000.f);
  }
  std::sort(ts.begin(), ts.end());
  int o;
  CK(hipMemcpy(&o, out, 4, hipMemcpyDeviceToHost));
  const int want = __builtin_bit_cast(int, expect);
  printf("%-34s grid %5d block %4d U %2d ticket %d G %2d: median %6.2f us  min %6.2f us  (%.2f TB/s)  %s\n", name, grid, BS,
         U, (int)TICKET, G, ts[ts.size() / 2], ts[0], n * 4.0 / (ts[ts.size() / 2] * 1e-6) / 1e12,
         TICKET ? (o == want ? "max ok" : "MAX WRONG") : "");
  return 0;
}

int main() {
  const long n = 8L * 3 * 640 * 640;
  std::vector<float> h(n);
  for (long i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.1f;
  h[n / 3] = 255.f;
  float *x;
  int *part, *ticket, *out;
  char* flush;
  const size_t fb = 1ull << 30;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&part, 8192 * 4));
  CK(hipMalloc(&ticket, 256 * 80));
  CK(hipMalloc(&out, 256));
  CK(hipMalloc(&flush, fb));
  CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(ticket, 0, 256 * 80));
  const float expect = 255.f;
  int rc = 0;
  rc |= run<256, 10, true>("current (1024 x 256, U10)", 1024, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 10, false>("current, no ticket", 1024, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 10, true, 16>("1024 x 256, two-level 16", 1024, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 10, true, 32>("1024 x 256, two-level 32", 1024, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 10, true, 64>("1024 x 256, two-level 64", 1024, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<1024, 10, true>("256 x 1024, U10", 256, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<1024, 10, false>("256 x 1024, no ticket", 256, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<1024, 10, true, 16>("256 x 1024, two-level 16", 256, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<512, 10, true, 16>("512 x 512, two-level 16", 512, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<512, 10, false>("512 x 512, no ticket", 512, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 5, true, 32>("2048 x 256 U5, two-level 32", 2048, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 5, false>("2048 x 256 U5, no ticket", 2048, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<1024, 12, true, 16>("200 x 1024 U12, two-level 16", 200, x, n, part, ticket, out, flush, fb, expect);
  rc |= run<256, 10, true, 16>("1024 x 256, two-level 16 again", 1024, x, n, part, ticket, out, flush, fb, expect);
  return rc;
}
