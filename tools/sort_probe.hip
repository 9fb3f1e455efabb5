// Stand-alone timing of the NMS key sort (csrc/ym_misc.hip bitonic_sort_desc) in one 1024-thread workgroup over
// n2 keys in LDS, as nms_image's blocked path runs it; cycle stamps of thread 0 around the load and the sort.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sort_probe.hip -o tools/ab/sort_probe -Lyolo-infer_amd/yolomi -lyolomi \
//     -Wl,-rpath,'$ORIGIN/../../yolo-infer_amd/yolomi'   (the other kernels' launchers come from the library)
//   tools/ab/sort_probe [n2] [variant: 0 bitonic_sort_desc, 1 register-tiled]
#include "../yolo-infer_amd/csrc/ym_misc.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>


// the register-tiled variant of the same network (tried in round 5): NMS_T threads x K keys, key slot r of thread t
// is element e = K t + r; strides below K inside a thread, below 64 K by 64-bit shuffles, larger through LDS ([r][t])
template <int K, int S>
__device__ __forceinline__ void cx_local(unsigned long long* v, int e0, int size) {
#pragma unroll
  for (int r = 0; r < K; ++r) {
    if (r & S) continue;
    const bool desc = ((e0 + r) & size) == 0;
    const unsigned long long x = v[r], y = v[r | S];
    if ((x < y) == desc) { v[r] = y; v[r | S] = x; }
  }
}
template <int K>
__device__ __forceinline__ void sort_reg_desc(unsigned long long* k, int tid) {
  constexpr int n2 = K * NMS_T;
  unsigned long long v[K];
#pragma unroll
  for (int r = 0; r < K; ++r) v[r] = k[r * NMS_T + tid];
  const int e0 = K * tid;
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride < K) {
        switch (stride) {
          case 1: cx_local<K, 1>(v, e0, size); break;
          case 2: if constexpr (K > 2) cx_local<K, 2>(v, e0, size); break;
          case 4: if constexpr (K > 4) cx_local<K, 4>(v, e0, size); break;
          default: if constexpr (K > 8) cx_local<K, 8>(v, e0, size); break;
        }
      } else {
        const int lm = stride / K;
        const bool lo = (tid & lm) == 0;
        if (lm < 64) {
#pragma unroll
          for (int r = 0; r < K; ++r) {
            const unsigned long long o = __shfl_xor(v[r], lm);
            const bool keep_max = lo == (((e0 + r) & size) == 0);
            v[r] = keep_max ? (v[r] > o ? v[r] : o) : (v[r] < o ? v[r] : o);
          }
        } else {
          __syncthreads();
#pragma unroll
          for (int r = 0; r < K; ++r) k[r * NMS_T + tid] = v[r];
          __syncthreads();
#pragma unroll
          for (int r = 0; r < K; ++r) {
            const unsigned long long o = k[r * NMS_T + (tid ^ lm)];
            const bool keep_max = lo == (((e0 + r) & size) == 0);
            v[r] = keep_max ? (v[r] > o ? v[r] : o) : (v[r] < o ? v[r] : o);
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < K; ++r) k[e0 + r] = v[r];
  __syncthreads();
}

__global__ __launch_bounds__(NMS_T) void sort_probe(const unsigned long long* in, unsigned long long* out, int n2,
                                                  long long* stamps, int variant) {
  __shared__ __attribute__((aligned(16))) unsigned long long arena[NMS_SORT];
  const int tid = threadIdx.x;
  const long long t0 = wall_clock64();
  for (int i = tid; i < n2; i += NMS_T) arena[i] = in[i];
  __syncthreads();
  const long long t1 = wall_clock64();
  if (variant == 1 && n2 == 16 * NMS_T) sort_reg_desc<16>(arena, tid);
  else if (variant == 1 && n2 == 8 * NMS_T) sort_reg_desc<8>(arena, tid);
  else if (variant == 1 && n2 == 2 * NMS_T) sort_reg_desc<2>(arena, tid);
  else bitonic_sort_desc(arena, n2, tid);
  const long long t2 = wall_clock64();
  for (int i = tid; i < n2; i += NMS_T) out[i] = arena[i];
  if (tid == 0) {
    stamps[0] = t1 - t0;
    stamps[1] = t2 - t1;
  }
}

int main(int argc, char** argv) {
  const int n2 = argc > 1 ? atoi(argv[1]) : 16384;
  const int variant = argc > 2 ? atoi(argv[2]) : 0;  // 0: bitonic_sort_desc, 1: the register-tiled network
  std::vector<unsigned long long> h(n2);
  std::mt19937_64 g(7);
  for (auto& v : h) v = g();
  unsigned long long *din, *dout;
  long long* ds;
  if (hipMalloc(&din, n2 * 8) || hipMalloc(&dout, n2 * 8) || hipMalloc(&ds, 16)) return 1;
  hipMemcpy(din, h.data(), n2 * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(sort_probe, dim3(1), dim3(NMS_T), 0, 0, din, dout, n2, ds, variant);
    hipEventRecord(e1, 0);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    long long s[2];
    hipMemcpy(s, ds, 16, hipMemcpyDeviceToHost);
    std::vector<unsigned long long> o(n2);
    hipMemcpy(o.data(), dout, n2 * 8, hipMemcpyDeviceToHost);
    bool ok = true;
    for (int i = 1; i < n2; ++i) ok &= o[i - 1] >= o[i];
    printf("variant %d n2 %d: kernel %.1f us (event), load %.2f us, sort %.2f us (100 MHz wall clock), sorted %s\n", variant, n2,
           ms * 1e3, s[0] / 100.0, s[1] / 100.0, ok ? "yes" : "NO");
  }
  return 0;
}
