// Stand-alone timing of the NMS key sort (csrc/ym_misc.hip bitonic_sort_desc) in one 1024-thread workgroup over
// n2 keys in LDS, as nms_image's blocked path runs it; cycle stamps of thread 0 around the load and the sort.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sort_probe.hip -o tools/ab/sort_probe -Lyolo-infer_amd/yolomi -lyolomi \
//     -Wl,-rpath,'$ORIGIN/../../yolo-infer_amd/yolomi'   (the other kernels' launchers come from the library)
//   tools/ab/sort_probe [n2]
#include "../yolo-infer_amd/csrc/ym_misc.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ __launch_bounds__(NMS_T) void sort_probe(const unsigned long long* in, unsigned long long* out, int n2,
                                                  long long* stamps) {
  __shared__ __attribute__((aligned(16))) unsigned long long arena[NMS_SORT];
  const int tid = threadIdx.x;
  const long long t0 = wall_clock64();
  for (int i = tid; i < n2; i += NMS_T) arena[i] = in[i];
  __syncthreads();
  const long long t1 = wall_clock64();
  bitonic_sort_desc(arena, n2, tid);
  const long long t2 = wall_clock64();
  for (int i = tid; i < n2; i += NMS_T) out[i] = arena[i];
  if (tid == 0) {
    stamps[0] = t1 - t0;
    stamps[1] = t2 - t1;
  }
}

int main(int argc, char** argv) {
  const int n2 = argc > 1 ? atoi(argv[1]) : 16384;
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
    hipLaunchKernelGGL(sort_probe, dim3(1), dim3(NMS_T), 0, 0, din, dout, n2, ds);
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
    printf("n2 %d: kernel %.1f us (event), load %.2f us, sort %.2f us (100 MHz wall clock), sorted %s\n", n2,
           ms * 1e3, s[0] / 100.0, s[1] / 100.0, ok ? "yes" : "NO");
  }
  return 0;
}
