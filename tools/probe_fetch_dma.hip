// Probe: how gfx950's FETCH_SIZE counts LDS-DMA loads (buffer_load ... lds, 16 B per lane — the conv_dma ring's
// loads) against plain 16 B/lane global loads.  MI355X_MICROARCH.md §HBM prescribes FETCH_SIZE x2 for wide
// coalesced 16 B/lane reads; tools/rocprof_summary.py applies it to every conv kernel.  Each kernel reads the same
// 256 MiB buffer exactly once (no reuse), so the raw FETCH_SIZE of each dispatch against 262,144 KiB gives the factor.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_fetch_dma.hip -o tools/probe_fetch_dma
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- ./tools/probe_fetch_dma
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr long kBytes = 256L << 20;
constexpr int kBlocks = 4096, kThreads = 256;

// plain: every lane loads 16 B per step, the block a contiguous 4 KiB per step; a checksum keeps the loads alive
__global__ __launch_bounds__(kThreads) void plain_read(const u32x4* __restrict__ x, unsigned* out) {
  const long n = kBytes / 16, per = n / kBlocks;
  const u32x4* p = x + blockIdx.x * per;
  unsigned s = 0;
  for (long i = threadIdx.x; i < per; i += kThreads) {
    const u32x4 v = p[i];
    s ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (s == 0x12345678u) out[0] = s;  // (never true for the data below; keeps the loads)
}

// LDS-DMA: the same bytes, each wave instruction moving 64 lanes x 16 B into a 1 KiB LDS slot (conv_dma's dma16)
__global__ __launch_bounds__(kThreads) void dma_read(const void* x, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 1024];
  const long per = kBytes / kBlocks;  // bytes per block
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(static_cast<const char*>(x)) + blockIdx.x * per, 0, (int)per, 0x00020000);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (long o = 0; o < per; o += kThreads * 16) {
    const unsigned voff = (unsigned)(o + (w * 64 + lane) * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(lds + w * 1024), 16, voff, 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && *reinterpret_cast<unsigned*>(lds) == 0x12345678u) out[0] = 1;
}

int main() {
  void* x;
  unsigned* out;
  if (hipMalloc(&x, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(x, 0x5A, kBytes);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(plain_read, dim3(kBlocks), dim3(kThreads), 0, 0, static_cast<const u32x4*>(x), out);
    hipLaunchKernelGGL(dma_read, dim3(kBlocks), dim3(kThreads), 0, 0, x, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("probe_fetch_dma: 3 x (plain_read, dma_read) over %ld MiB each\n", kBytes >> 20);
  return 0;
}
