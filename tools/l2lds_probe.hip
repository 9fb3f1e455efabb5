// Probe: chip-wide L2-hit read rate into LDS / VGPRs by load path (standalone; not part of the library).
//   hipcc -O3 --offload-arch=gfx950 tools/l2lds_probe.hip -o gpurun_out/l2lds_probe && gpurun_out/l2lds_probe
// Every workgroup re-reads a window of a 2 MiB buffer (L2-resident after the first pass) R times, 16 B per lane per
// instruction, D instructions in flight per wave:
//   mode 0: buffer_load ... lds (LDS-DMA), counted vmcnt waits
//   mode 1: global_load_dwordx4 into VGPRs, then ds_write_b128
//   mode 2: global_load_dwordx4 into VGPRs only (values folded so the loads are live)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int D, int MODE>
__global__ __launch_bounds__(256) void probe(const u32x4* __restrict__ buf, unsigned nvec, int R, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char lds[D * 4 * 1024];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(buf), 0, nvec * 16, 0x00020000);
  unsigned base = (blockIdx.x * 4096u + wave * 64u * D) % (nvec - 64u * D * 4u);
  u32x4 accv = {0, 0, 0, 0};
  for (int r = 0; r < R; ++r) {
    const unsigned b = (base + (unsigned)r * 8192u) % (nvec - 64u * D * 4u);
    if constexpr (MODE == 0) {
#pragma unroll
      for (int d = 0; d < D; ++d)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + (wave * D + d) * 1024), 16,
                                                 (b + d * 64u + lane) * 16u, 0, 0, 0);
      __builtin_amdgcn_s_waitcnt(0x0F70);
    } else {
      u32x4 v[D];
#pragma unroll
      for (int d = 0; d < D; ++d) v[d] = buf[b + d * 64u + lane];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if constexpr (MODE == 1) *reinterpret_cast<u32x4*>(lds + (wave * D + d) * 1024 + lane * 16) = v[d];
        else accv ^= v[d];
      }
    }
  }
  __syncthreads();
  if (MODE == 2) {
    if ((accv.x ^ accv.y ^ accv.z ^ accv.w) == 0x12345u) out[0] = 1;
  } else if (tid == 0 && lds[5] == 77) {
    out[0] = 2;
  }
}

template <int D, int MODE>
void run(const u32x4* buf, unsigned nvec, unsigned* out, int grid) {
  const int R = 64;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) probe<D, MODE><<<grid, 256>>>(buf, nvec, R, out);
  hipEventRecord(e0);
  const int reps = 20;
  for (int w = 0; w < reps; ++w) probe<D, MODE><<<grid, 256>>>(buf, nvec, R, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)grid * 256 * 16 * D * R * reps;
  printf("mode %d D %2d grid %5d: %8.1f GB/s chip, %6.1f GB/s per CU, %.2f us per launch\n", MODE, D, grid,
         bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e9 / 256, ms * 1e3 / reps);
}

int main() {
  const unsigned nvec = (2u << 20) / 16;
  u32x4* buf;
  unsigned* out;
  hipMalloc(&buf, nvec * 16);
  hipMalloc(&out, 16);
  hipMemset(buf, 1, nvec * 16);
  for (int grid : {256, 512, 1024}) {
    run<2, 0>(buf, nvec, out, grid);
    run<4, 0>(buf, nvec, out, grid);
    run<8, 0>(buf, nvec, out, grid);
    run<2, 1>(buf, nvec, out, grid);
    run<4, 1>(buf, nvec, out, grid);
    run<8, 1>(buf, nvec, out, grid);
    run<8, 2>(buf, nvec, out, grid);
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
