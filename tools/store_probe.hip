// Store-pattern probe (gfx950): HBM write rate of the epilogue store shapes the conv kernels use.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/store_probe tools/store_probe.hip && /tmp/store_probe
// Every pattern writes the same 256 MiB buffer exactly once (each byte by one lane), 4 waves per workgroup:
//   0  contiguous: a wave-instruction stores 64 lanes x 16 B = 1 KiB contiguous
//   1  32 B runs in 128-B rows: lanes 2j, 2j+1 write 16 B slots 2k, 2k+1 of row j (k = 0..3 over 4 instructions)
//   2  8 B pieces, 4 lanes per 32-B run, 16 rows of 64 B per instruction (the f16 streaming epilogue, 8-byte stores)
//   3  32 B pieces: lane pairs write 32 contiguous bytes of 32 rows of 256 B (one 16 B store per lane)
//   4  the x3 pair-layout epilogue (ym_p2_store4): 64-B rows (16 channels = two [hi x8 | lo x8] chunks), lane (g, c)
//      writes 8 B of hi at row c, byte 32 (g >> 1) + 8 (g & 1), then 8 B of lo 16 bytes further: per instruction 16
//      rows x two 16-B runs
//   5  the lane-pair x3 epilogue (ym_p2_store4_pair): lanes (g, c) of the same 64-B row exchange halves, lane g writes
//      16 B at byte 16 g: per instruction 16 rows x one 64-B run
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void st_contig(float4* p, long n16) {
  const long i0 = (long)blockIdx.x * 256 + threadIdx.x;
  for (long i = i0; i < n16; i += (long)gridDim.x * 256) p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

// pattern 1: rows of 128 B (8 x 16 B slots); a wave covers 32 rows per instruction group: lane l -> row l >> 1,
// slot (l & 1) + 2k for k = 0..3
__global__ __launch_bounds__(256) void st_p1(float4* p, long rows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (long r0 = ((long)blockIdx.x * 4 + wave) * 32; r0 < rows; r0 += (long)gridDim.x * 4 * 32) {
    const long row = r0 + (lane >> 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) p[row * 8 + (lane & 1) + 2 * k] = make_float4(1.f, 2.f, 3.f, 4.f);
  }
}

// pattern 2: rows of 64 B; 8-byte stores, lanes (g, c): row c (16 rows per instruction), bytes 8 g .. (g = 0..3),
// then +32 B in a second instruction
__global__ __launch_bounds__(256) void st_p2(float2* p, long rows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  for (long r0 = ((long)blockIdx.x * 4 + wave) * 16; r0 < rows; r0 += (long)gridDim.x * 4 * 16) {
    const long row = r0 + c;
#pragma unroll
    for (int k = 0; k < 2; ++k) p[row * 8 + g + 4 * k] = make_float2(1.f, 2.f);
  }
}

// pattern 3: rows of 256 B (16 slots); lanes 2j, 2j+1 write slots s, s+1 of row j (32 rows per instruction)
__global__ __launch_bounds__(256) void st_p3(float4* p, long rows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (long r0 = ((long)blockIdx.x * 4 + wave) * 32; r0 < rows; r0 += (long)gridDim.x * 4 * 32) {
    const long row = r0 + (lane >> 1);
#pragma unroll
    for (int k = 0; k < 8; ++k) p[row * 16 + (lane & 1) + 2 * k] = make_float4(1.f, 2.f, 3.f, 4.f);
  }
}

__global__ __launch_bounds__(256) void st_p4(float2* p, long rows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  for (long r0 = ((long)blockIdx.x * 4 + wave) * 16; r0 < rows; r0 += (long)gridDim.x * 4 * 16) {
    float2* q = p + (r0 + c) * 8 + 4 * (g >> 1) + (g & 1);  // float2 units: 32 B = 4, 8 B = 1
    q[0] = make_float2(1.f, 2.f);
    q[2] = make_float2(3.f, 4.f);
  }
}

__global__ __launch_bounds__(256) void st_p5(float4* p, long rows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  for (long r0 = ((long)blockIdx.x * 4 + wave) * 16; r0 < rows; r0 += (long)gridDim.x * 4 * 16)
    p[(r0 + c) * 4 + g] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
  const size_t bytes = 256ull << 20;
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[6] = {"contiguous 1 KiB / instr", "32 B runs, 128-B rows", "8 B x 4 per 64-B row", "32 B runs, 256-B rows",
                          "x3 pair epilogue (2x16 B/row)", "x3 lane-pair epilogue (64 B/row)"};
  for (int grid : {1024, 2048, 4096}) {
    for (int pat = 0; pat < 6; ++pat) {
      auto launch = [&]() {
        if (pat == 0) hipLaunchKernelGGL(st_contig, dim3(grid), dim3(256), 0, 0, (float4*)d, (long)(bytes / 16));
        if (pat == 1) hipLaunchKernelGGL(st_p1, dim3(grid), dim3(256), 0, 0, (float4*)d, (long)(bytes / 128));
        if (pat == 2) hipLaunchKernelGGL(st_p2, dim3(grid), dim3(256), 0, 0, (float2*)d, (long)(bytes / 64));
        if (pat == 3) hipLaunchKernelGGL(st_p3, dim3(grid), dim3(256), 0, 0, (float4*)d, (long)(bytes / 256));
        if (pat == 4) hipLaunchKernelGGL(st_p4, dim3(grid), dim3(256), 0, 0, (float2*)d, (long)(bytes / 64));
        if (pat == 5) hipLaunchKernelGGL(st_p5, dim3(grid), dim3(256), 0, 0, (float4*)d, (long)(bytes / 64));
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      for (int r = 0; r < 10; ++r) launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("grid %5d  %-28s %7.2f TB/s\n", grid, names[pat], bytes * 10.0 / (ms * 1e-3) / 1e12);
    }
  }
  hipFree(d);
  return 0;
}
