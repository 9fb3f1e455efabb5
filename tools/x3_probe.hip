// Probe: does v_mfma_f32_32x32x16_f16 keep fp16 subnormal inputs (the lo halves of the split-f16 "x3" plan)?
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/x3_probe tools/x3_probe.hip && tools/bin/x3_probe
// A = 1 on one K slot, B = a subnormal (and a normal) value: the product must come back unchanged.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const float* vals, float* out) {
  const int lane = threadIdx.x;
  f16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
  // row n = lane&31 of A, K slot 0 (lane half 0): A[n][0] = 1; B[0][m] = vals[m] for column m = lane&31
  if (lane < 32) {
    a[0] = (f16)1.0f;
    b[0] = (f16)vals[lane];
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  // D[n][m]: lane holds column m = lane&31, rows (r&3) + 8(r>>2) + 4(lane>>5); row 0 = acc[0] of lanes 0..31
  if (lane < 32) out[lane] = acc[0];
  // the f32 -> f16 conversion of a subnormal value (v_cvt_f16_f32 under the default fp16 denormal mode)
  if (lane < 32) out[32 + lane] = (float)(f16)vals[lane];
}

int main() {
  float h[32];
  for (int i = 0; i < 32; ++i) h[i] = (i + 1) * 5.96046448e-08f * (i < 16 ? 1.0f : 4096.0f);
  float *dv, *dout;
  hipMalloc(&dv, 128);
  hipMalloc(&dout, 256);
  hipMemcpy(dv, h, 128, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dv, dout);
  float o[64];
  hipMemcpy(o, dout, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; ++i) {
    const float want = (float)(f16)h[i];
    printf("in %.6g  cvt %.6g  mfma %.6g%s\n", h[i], o[32 + i], o[i], o[i] == want ? "" : "  <-- differs");
    bad += o[i] != want;
  }
  printf(bad ? "MFMA f16 subnormals: FLUSHED/changed (%d)\n" : "MFMA f16 subnormals: preserved\n", bad);
  return 0;
}
