// Quantized-conv epilogue helpers shared by the int8 kernels (csrc/ym_conv_i8.hip, ym_conv_i8_stream.hip).
// Numerics: oracle/quant.py (torch.ao quantized::conv2d restated); every float step rounds once, as torch's separate
// fp32 ops do (ym_opaque keeps hipcc from contracting a multiply into the following add).
#pragma once
#include "ym_common.h"

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef signed char i8x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// quantized::conv2d output requantisation
__device__ __forceinline__ int requant_out(int acc, float sasw, float bias, const QRec* Q) {
  const float y = ym_opaque((float)acc * sasw) + bias;  // two roundings (no FMA), as torch's mul then add
  return clampi((int)rintf(__fmul_rn(y, Q->inv_sc)) + Q->zc, Q->qlo, Q->qhi);
}
// quantize a float into a stored tensor: returns the int8 storage value q - 128
__device__ __forceinline__ int quant_store(float v, float inv, int z, int lo, int hi) {
  return clampi((int)rintf(__fmul_rn(v, inv)) + z, lo, hi) - 128;
}
__device__ __forceinline__ float deq(int q, int z, float s) { return ym_opaque((float)(q - z) * s); }
__device__ __forceinline__ int pack4(const int* v) {
  return (v[0] & 0xFF) | ((v[1] & 0xFF) << 8) | ((v[2] & 0xFF) << 16) | ((unsigned)(v[3] & 0xFF) << 24);
}
