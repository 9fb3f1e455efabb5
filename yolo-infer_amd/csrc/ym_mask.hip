// Instance-mask assembly of the Segment head: Ultralytics `ops.process_mask(proto, coef, boxes, shape, upsample=True)`
// as the segmentation predictor calls it for tensor sources (reached from `YOLO11Model.predict`,
// /root/reference/core/model.py:133), then the non-empty filter of the predictor's result construction.
//   1. mask_lowres: m[d](y, x) = Σ_c coef[d][c] · proto[b](y, x, c), zeroed outside the box scaled to prototype
//      resolution (crop_mask: x1·r ≤ x < x2·r, same for y, compared in fp32 as torch does on float aranges);
//   2. mask_upsample: bilinear resize to (H, W) with align_corners=False (torch upsample_bilinear2d source index
//      (dst + 0.5)·in/out − 0.5 clamped at 0, neighbour clamped at in − 1), then > 0 → one byte per pixel; a
//      ballot per wave sets the detection's non-empty flag.
// Both kernels are bandwidth-light per pixel; the (n, H, W) byte masks are the dominant traffic (n · H · W bytes).
#include "ym_common.h"

namespace {

__device__ __forceinline__ int image_of(const int* off, int B, int d) {
  int b = 0;
  while (b + 1 < B && off[b + 1] <= d) ++b;
  return b;
}

__global__ __launch_bounds__(256) void mask_lowres(const MaskArgs a) {
  const int d = blockIdx.y;
  const int b = image_of(a.offsets, a.B, d);
  const float* row = a.dets + ((size_t)b * a.max_det + (d - a.offsets[b])) * a.no;
  __shared__ float coef[64];
  if (threadIdx.x < a.nm) coef[threadIdx.x] = row[6 + threadIdx.x];
  __syncthreads();
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= a.MH * a.MW) return;
  const int y = p / a.MW, x = p - (p / a.MW) * a.MW;
  // crop_mask on boxes scaled by (mw / iw, mh / ih)
  const float rw = (float)a.MW / (float)a.W, rh = (float)a.MH / (float)a.H;
  const float bx1 = row[0] * rw, by1 = row[1] * rh, bx2 = row[2] * rw, by2 = row[3] * rh;
  const bool in = (float)x >= bx1 && (float)x < bx2 && (float)y >= by1 && (float)y < by2;
  float v = 0.f;
  if (in) {
    const f32x4* pr = reinterpret_cast<const f32x4*>(a.proto + ((size_t)b * a.MH * a.MW + p) * a.nm);
#pragma unroll 8
    for (int c4 = 0; c4 < a.nm / 4; ++c4) {
      const f32x4 q = pr[c4];
      v = fmaf(coef[4 * c4], q[0], v);
      v = fmaf(coef[4 * c4 + 1], q[1], v);
      v = fmaf(coef[4 * c4 + 2], q[2], v);
      v = fmaf(coef[4 * c4 + 3], q[3], v);
    }
  }
  a.lowres[(size_t)d * a.MH * a.MW + p] = v;
}

__global__ __launch_bounds__(256) void mask_upsample(const MaskArgs a) {
  const int d = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  bool on = false;
  if (p < a.H * a.W) {
    const int oy = p / a.W, ox = p - (p / a.W) * a.W;
    const float sy_ = (float)a.MH / (float)a.H, sx_ = (float)a.MW / (float)a.W;
    float fy = ((float)oy + 0.5f) * sy_ - 0.5f, fx = ((float)ox + 0.5f) * sx_ - 0.5f;
    fy = fy < 0.f ? 0.f : fy;
    fx = fx < 0.f ? 0.f : fx;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 < a.MH - 1 ? y0 + 1 : y0, x1 = x0 < a.MW - 1 ? x0 + 1 : x0;
    const float ly = fy - (float)y0, lx = fx - (float)x0;
    const float* m = a.lowres + (size_t)d * a.MH * a.MW;
    const float v = (1.f - ly) * ((1.f - lx) * m[y0 * a.MW + x0] + lx * m[y0 * a.MW + x1]) +
                    ly * ((1.f - lx) * m[y1 * a.MW + x0] + lx * m[y1 * a.MW + x1]);
    on = v > 0.f;
    a.masks[(size_t)d * a.H * a.W + p] = on ? 1 : 0;
  }
  const unsigned long long bal = __ballot(on);  // every lane reaches this (no early return above)
  if (bal && (threadIdx.x & 63) == __builtin_ctzll(bal)) a.nonempty[d] = 1;
}

}  // namespace

hipError_t ym_launch_masks(const MaskArgs& a, hipStream_t st) {
  if (a.total <= 0) return hipSuccess;
  if (a.nm > 64 || a.nm % 4) return hipErrorInvalidValue;
  (void)hipMemsetAsync(a.nonempty, 0, (size_t)a.total * sizeof(int), st);
  hipLaunchKernelGGL(mask_lowres, dim3((a.MH * a.MW + 255) / 256, a.total), dim3(256), 0, st, a);
  hipLaunchKernelGGL(mask_upsample, dim3((a.H * a.W + 255) / 256, a.total), dim3(256), 0, st, a);
  return hipGetLastError();
}
