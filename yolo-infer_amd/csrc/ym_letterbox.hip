// Image-source preprocessing: Ultralytics `LetterBox` + `BasePredictor.preprocess` for one
// HWC uint8 image already on the device — OpenCV's 8-bit INTER_LINEAR resize (11-bit fixed-point weights, scalar
// path: horizontal sums, then (S0·b0 + S1·b1 + 2^21) >> 22), the 114 border, BGR→RGB, HWC→CHW and /255, written
// straight into one image slot of the fp32 NCHW batch that ym_infer reads.  Restatement and its caveats:
// oracle/letterbox.py (bit-exact against it; parity with cv2 itself is unpinned).
// One thread per output pixel; the source (a few MB) is read through L2 with 3-byte gathers — HBM-bound at the
// output write (12 B per pixel), far below the network's cost.
#include "ym_common.h"

namespace {

__device__ __forceinline__ double opaque_d(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

// source index pair and 11-bit weights of destination index d (oracle/letterbox.py _axis)
__device__ __forceinline__ void axis(int d, int src, double scale, int& s0, int& s1, int& a0, int& a1, bool& edge) {
  float f = (float)(opaque_d((d + 0.5) * scale) - 0.5);  // (double) (d + .5)·scale − .5 in two roundings, to float
  int s = (int)floorf(f);
  f -= (float)s;
  edge = false;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= src - 1) { f = 0.f; s = src - 1; edge = true; }
  a0 = (int)rintf((1.f - f) * 2048.f);
  a1 = (int)rintf(f * 2048.f);
  s0 = s;
  s1 = s + 1 < src ? s + 1 : src - 1;
}

__global__ __launch_bounds__(256) void letterbox_u8(const LetterboxArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.Hn * a.Wn) return;
  const int y = i / a.Wn, x = i - (i / a.Wn) * a.Wn;
  const size_t plane = (size_t)a.Hn * a.Wn;
  float* out = a.dst + i;
  const int dy = y - a.top, dx = x - a.left;
  if ((unsigned)dy >= (unsigned)a.uh || (unsigned)dx >= (unsigned)a.uw) {
    const float pad = 114.f / 255.f;
    out[0] = pad; out[plane] = pad; out[2 * plane] = pad;
    return;
  }
  int v[3];
  if (a.uh == a.h && a.uw == a.w) {
    const unsigned char* p = a.src + (size_t)dy * a.row_bytes + (size_t)dx * 3;
    v[0] = p[0]; v[1] = p[1]; v[2] = p[2];
  } else {
    int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
    bool xedge, yedge;
    axis(dx, a.w, a.scale_x, sx0, sx1, a0, a1, xedge);
    axis(dy, a.h, a.scale_y, sy0, sy1, b0, b1, yedge);
    const unsigned char* r0 = a.src + (size_t)sy0 * a.row_bytes;
    const unsigned char* r1 = a.src + (size_t)sy1 * a.row_bytes;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int s0 = xedge ? r0[sx0 * 3 + c] * 2048 : r0[sx0 * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
      const int s1 = xedge ? r1[sx0 * 3 + c] * 2048 : r1[sx0 * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
      const int t = (s0 * b0 + s1 * b1 + (1 << 21)) >> 22;
      v[c] = t < 0 ? 0 : (t > 255 ? 255 : t);
    }
  }
  // RGB planes: BGR sources (cv2.imread order) are flipped, as upstream's im[..., ::-1]
#pragma unroll
  for (int c = 0; c < 3; ++c) out[c * plane] = (float)v[a.bgr ? 2 - c : c] / 255.f;
}

}  // namespace

hipError_t ym_launch_letterbox(const LetterboxArgs& a, hipStream_t st) {
  if (!a.src || !a.dst || a.h < 1 || a.w < 1 || a.uh < 1 || a.uw < 1 || a.top < 0 || a.left < 0 ||
      a.top + a.uh > a.Hn || a.left + a.uw > a.Wn || a.row_bytes < 3 * a.w)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(letterbox_u8, dim3((a.Hn * a.Wn + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}
