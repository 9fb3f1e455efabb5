// Stem conv of YOLO11 (layer 0: Conv(3, c, 3, 2) = conv2d → folded BN → SiLU) straight from the caller's NCHW fp32
// batch — the `LoadTensor` /255 rule (/root/reference/core/model.py:133 → ultralytics LoadTensor._single_check) and
// the NCHW → NHWC change of layout are folded into its loader, so the input is read exactly once.
//
// It is HBM-bound (27 MACs per output channel): a direct VALU kernel, not MFMA.  A workgroup computes an 8-row x
// TW-column output tile; the 17 x (2*TW+1) x 3 input patch is staged in LDS with coalesced row loads, the
// [27][Cout] weights are broadcast from LDS, and each thread writes 16 channels of one pixel as 16-byte vectors.
#include "ym_common.h"

namespace {

constexpr int TH = 8;

// G = Cout/16 channel groups per pixel, TW = 32/G output columns per tile.  The patch starts 4 floats left of the
// window (16-byte aligned, W % 32 == 0) and is loaded as float4 rows: [3][17][PW4*4].
template <typename T, int G>
__global__ __launch_bounds__(256) void stem_conv3x3s2(const ConvArgs a) {
  constexpr int TW = 32 / G;
  constexpr int PH = 2 * TH + 1;
  constexpr int PW4 = (2 * TW + 4 + 3) / 4 + 1;  // float4s per patch row (covers x0-4 .. x0+2TW)
  constexpr int PW = PW4 * 4;
  constexpr int N = 16 * G;
  extern __shared__ float sm[];
  float* patch = sm;                   // [3][PH][PW]
  float* wl = patch + 3 * PH * PW;     // [27][N]
  float* bl = wl + 27 * N;             // [N]
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = 2 * oy0 - 1, xs = 2 * ox0 - 4;  // patch column 0 = input column xs (xs % 4 == 0)
  const bool div = ym_input_max(a.ctl) > 1.0f + a.eps;
  const size_t HW = (size_t)a.Hin * a.Win;
  const float* img = a.nchw + (size_t)b * 3 * HW;
  for (int i = threadIdx.x; i < 3 * PH * PW4; i += 256) {
    const int c = i / (PH * PW4), r = i - c * (PH * PW4);
    const int py = r / PW4, q = r - (r / PW4) * PW4;
    const int iy = iy0 + py, ix = xs + 4 * q;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win)
      v = *reinterpret_cast<const f32x4*>(img + c * HW + (size_t)iy * a.Win + ix);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (div) x = x / 255.0f;
      v[e] = (float)(T)x;  // the activation storage precision, as the NHWC input of the MFMA path
    }
    *reinterpret_cast<f32x4*>(patch + (c * PH + py) * PW + 4 * q) = v;
  }
  const T* W = static_cast<const T*>(a.w);
  for (int i = threadIdx.x; i < 27 * N; i += 256) {
    const int tap = i / N, n = i - (i / N) * N;  // tap = (ky*3 + kx)*3 + c
    const int kk = tap / 3, c = tap - (tap / 3) * 3;
    wl[i] = (float)W[(size_t)n * a.Kpad + kk * 8 + c];
  }
  for (int i = threadIdx.x; i < N; i += 256) bl[i] = a.bias[i];
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= TH * TW * G) return;
  const int g = t % G, pix = t / G;
  const int ly = pix / TW, lx = pix - (pix / TW) * TW;
  const int oy = oy0 + ly, ox = ox0 + lx;
  if (oy >= a.Ho || ox >= a.Wo) return;
  float x[27];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        x[(ky * 3 + kx) * 3 + c] = patch[(c * PH + 2 * ly + ky) * PW + 2 * lx + kx + 3];  // +3: xs = x0 - 4
  const int n0 = g * 16;
  float acc[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = bl[n0 + e];
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    const float* wr = wl + k * N + n0;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = fmaf(x[k], wr[e], acc[e]);
  }
  typename Vec8<T>::type o0, o1;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o0[e] = (T)ym_silu(acc[e]);
    o1[e] = (T)ym_silu(acc[8 + e]);
  }
  T* dst = static_cast<T*>(a.dst) + (size_t)(b * a.d_P + oy * a.d_W + ox) * a.d_ctot + a.d_coff + n0;
  Vec8<T>::store(dst, o0);
  Vec8<T>::store(dst + 8, o1);
  if (a.raw) {  // f32 calibration run: the pre-activation output, (M, N) row-major
    float* r = a.raw + ((size_t)(b * a.Ho + oy) * a.Wo + ox) * N + n0;
#pragma unroll
    for (int e = 0; e < 16; ++e) r[e] = acc[e];
  }
}

}  // namespace

template <typename T, int G>
hipError_t launch_g(const ConvArgs& a, hipStream_t st) {
  constexpr int TW = 32 / G;
  constexpr int PW = ((2 * TW + 4 + 3) / 4 + 1) * 4;
  const int B = a.M / (a.Ho * a.Wo);
  const dim3 grid(B * ((a.Ho + TH - 1) / TH) * ((a.Wo + TW - 1) / TW));
  const size_t lds = ((size_t)3 * (2 * TH + 1) * PW + 28 * 16 * G) * sizeof(float);
  hipLaunchKernelGGL((stem_conv3x3s2<T, G>), grid, dim3(256), lds, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_t(const ConvArgs& a, hipStream_t st) {
  switch (a.N) {
    case 16: return launch_g<T, 1>(a, st);
    case 32: return launch_g<T, 2>(a, st);
    case 64: return launch_g<T, 4>(a, st);
    case 96: return launch_g<T, 6>(a, st);
  }
  return hipErrorInvalidValue;
}

hipError_t ym_launch_stem(int dtype, const ConvArgs& a, hipStream_t st) {
  if (dtype == YM_DT_I8) return ym_launch_stem_i8(a, st);
  if (a.k != 3 || a.s != 2 || !a.nchw || a.shuffle || a.res || !a.act || a.Win % 4) return hipErrorInvalidValue;
  return dtype == YM_DT_F16 ? launch_t<f16>(a, st) : launch_t<float>(a, st);
}
