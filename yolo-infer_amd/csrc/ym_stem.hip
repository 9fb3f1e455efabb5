// Stem conv: Conv(3, C, 3, 2) + SiLU on the caller's NCHW fp32 batch.  LoadTensor's /255 rule
// (ultralytics/data/loaders.py LoadTensor) and the NCHW → NHWC change of layout are folded into its
// loader, so the input is read exactly once.
//
// A workgroup computes a TH-row x 32-column output tile (TH = 16 on the MFMA path, 8 on the VALU path).  The
// (2 TH + 1) x 68 x 3 input patch is staged in LDS with coalesced float4 row loads, all in flight at once (the rows
// start 4 floats left of the window: 16-byte aligned, W % 4 == 0).
//
// f16 / int8 plans — stem_mfma: the 27-tap contraction (K = 27, padded to 32) is ONE v_mfma_f32_16x16x32_f16 per
// 16 pixels x 16 channels, in the transposed orientation of csrc/ym_conv.hip (A = weights, so a lane owns 4
// consecutive output channels of one pixel: 8-byte NHWC stores).  The patch is kept in fp16: the activation storage
// precision of the f16 plan, and for int8 plans the exact integers q - z_in (|v| <= 255) — int8 weights are exact in
// fp16 as well, products are exact in fp32 and the 27-term sums stay below 2^24, so the int8 accumulator is exact.
// Each lane gathers its 8 K values of one pixel from the LDS patch through per-lane tap offsets.
// int8 plans quantize the image on load (q = clamp(rint(x / s_in) + z_in), patch = q - z_in, padding 0), then run the
// quantized-conv epilogue (csrc/ym_conv_i8.hip; numerics oracle/quant.py).
//
// f32 parity plan — stem_valu: one thread per output pixel, fp32 FMAs, weights read with wave-uniform addresses;
// optionally the pre-activation output for the calibration runs.
#include <type_traits>

#include "ym_common.h"
#include "ym_quant.h"

namespace {

constexpr int TW = 32;
constexpr int PW4 = (2 * TW + 4) / 4 + 1;  // 4-wide groups per patch row: columns x0-4 .. x0+2TW+3
constexpr int PW = PW4 * 4;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <int TH>
__device__ __forceinline__ void tile_of(const ConvArgs& a, int& b, int& oy0, int& ox0) {
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  int bid = ym_xcd_block(blockIdx.x, gridDim.x);  // neighbouring tiles (shared halo lines) on one XCD
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  b = bid / tiles_y;
  oy0 = ty * TH;
  ox0 = tx * TW;
}

// ------------------------------------------------------------------------------------------------ MFMA (f16, i8)
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int MTH = 16;  // MFMA path: 16 output rows per workgroup (32 groups of 16 pixels, 8 per wave)

// NT = Cout / 16 channel tiles; F8 (T = i8 storage): the fp8 e4m3 PTQ plan (csrc/ym_quant.h); T = P2: the x3 plan —
// the patch and the weights are split into fp16 hi / lo parts and every tile takes the three MFMAs of the split
// product (w_lo·x_hi + w_hi·x_lo + w_hi·x_hi), the output is stored in the pair layout with the exact SiLU
template <typename T, int NT, bool F8 = false>
__global__ __launch_bounds__(256) void stem_mfma(const ConvArgs a) {
  ym_warm_kernargs<sizeof(ConvArgs)>();  // one round trip for the whole argument block (ym_common.h)
  constexpr bool QUANT = sizeof(T) == 1;
  constexpr bool X3 = std::is_same<T, P2>::value;
  constexpr int TH = MTH, PH = 2 * TH + 1;
  __shared__ __attribute__((aligned(16))) f16 patch[3 * PH * PW];
  __shared__ __attribute__((aligned(16))) f16 patch_lo[X3 ? 3 * PH * PW : 8];
  __shared__ float post[QUANT ? 256 : 1];
  int b, oy0, ox0;
  tile_of<TH>(a, b, oy0, ox0);
  const int iy0 = 2 * oy0 - 1, xs = 2 * ox0 - 4;
  const bool div = ym_input_max(a.ctl) > 1.0f + a.eps;
  const size_t HW = (size_t)a.Hin * a.Win;
  const float* img = a.nchw + (size_t)b * 3 * HW;
  const QRec* Q = a.q;
  float inv = 0.f;
  int zi = 0, lo = 0, hi = 0;
  if constexpr (QUANT) {
    inv = Q->inv_s_in;
    zi = Q->z_in;
    lo = Q->qlo;
    hi = Q->qhi;
    post[threadIdx.x] = Q->post[threadIdx.x];
  }
  // Per-lane K slots: lane l covers K = 8(l>>4) .. +7 of pixel column l&15; K = tap (ky*3 + kx)*3 + c (the wstem row
  // order), K >= 27 zero weights (their patch reads point at a valid element).  The weight / bias loads are
  // unconditional (clamped rows) and issued before the patch loads, so their latency hides behind the staging.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kg = lane >> 4, col = lane & 15;
  int off[8];
  float wraw[NT][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    const int kk = k / 3, c = k - (k / 3) * 3;
    const int ky = kk / 3, kx = kk - (kk / 3) * 3;
    off[j] = k < 27 ? (c * PH + ky) * PW + kx + 3 : 3;  // +3: the patch starts at x0 - 4, the window at x0 - 1
    const int kr = k < 27 ? k : 26;
#pragma unroll
    for (int t = 0; t < NT; ++t) wraw[t][j] = a.wstem[kr * a.N + 16 * t + col];
  }
  float bias[NT][4], sasw[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bias[t][r] = a.bias[16 * t + 4 * kg + r];
      if constexpr (QUANT) sasw[t][r] = a.sasw[16 * t + 4 * kg + r];
    }
  // all of a thread's patch loads are issued before the first is consumed (one memory latency, not NIT)
  constexpr int NIT = (3 * PH * PW4 + 255) / 256;
  f32x4 v[NIT];
  bool in[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = threadIdx.x + 256 * it;
    const int c = i / (PH * PW4), r = i - c * (PH * PW4);
    const int py = r / PW4, q = r - (r / PW4) * PW4;
    const int iy = iy0 + py, ix = xs + 4 * q;
    in[it] = i < 3 * PH * PW4 && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
    v[it] = in[it] ? *reinterpret_cast<const f32x4*>(img + c * HW + (size_t)iy * a.Win + ix) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = threadIdx.x + 256 * it;
    if (i >= 3 * PH * PW4) break;
    f16x4 h = {0, 0, 0, 0}, hl = {0, 0, 0, 0};
    if (in[it]) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[it][e];
        if (div) x = x / 255.0f;
        if constexpr (F8) h[e] = (f16)f8_dec(f8_enc(x, inv));  // e4m3 values are exact in f16
        else if constexpr (QUANT) h[e] = (f16)(float)(clampi((int)rintf(__fmul_rn(x, inv)) + zi, lo, hi) - zi);
        else h[e] = (f16)x;  // the activation storage precision, as the NHWC input of the MFMA path
        if constexpr (X3) hl[e] = (f16)(x - (float)h[e]);
      }
    }
    *reinterpret_cast<f16x4*>(patch + 4 * i) = h;  // i = (c*PH + py)*PW4 + q
    if constexpr (X3) *reinterpret_cast<f16x4*>(patch_lo + 4 * i) = hl;
  }
  h8 wf[NT], wfl[X3 ? NT : 1];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      wf[t][j] = 8 * kg + j < 27 ? (f16)wraw[t][j] : (f16)0.f;
      if constexpr (X3) wfl[t][j] = 8 * kg + j < 27 ? (f16)(wraw[t][j] - (float)wf[t][j]) : (f16)0.f;
    }
  __syncthreads();
  // wave w: pixel groups 8w .. 8w+7 of the tile's 32 (16 consecutive columns of one row each)
#pragma unroll
  for (int gi = 0; gi < 8; ++gi) {
    const int g = 8 * wave + gi;
    const int ly = g >> 1, lx = (g & 1) * 16 + col;
    const f16* pp = patch + 2 * ly * PW + 2 * lx;
    h8 bf, bfl;
#pragma unroll
    for (int j = 0; j < 8; ++j) bf[j] = pp[off[j]];
    if constexpr (X3) {
      const f16* pl = patch_lo + 2 * ly * PW + 2 * lx;
#pragma unroll
      for (int j = 0; j < 8; ++j) bfl[j] = pl[off[j]];
    }
    const int oy = oy0 + ly, ox = ox0 + lx;
    const bool ok = oy < a.Ho && ox < a.Wo;
    T* dst = static_cast<T*>(a.dst) + (size_t)(b * a.d_P + oy * a.d_W + ox) * a.d_ctot + a.d_coff + 4 * kg;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (X3) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wfl[t], bf, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[t], bfl, acc, 0, 0, 0);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[t], bf, acc, 0, 0, 0);
      if constexpr (X3) {
        if ((a.pst & 4) && ((a.d_coff | a.d_ctot) & 7) == 0) {  // lanes (kg, kg ^ 1) of a pixel write whole 32-byte chunks
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = ym_silu_x3(acc[r] + bias[t][r]);
          ym_p2_store4_pair<16>(ok ? dst + 16 * t : static_cast<T*>(a.dst), o, kg & 1, ok, a.pst & 16);
          continue;
        }
      }
      if (!ok) continue;
      if constexpr (X3) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = ym_silu_x3(acc[r] + bias[t][r]);
        ym_p2_store4(dst + 16 * t, o);
      } else if constexpr (QUANT) {
        int ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = ym_opaque(acc[r] * sasw[t][r]) + bias[t][r];  // two roundings, as the oracle's mul + add
          if constexpr (F8) {
            ov[r] = f8_enc(post[f8_enc(y, Q->inv_sc)], Q->inv_so);
          } else {
            const int qc = clampi((int)rintf(__fmul_rn(y, Q->inv_sc)) + Q->zc, lo, hi);
            ov[r] = clampi((int)rintf(__fmul_rn(post[qc], Q->inv_so)) + Q->zo, lo, hi) - 128;
          }
        }
        *reinterpret_cast<int*>(dst + 16 * t) =
            (ov[0] & 0xFF) | ((ov[1] & 0xFF) << 8) | ((ov[2] & 0xFF) << 16) | ((unsigned)(ov[3] & 0xFF) << 24);
      } else {
        f16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (f16)ym_silu_fast(acc[r] + bias[t][r]);
        *reinterpret_cast<f16x4*>(dst + 16 * t) = o;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ VALU (f32 parity)
__global__ __launch_bounds__(256) void stem_valu(const ConvArgs a) {
  constexpr int TH = 8, PH = 2 * TH + 1;  // one thread per output pixel: 8 x 32
  __shared__ __attribute__((aligned(16))) float patch[3 * PH * PW];
  int b, oy0, ox0;
  tile_of<TH>(a, b, oy0, ox0);
  const int iy0 = 2 * oy0 - 1, xs = 2 * ox0 - 4;
  const bool div = ym_input_max(a.ctl) > 1.0f + a.eps;
  const size_t HW = (size_t)a.Hin * a.Win;
  const float* img = a.nchw + (size_t)b * 3 * HW;
  for (int i = threadIdx.x; i < 3 * PH * PW4; i += 256) {
    const int c = i / (PH * PW4), r = i - c * (PH * PW4);
    const int py = r / PW4, q = r - (r / PW4) * PW4;
    const int iy = iy0 + py, ix = xs + 4 * q;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win) {
      v = *reinterpret_cast<const f32x4*>(img + c * HW + (size_t)iy * a.Win + ix);
      if (div) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] / 255.0f;
      }
    }
    *reinterpret_cast<f32x4*>(patch + (c * PH + py) * PW + 4 * q) = v;
  }
  __syncthreads();
  const int t = threadIdx.x;
  const int ly = t / TW, lx = t - (t / TW) * TW;
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
  const size_t pix = (size_t)(b * a.Ho + oy) * a.Wo + ox;
  const float* __restrict__ Wt = a.wstem;  // [27][N] fp32, wave-uniform addresses
  for (int g = 0; g < a.N; g += 16) {
    float acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = a.bias[g + e];
#pragma unroll
    for (int k = 0; k < 27; ++k)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = fmaf(x[k], Wt[k * a.N + g + e], acc[e]);
    float* dst = static_cast<float*>(a.dst) + (size_t)(b * a.d_P + oy * a.d_W + ox) * a.d_ctot + a.d_coff + g;
    f32x8 o0, o1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o0[e] = ym_silu(acc[e]);
      o1[e] = ym_silu(acc[8 + e]);
    }
    Vec8<float>::store(dst, o0);
    Vec8<float>::store(dst + 8, o1);
    if (a.raw) {  // f32 calibration run: the pre-activation output, (M, N) row-major
#pragma unroll
      for (int e = 0; e < 16; ++e) a.raw[pix * a.N + g + e] = acc[e];
    }
  }
}

dim3 grid_of(const ConvArgs& a, int TH) {
  const int B = a.M / (a.Ho * a.Wo);
  return dim3(B * ((a.Ho + TH - 1) / TH) * ((a.Wo + TW - 1) / TW));
}

template <typename T, bool F8 = false>
hipError_t launch_mfma(const ConvArgs& a, hipStream_t st) {
  switch (a.N / 16) {
    case 1: hipLaunchKernelGGL((stem_mfma<T, 1, F8>), grid_of(a, MTH), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((stem_mfma<T, 2, F8>), grid_of(a, MTH), dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((stem_mfma<T, 4, F8>), grid_of(a, MTH), dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL((stem_mfma<T, 6, F8>), grid_of(a, MTH), dim3(256), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t ym_launch_stem(int dtype, const ConvArgs& a, hipStream_t st) {
  if (a.k != 3 || a.s != 2 || !a.nchw || a.shuffle || a.res || !a.act || a.Win % 4 || !a.wstem || a.N % 16 ||
      a.M % (a.Ho * a.Wo))
    return hipErrorInvalidValue;
  if (dtype == YM_DT_I8) return a.q && a.sasw ? launch_mfma<i8>(a, st) : hipErrorInvalidValue;
  if (dtype == YM_DT_F8) return a.q && a.sasw ? launch_mfma<i8, true>(a, st) : hipErrorInvalidValue;
  if (dtype == YM_DT_F16) return a.raw ? hipErrorInvalidValue : launch_mfma<f16>(a, st);
  if (dtype == YM_DT_X3) return a.raw ? hipErrorInvalidValue : launch_mfma<P2>(a, st);
  hipLaunchKernelGGL(stem_valu, grid_of(a, 8), dim3(256), 0, st, a);
  return hipGetLastError();
}
