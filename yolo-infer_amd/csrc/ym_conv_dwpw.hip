// Depthwise 3x3 → 1x1 conv in one launch: the Detect head's classification chains (reference
// core/model.py → Ultralytics Detect.cv3[l] = Sequential(Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
// Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)), Conv2d(c3, nc, 1))).  yolomi/arch.py GraphBuilder.fuse_dw merges a
// depthwise op into the 1x1 conv that is the only reader of its output; the depthwise output never reaches HBM.
//
// A wave owns 16 consecutive output pixels and every output channel (N <= 128: 8 blocks of 16).  Per K block of 32
// logical channels, lane (g, col) computes the depthwise output of pixel col, channels 32 kb + 8 g .. + 7 — exactly its
// B operand of v_mfma_f32_16x16x32_f16 (k = 8 g .. 8 g + 7 of pixel col), so the depthwise result goes from VALU
// registers straight into the MFMAs: no LDS tile, no barrier inside the K loop.
//   * taps: 9 16-byte loads per lane (x3: 18, the hi and lo halves of the pair layout) through a buffer resource, an
//     out-of-image tap or a channel chunk past C at an out-of-range offset (the hardware returns zeros): no branch;
//   * depthwise arithmetic exactly as csrc/ym_misc.hip dwconv3x3*: acc = bias, then fmaf over taps 0..8 on the values
//     as stored (x3: hi + lo in fp32), SiLU (x3: ym_silu_x3, f16: ym_silu_fast), then x3: hi = fp16(v),
//     lo = fp16(v - hi) — the same B operands the unfused 1x1 reads back from the stored depthwise tensor;
//   * the 1x1: A = weight rows from global (L2-resident; x3 pair-chunk rows give w_hi and w_lo of the lane's chunk in
//     one 32-byte run), issued with the taps so their latency hides under the depthwise VALU work; x3 takes three MFMAs
//     per block (w_lo·x_hi + w_hi·x_lo + w_hi·x_hi), f16 one;
//   * KW > 1: the KW waves of a workgroup split the K blocks of one pixel group (the 20² / 40² maps have too few pixel
//     groups to fill the GPU), their partial sums meet in LDS in wave order (deterministic);
//   * epilogue as the other x3 convs: fmaf(acc, 2^-s, bias), SiLU, lane-pair whole-chunk stores (x3) / fp16x4.
// The depthwise weights ([9][C] fp32 then the bias [C]) are staged in LDS once per workgroup; lanes of one g read the
// same address (broadcast).
#include <type_traits>

#include "ym_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define YM_DWPW_CFGS(X) X(0, 1) X(1, 2) X(2, 4)
struct DwpwCfg {
  int kw;  // waves of a workgroup splitting the K blocks of one 16-pixel group (4 / kw pixel groups per workgroup)
};
constexpr DwpwCfg kDwpw[] = {
#define YM_X(id, kw) {kw},
    YM_DWPW_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumDwpw = sizeof(kDwpw) / sizeof(kDwpw[0]);
constexpr int kDwpwMaxC = 512;  // depthwise channels staged in LDS (10 x C fp32)
constexpr int kDwpwNB = 8;      // output-channel blocks of 16 per wave (N <= 128)
constexpr unsigned OOBX = 0x80000000u;

__device__ __forceinline__ h8 bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <typename T, int KW>
__global__ __launch_bounds__(256) void conv_dwpw(const ConvArgs a) {
  constexpr bool X3 = std::is_same<T, P2>::value;
  constexpr int XS = X3 ? 2 : 1;  // fp16 storage elements per logical channel
  constexpr int PXG = 4 / KW;     // 16-pixel groups per workgroup
  __shared__ __attribute__((aligned(16))) float wl[10 * kDwpwMaxC];  // depthwise taps [9][C], then bias [C]
  __shared__ __attribute__((aligned(16))) f32x4 red[KW > 1 ? (KW - 1) * PXG * kDwpwNB * 64 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int kw = __builtin_amdgcn_readfirstlane(wave % KW), pg = wave / KW;
  const int C = a.C0;
  for (int i = tid; i < 10 * C / 4; i += 256) {
    const int t = (4 * i) / C, c = 4 * i - t * C;
    *reinterpret_cast<f32x4*>(wl + 4 * i) =
        ym_gld<f32x4>(t < 9 ? a.dw_w + t * C + c : a.dw_b + c);
  }

  // this lane's pixel and its 3x3 window (bit t: tap t inside the image; none for a pixel past M)
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);
  const int m = (vb * PXG + pg) * 16 + col;
  const bool okm = m < a.M;
  const int mm = okm ? m : 0;
  const int b = ym_div(mm, a.fd_hw), rem = mm - b * (a.Ho * a.Wo);
  const int y = ym_div(rem, a.fd_w), x = rem - y * a.Wo;
  unsigned tmask = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = y - 1 + t / 3, ix = x - 1 + t % 3;
    tmask |= ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win) ? (1u << t) : 0u;
  }
  if (!okm) tmask = 0;
  // byte offset of the lane's window origin (pixel (y-1, x-1), channel 0) in the source; only in-image taps are used
  const int pix0 = (b * a.s0_P + (y - 1) * a.s0_W + (x - 1)) * a.s0_ctot + a.s0_coff;  // logical elements
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.src0), 0,
                                                                      (int)(a.s0_elems * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0,
                                                                      (int)((long)a.N * a.Kpad * 2), 0x00020000);
  const int NB = (a.N + 15) >> 4;
  const int nkb = (C + 31) >> 5;  // K blocks of 32 logical channels
  const int kb0 = nkb * kw / KW, kb1 = nkb * (kw + 1) / KW;

  f32x4 acc[kDwpwNB];
#pragma unroll
  for (int nb = 0; nb < kDwpwNB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // depthwise weights in LDS

  for (int kb = kb0; kb < kb1; ++kb) {
    const int c = 32 * kb + 8 * g;  // the lane's first logical channel
    const bool kc = c < C;
    // the 9 taps of the lane's chunk
    h8 th[9], tl[X3 ? 9 : 1];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const bool ok = kc && ((tmask >> t) & 1u);
      const unsigned off = (unsigned)(pix0 + ((t / 3) * a.s0_W + t % 3) * a.s0_ctot + c) * (2u * XS);
      th[t] = bld(rs, ok ? off : OOBX);
      if constexpr (X3) tl[t] = bld(rs, ok ? off + 16u : OOBX);
    }
    // depthwise: bias, taps 0..8 (csrc/ym_misc.hip dwconv3x3_lds order), SiLU
    const int cc = kc ? c : 0;
    float v[8];
    {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(wl + 9 * C + cc), b1 = *reinterpret_cast<const f32x4*>(wl + 9 * C + cc + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = b0[e]; v[4 + e] = b1[e]; }
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(wl + t * C + cc), w1 = *reinterpret_cast<const f32x4*>(wl + t * C + cc + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = X3 ? (float)th[t][e] + (float)tl[t][e] : (float)th[t][e];
        v[e] = fmaf(xv, e < 4 ? w0[e] : w1[e - 4], v[e]);
      }
    }
    h8 xh, xl;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = a.dw_act ? (X3 ? ym_silu_x3(v[e]) : ym_silu_fast(v[e])) : v[e];
      s = kc ? s : 0.f;  // channels past C: a zero operand (their weights are zero-padded too)
      xh[e] = (f16)s;
      if constexpr (X3) xl[e] = (f16)(s - (float)xh[e]);
    }
    // 1x1 weight fragments of the block: row 16 nb + col, the lane's 8 channels (x3: hi then lo, one 32-byte run)
    h8 wa[kDwpwNB], wb[X3 ? kDwpwNB : 1];
#pragma unroll
    for (int nb = 0; nb < kDwpwNB; ++nb) {
      const int n = 16 * nb + col;
      const bool ok = nb < NB && n < a.N;
      const unsigned off = (unsigned)(n * a.Kpad + XS * c) * 2u;
      wa[nb] = bld(rw, ok ? off : OOBX);
      if constexpr (X3) wb[nb] = bld(rw, ok ? off + 16u : OOBX);
    }
#pragma unroll
    for (int nb = 0; nb < kDwpwNB; ++nb) {
      if (nb >= NB) break;
      if constexpr (X3) {
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb[nb], xh, acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nb], xl, acc[nb], 0, 0, 0);
      }
      acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nb], xh, acc[nb], 0, 0, 0);
    }
  }

  if constexpr (KW > 1) {  // partial sums of waves kw > 0 → wave kw = 0 of the pixel group, added in wave order
    if (kw > 0) {
#pragma unroll
      for (int nb = 0; nb < kDwpwNB; ++nb)
        if (nb < NB) red[(((kw - 1) * PXG + pg) * kDwpwNB + nb) * 64 + lane] = acc[nb];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int q = 1; q < KW; ++q)
#pragma unroll
      for (int nb = 0; nb < kDwpwNB; ++nb)
        if (nb < NB) acc[nb] += red[(((q - 1) * PXG + pg) * kDwpwNB + nb) * 64 + lane];
  }

  // epilogue: lane (g, col) holds channels 16 nb + 4 g .. + 3 of pixel m
  const int ob = b * a.d_P + a.d_pixoff + y * a.d_W + x;
  T* dst = static_cast<T*>(a.dst);
  const bool pair = X3 && ((a.N | a.d_coff | a.d_ctot) & 7) == 0;
#pragma unroll
  for (int nb = 0; nb < kDwpwNB; ++nb) {
    if (nb >= NB) break;
    const int n0 = 16 * nb + 4 * g;
    const bool ok = okm && n0 < a.N;
    const f32x4 b4 = ym_gld<f32x4>(a.bias + (n0 < a.N ? n0 : 0));
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float xv = X3 ? ym_x3_pre(acc[nb][r], a.wsc, b4[r]) : acc[nb][r] + b4[r];
      o[r] = a.act ? (X3 ? ym_silu_x3(xv) : ym_silu_fast(xv)) : xv;
    }
    if constexpr (X3) {
      if (pair) {  // lanes (g, g ^ 1) of one pixel: one 32-byte chunk run
        ym_p2_store4_pair<16>(reinterpret_cast<P2*>(dst) + (size_t)(ok ? ob : 0) * a.d_ctot + a.d_coff + n0, o, g & 1,
                              ok, true);
        continue;
      }
      if (ok) ym_p2_store4(reinterpret_cast<P2*>(dst) + (size_t)ob * a.d_ctot + a.d_coff + n0, o);
    } else {
      if (ok)
        *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(dst) + (size_t)ob * a.d_ctot + a.d_coff + n0) =
            f16x4{(f16)o[0], (f16)o[1], (f16)o[2], (f16)o[3]};
    }
  }
}

template <typename T, int KW>
hipError_t launch(const ConvArgs& a, hipStream_t st) {
  const int groups = (a.M + 15) / 16, pxg = 4 / KW;
  hipLaunchKernelGGL((conv_dwpw<T, KW>), dim3((groups + pxg - 1) / pxg), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace

int ym_conv_dwpw_num_cfgs() { return kNumDwpw; }

// cfg: a configuration index (the tuner's id space for these ops; ym_launch_conv), or -1 / out of range: heuristic
// (strict: out of range is rejected)
hipError_t ym_launch_conv_dwpw(int dtype, int out_f32, const ConvArgs& a, int cfg, hipStream_t st, bool strict) {
  if (dtype != YM_DT_F16 && dtype != YM_DT_X3) return hipErrorInvalidValue;
  if (out_f32 || a.k != 1 || a.s != 1 || a.src1 || a.up0 || a.shuffle || a.res || a.w2 || a.nchw) return hipErrorInvalidValue;
  if (a.N > 16 * kDwpwNB || a.N % 4 || a.C0 % 8 || a.C0 > kDwpwMaxC || a.Hin != a.Ho || a.Win != a.Wo) return hipErrorInvalidValue;
  if (a.Kpad < (dtype == YM_DT_X3 ? 2 : 1) * ((a.C0 + 31) / 32) * 32) return hipErrorInvalidValue;  // whole K blocks
  // 32-bit offsets of the buffer loads
  if (a.s0_elems * 2 >= 0x7FFFFFF0L || (long)a.N * a.Kpad * 2 >= 0x7FFFFFF0L) return hipErrorInvalidValue;
  if (cfg < 0 || cfg >= kNumDwpw) {
    if (strict) return hipErrorInvalidValue;
    // enough waves for the GPU (~2k), each K range at least two blocks
    const int groups = (a.M + 15) / 16, nkb = (a.C0 + 31) / 32;
    cfg = 0;
    while (cfg + 1 < kNumDwpw && groups * kDwpw[cfg].kw < 2048 && nkb >= 2 * kDwpw[cfg + 1].kw) ++cfg;
  }
  const int kw = kDwpw[cfg].kw;
  if (dtype == YM_DT_X3) {
    switch (kw) {
      case 1: return launch<P2, 1>(a, st);
      case 2: return launch<P2, 2>(a, st);
      default: return launch<P2, 4>(a, st);
    }
  }
  switch (kw) {
    case 1: return launch<f16, 1>(a, st);
    case 2: return launch<f16, 2>(a, st);
    default: return launch<f16, 4>(a, st);
  }
}
