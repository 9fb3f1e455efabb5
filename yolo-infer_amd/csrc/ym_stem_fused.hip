// The stem and the first downsampling pair of the x3 plan in ONE launch: Conv(3, 32, 3, 2) on the caller's NCHW fp32
// image (LoadTensor's /255 rule folded in) -> model.1 Conv(32, 64, 3, 2) -> model.2.cv1 Conv(64, 64, 1) (yolo11s;
// reference core/model.py:133 -> the Ultralytics module tree; verdict r5 item 5: the large-map
// traffic).  Unfused, the stem writes its 320x320x32 output (105 MB of pair-layout activations at B = 8) and the
// model.1+cv1 pair reads it back: ~210 MB of the forward's conv traffic for a tensor nobody else reads.  Here a
// workgroup owns RB x TW = 2 x 32 output pixels of the 160x160 maps and
//   A  stages the image patch its stem pixels read (4 RB + 3 rows x 4 TW + 4 columns x 3 channels, coalesced float4
//      loads, all in flight at once), /255 when the batch max says so, split hi / lo into two fp16 LDS planes;
//   B  computes the (2 RB + 1) x (2 TW + 1) stem pixels model.1's 3x3 s2 window needs — exactly stem_mfma's arithmetic
//      (csrc/ym_stem.hip: one v_mfma_f32_16x16x32_f16 triple per 16 pixels x 16 channels, K = 27 taps in the wstem
//      order, bias, ym_silu_x3), so they equal the stored stem tensor bit for bit — split hi / lo into the LDS stem
//      image (zero outside the stem map: model.1's padding), even columns first, then the odd ones, so the taps of
//      consecutive output columns read consecutive pixel slots, chunks XOR-swizzled by pixel (conflict-free b128 reads);
//   C  model.1: each wave a 32-pixel x 32-channel block, K = 9 taps x 32 channels in 18 steps of two 8-channel
//      chunks, three v_mfma_f32_32x32x16_f16 per step on split operands (w_hi·x_hi, w_hi·x_lo, w_lo·x_hi), weights
//      from L2 (pair-chunk rows, as every x3 GEMM), the stem image from LDS;
//   D  its epilogue (x3 weight scale + bias, SiLU) split hi / lo into an LDS tile — the pair's intermediate, never
//      stored;
//   E  model.2.cv1 (1x1, K = 64) from that tile, three MFMAs per step, and the pair-layout store of its output.
// The stem recomputes 325 / 256 of its pixels and the patch re-reads 1.36x of the image (tile halos); both are cheap
// against the round trip they remove.  Summation orders inside model.1 / cv1 differ from the split launches (fp32
// rounding level; the x3 plan's bar is against float64, tests/test_gpu_kernels.py).
#include <stdlib.h>

#include "ym_common.h"

namespace {

constexpr int RB = 2, TW = 32;                       // output tile: RB rows x TW columns (64 pixels)
constexpr int XR = 2 * RB + 1, XC = 2 * TW + 1;      // stem pixels of a tile: 5 x 65
constexpr int XE = TW + 1;                           // even stem columns (33) first, then the odd ones (32)
constexpr int NPX = XR * XC;                         // 325
constexpr int PR = 4 * RB + 3, PC = 4 * TW + 4;      // image patch: 11 rows x 132 columns (16-byte aligned start)
constexpr int PC4 = PC / 4;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct StemFuseArgs {
  ConvArgs s;  // the stem (nchw input)
  ConvArgs p;  // the model.1 -> cv1 pair (w2, k2 = 1)
  int dbg;     // phase ablations for timing only (YM_STEMFUSE_DBG): 1 no patch loads, 2 no stem MFMAs, 4 no model.1
               // MFMAs, 8 no cv1 MFMAs, 16 no stores
};

// split-column slot of stem-image column xc
__device__ __forceinline__ int xslot(int xr, int xc) { return xr * XC + ((xc & 1) ? XE + (xc >> 1) : (xc >> 1)); }

template <int C0, int N1, int N2>
__global__ __launch_bounds__(256) void stem_down_x3(const StemFuseArgs A) {
  static_assert(C0 == 32 && N1 == 64 && N2 == 64, "the yolo11s geometry (32 -> 64 -> 64)");
  constexpr int NT0 = C0 / 16;        // stem channel tiles of 16
  constexpr int XCH = C0 / 8;         // 8-channel chunks per stem pixel
  constexpr int XPB = C0 * 2;         // stem image bytes per pixel and plane
  constexpr int XPL = NPX * XPB;      // stem image plane (20,800 B)
  constexpr int PPL = 3 * PR * PC * 2;  // patch plane (8,712 B)
  constexpr int TPB = N1 * 2;         // model.1 tile bytes per pixel and plane
  constexpr int TPL = RB * TW * TPB;  // 8 KB
  constexpr int UB = 2 * PPL > 2 * TPL ? 2 * PPL : 2 * TPL;
  __shared__ __attribute__((aligned(16))) char lds[2 * XPL + UB];
  char* X = lds;            // stem image: hi plane, then lo plane
  char* U = lds + 2 * XPL;  // the image patch (hi, lo), then the model.1 tile (hi, lo)
  ym_warm_kernargs<sizeof(StemFuseArgs)>();
  const ConvArgs& s = A.s;
  const ConvArgs& p = A.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_x = p.Wo / TW, tiles_y = p.Ho / RB;
  int bid = ym_xcd_block(blockIdx.x, gridDim.x);  // neighbouring tiles (shared patch rows) on one XCD
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * RB, ox0 = tx * TW;

  // ---- A: the image patch, all loads in flight before the first LDS store
  const bool div = ym_input_max(s.ctl) > 1.0f + s.eps;
  const size_t HW = (size_t)s.Hin * s.Win;
  const float* img = s.nchw + (size_t)b * 3 * HW;
  const int iy0 = 4 * oy0 - 3, ix0 = 4 * ox0 - 4;
  constexpr int NIT = (3 * PR * PC4 + 255) / 256;
  f32x4 v[NIT];
  bool in[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + 256 * it;
    const int c = i / (PR * PC4), r = i - c * (PR * PC4);
    const int py = r / PC4, q = r - py * PC4;
    const int iy = iy0 + py, ix = ix0 + 4 * q;
    in[it] = i < 3 * PR * PC4 && (unsigned)iy < (unsigned)s.Hin && (unsigned)ix < (unsigned)s.Win && !(A.dbg & 1);
    v[it] = in[it] ? *reinterpret_cast<const f32x4*>(img + c * HW + (size_t)iy * s.Win + ix) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // stem weights (A = weights: lane row = channel col of a 16-channel tile, K = 8 kg .. 8 kg + 7) and biases, as
  // stem_mfma: K = tap (ky*3 + kx)*3 + c, K >= 27 zero
  const int kg = lane >> 4, col = lane & 15;
  int off[8];
  float wraw[NT0][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    const int kk = k / 3, c = k - (k / 3) * 3;
    const int ky = kk / 3, kx = kk - (kk / 3) * 3;
    off[j] = k < 27 ? (c * PR + ky) * PC + kx + 1 : 1;  // +1: the patch starts one column left of the stem window
    const int kr = k < 27 ? k : 26;
#pragma unroll
    for (int t = 0; t < NT0; ++t) wraw[t][j] = s.wstem[kr * s.N + 16 * t + col];
  }
  float sbias[NT0][4];
#pragma unroll
  for (int t = 0; t < NT0; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) sbias[t][r] = s.bias[16 * t + 4 * kg + r];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + 256 * it;
    if (i >= 3 * PR * PC4) break;
    f16x4 hh = {0, 0, 0, 0}, hl = {0, 0, 0, 0};
    if (in[it]) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[it][e];
        if (div) x = x / 255.0f;
        hh[e] = (f16)x;
        hl[e] = (f16)(x - (float)hh[e]);
      }
    }
    *reinterpret_cast<f16x4*>(U + 8 * i) = hh;  // element 4i = (c*PR + py)*PC + 4q
    *reinterpret_cast<f16x4*>(U + PPL + 8 * i) = hl;
  }
  h8 wf[NT0], wfl[NT0];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < NT0; ++t) {
      wf[t][j] = 8 * kg + j < 27 ? (f16)wraw[t][j] : (f16)0.f;
      wfl[t][j] = 8 * kg + j < 27 ? (f16)(wraw[t][j] - (float)wf[t][j]) : (f16)0.f;
    }
  // model.1 / cv1 epilogue operands and weight fragments early (their latency hides behind phases A and B): all of
  // cv1's (4 steps) and model.1's first WPF steps, then a ring WPF steps ahead inside the K loop
  const int l32 = lane & 31, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;  // this wave's block: output row wm (32 pixels), channels 32 wn .. + 31
  const f16* W1 = static_cast<const f16*>(p.w) + (size_t)(32 * wn + l32) * p.Kpad;    // this lane's weight rows
  const f16* W2 = static_cast<const f16*>(p.w2) + (size_t)(32 * wn + l32) * p.Kpad2;
  constexpr int KST1 = 9 * XCH / 2, KST2 = N1 / 16, WPF = 6;
  h8 w1h[WPF], w1l[WPF], w2h[KST2], w2l[KST2];
#pragma unroll
  for (int t = 0; t < WPF; ++t) {
    w1h[t] = ym_gld<h8>(W1 + 16 * (2 * t + h));
    w1l[t] = ym_gld<h8>(W1 + 16 * (2 * t + h) + 8);
  }
#pragma unroll
  for (int t = 0; t < (A.dbg & 8 ? 0 : KST2); ++t) {
    w2h[t] = ym_gld<h8>(W2 + 16 * (2 * t + h));
    w2l[t] = ym_gld<h8>(W2 + 16 * (2 * t + h) + 8);
  }
  f32x4 b1[4], b2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    b1[q] = *reinterpret_cast<const f32x4*>(p.bias + 32 * wn + 8 * q + 4 * h);
    b2[q] = *reinterpret_cast<const f32x4*>(p.bias2 + 32 * wn + 8 * q + 4 * h);
  }
  __syncthreads();

  // ---- B: the stem pixels of the tile (16 per group, row-major over 5 x 65) -> the LDS stem image
  const f16* ph = reinterpret_cast<const f16*>(U);
  const f16* pl = reinterpret_cast<const f16*>(U + PPL);
  for (int g = wave; g < (NPX + 15) / 16; g += 4) {
    const int q = 16 * g + col;
    const bool qv = q < NPX;
    const int r = qv ? q / XC : 0, c = qv ? q - (q / XC) * XC : 0;
    const int sy = 2 * oy0 - 1 + r, sx = 2 * ox0 - 1 + c;
    const bool inmap = qv && sy >= 0 && sy < s.Ho && sx >= 0 && sx < s.Wo;
    const int base = 2 * r * PC + 2 * c;
    h8 bf, bfl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf[j] = ph[base + off[j]];
      bfl[j] = pl[base + off[j]];
    }
    const int xp = xslot(r, c);
#pragma unroll
    for (int t = 0; t < NT0; ++t) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!(A.dbg & 2)) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wfl[t], bf, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[t], bfl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[t], bf, acc, 0, 0, 0);
      }
      f16x4 oh, ol;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float o = inmap ? ym_silu_x3(acc[e] + sbias[t][e]) : 0.f;
        oh[e] = (f16)o;
        ol[e] = (f16)(o - (float)oh[e]);
      }
      const int chn = 16 * t + 4 * kg;  // channels chn .. chn + 3 of stem pixel xp
      const int byte = xp * XPB + (((chn >> 3) ^ ((xp >> 2) & (XCH - 1))) << 4) + (chn & 7) * 2;
      if (qv) {
        *reinterpret_cast<f16x4*>(X + byte) = oh;
        *reinterpret_cast<f16x4*>(X + XPL + byte) = ol;
      }
    }
  }
  __syncthreads();

  // ---- C: model.1 (3x3 s2 over the stem image), this wave's 32 x 32 block
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int t = 0; t < (A.dbg & 4 ? 0 : KST1); ++t) {
    const int J = 2 * t + h;  // this lane half's logical 8-channel chunk: (tap, channel chunk)
    const int tap = J / XCH, cj = J - tap * XCH;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int xp = xslot(2 * wm + ky, 2 * l32 + kx);
    const int byte = xp * XPB + ((cj ^ ((xp >> 2) & (XCH - 1))) << 4);
    const h8 xh = *reinterpret_cast<const h8*>(X + byte), xl = *reinterpret_cast<const h8*>(X + XPL + byte);
    const h8 wh = w1h[t % WPF], wl = w1l[t % WPF];
    if (t + WPF < KST1) {  // refill the ring slot WPF steps ahead
      w1h[t % WPF] = ym_gld<h8>(W1 + 16 * (J + 2 * WPF));
      w1l[t % WPF] = ym_gld<h8>(W1 + 16 * (J + 2 * WPF) + 8);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, acc, 0, 0, 0);
  }

  // ---- D: model.1's activated output split into the LDS tile (the patch region is dead since phase B)
  const int tp = 32 * wm + l32;  // tile pixel of this lane
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f16x4 oh, ol;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = ym_x3_pre(acc[4 * q + e], p.wsc, b1[q][e]);
      const float o = p.act ? ym_silu_x3(x) : x;
      oh[e] = (f16)o;
      ol[e] = (f16)(o - (float)oh[e]);
    }
    const int cj = 4 * wn + q;  // chunk of channels 32 wn + 8 q .. + 7; this lane's half at byte 8 h
    const int byte = tp * TPB + ((cj ^ (tp & 7)) << 4) + 8 * h;
    *reinterpret_cast<f16x4*>(U + byte) = oh;
    *reinterpret_cast<f16x4*>(U + TPL + byte) = ol;
  }
  __syncthreads();

  // ---- E: model.2.cv1 (1x1, K = N1) from the tile, then its pair-layout store
  f32x16 acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
#pragma unroll
  for (int t = 0; t < (A.dbg & 8 ? 0 : KST2); ++t) {
    const int J = 2 * t + h;
    const int byte = tp * TPB + ((J ^ (tp & 7)) << 4);
    const h8 xh = *reinterpret_cast<const h8*>(U + byte), xl = *reinterpret_cast<const h8*>(U + TPL + byte);
    const h8 wh = w2h[t], wl = w2l[t];
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, acc2, 0, 0, 0);
  }
  const int oy = oy0 + wm, ox = ox0 + l32;
  P2* dst = static_cast<P2*>(p.dst) + (size_t)(b * p.d_P + oy * p.d_W + ox) * p.d_ctot + p.d_coff;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = ym_x3_pre(acc2[4 * q + e], p.wsc2, b2[q][e]);
      o[e] = p.act2 ? ym_silu_x3(x) : x;
    }
    ym_p2_store4_pair<32>(dst + 32 * wn + 8 * q + 4 * h, o, h, !(A.dbg & 16), p.pst & 16);
  }
}

}  // namespace

// stem (s) + a fused 3x3 s2 -> 1x1 pair (p) reading the stem's output, x3 plans, yolo11s geometry (32 -> 64 -> 64);
// hipErrorInvalidValue for any other shape (the caller launches the two ops as before)
hipError_t ym_launch_stem_down_x3(const ConvArgs& s, const ConvArgs& p, hipStream_t st) {
  if (!s.nchw || !s.wstem || s.k != 3 || s.s != 2 || !s.act || s.N != 32 || s.Win % 4 || s.shuffle || s.res) return hipErrorInvalidValue;
  if (!p.x3 || !p.w2 || p.k2 != 1 || p.k != 3 || p.s != 2 || p.res || p.shuffle || p.src1 || p.up0 || p.dw_w || p.nchw)
    return hipErrorInvalidValue;
  if (p.src0 != s.dst || p.s0_coff != s.d_coff || p.s0_ctot != s.d_ctot || p.N != 64 || p.N2 != 64 ||
      p.Cin8 * 8 != 2 * 32 || p.Kpad < 2 * 9 * 32 || p.Kpad2 < 2 * 64)
    return hipErrorInvalidValue;
  if (s.Ho != 2 * p.Ho || s.Wo != 2 * p.Wo || s.Hin != 2 * s.Ho || s.Win != 2 * s.Wo || p.Wo % TW || p.Ho % RB ||
      ((p.N2 | p.d_coff | p.d_ctot) & 7) || s.M != 4 * p.M)
    return hipErrorInvalidValue;
  static const int dbg = [] { const char* e = getenv("YM_STEMFUSE_DBG"); return e ? atoi(e) : 0; }();
  StemFuseArgs A{s, p, dbg};
  const int B = p.M / (p.Ho * p.Wo);
  hipLaunchKernelGGL((stem_down_x3<32, 64, 64>), dim3(B * (p.Ho / RB) * (p.Wo / TW)), dim3(256), 0, st, A);
  return hipGetLastError();
}
