// Streaming and small-M int8 convs (PTQ plans): the int8 counterparts of csrc/ym_conv_stream.hip.
//
// Same structure as the f16 kernels — conv_stream_i8: a persistent grid, the whole int8 weight matrix plus the
// per-channel requantisation parameters and the activation LUT in LDS, each wave streaming 16-pixel groups with the
// next group's fragments in flight; conv_small_i8: one 16 px x 16 ch block per 4-wave workgroup with K split four
// ways, partial int32 blocks summed in LDS (integer sums: the split never changes the result).
// The MFMA is v_mfma_i32_16x16x64_i8 in the transposed orientation (A = weights [N][Kpad], B = 16 channels of one
// pixel per lane, one 16-byte load); a lane ends with 4 consecutive output channels of one pixel.  Accumulation is
// exact int32 and the epilogue is the quantized-conv epilogue of csrc/ym_conv_i8.hip (ym_quant.h), so every kernel
// and configuration produces the same bytes.  Storage holds q - 128; a 3x3 tap outside the image reads z_in - 128
// (the value whose (q - z_in) is 0), the (128 - z_in)·Σw offset being folded into the per-channel int32 bias.
#include "ym_common.h"
#include "ym_quant.h"

namespace {

struct SCfg {
  int kind, ks, px, cap;  // 1x1 / 3x3; K steps of 64 (Kpad / 64); 16-pixel groups per wave iteration; grid cap
};
#define YM_I8S_CFGS(X)                                                                                            \
  X(0, 1, 1, 1, 1024) X(1, 1, 2, 1, 1024) X(2, 1, 4, 1, 1024) X(3, 1, 1, 2, 4096) X(4, 1, 2, 2, 4096)            \
  X(5, 1, 1, 1, 4096) X(6, 1, 2, 1, 4096) X(7, 3, 3, 1, 1024) X(8, 3, 5, 1, 1024) X(9, 3, 9, 1, 1024)            \
  X(10, 3, 3, 1, 4096) X(11, 3, 5, 1, 4096) X(12, 3, 9, 1, 4096) X(13, 3, 2, 1, 4096) X(14, 3, 2, 1, 1024)
constexpr SCfg kStream[] = {
#define YM_X(id, kind, ks, px, cap) {kind, ks, px, cap},
    YM_I8S_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumStream = sizeof(kStream) / sizeof(kStream[0]);

#define YM_I8M_CFGS(X) \
  X(0, 1, 1, 1) X(1, 1, 2, 1) X(2, 1, 4, 1) X(3, 1, 8, 1) X(4, 1, 2, 2) X(5, 3, 3, 1) X(6, 3, 5, 1) X(7, 3, 9, 1)
constexpr int kSmall[][3] = {
#define YM_X(id, kind, ksw, pxg) {kind, ksw, pxg},
    YM_I8M_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumSmall = sizeof(kSmall) / sizeof(kSmall[0]);
constexpr int kMaxLds = 80 * 1024;

// 16 channels of the lane's pixel for K step ks (1x1: channels 64 ks + 16 g; 3x3: chunk 4 ks + g of (tap, 16 ch))
template <int KIND>
__device__ __forceinline__ i8x16 gather(const ConvArgs& a, const i8* img, bool ok, int y, int x, int ks, int g,
                                        unsigned c16m, i8x16 fill) {
  const i8x16 zero = __builtin_bit_cast(i8x16, i32x4{0, 0, 0, 0});
  if constexpr (KIND == 1) {
    const int k0 = 64 * ks + 16 * g;
    if (!ok || k0 >= a.C0) return zero;
    return *reinterpret_cast<const i8x16*>(img + (size_t)(y * a.s0_W + x) * a.s0_ctot + k0);
  } else {
    const int c = 4 * ks + g;
    if (!ok || c >= a.Kc) return zero;
    const int t = (int)(((unsigned)c * c16m) >> 24), cb = c - t * a.Cin8;
    const int ky = t >= 6 ? 2 : (t >= 3 ? 1 : 0), kx = t - 3 * ky;
    const int iy = y * a.s - 1 + ky, ix = x * a.s - 1 + kx;
    if ((unsigned)iy >= (unsigned)a.Hin || (unsigned)ix >= (unsigned)a.Win) return fill;
    return *reinterpret_cast<const i8x16*>(img + (size_t)(iy * a.Win + ix) * a.s0_ctot + 16 * cb);
  }
}

// the quantized-conv epilogue of 4 consecutive channels n0.. of one pixel (csrc/ym_conv_i8.hip conv_i8)
template <bool F8>
__device__ __forceinline__ void epilogue4(const ConvArgs& a, const QRec* Q, int mode, const float* post,
                                          const typename Q8<F8>::acc4 acc, const int* bi, const float* sa,
                                          const float* bf, int n0, size_t obase, size_t rbase) {
  typedef Q8<F8> QS;
  const i8* res = static_cast<const i8*>(a.res);
  const int r4 = res ? *reinterpret_cast<const int*>(res + rbase + n0) : 0;
  int ov[4];
  float fv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int qc = QS::code(acc[e], F8 ? 0 : bi[e], sa[e], bf[e], Q);
    if (mode == 1) {
      ov[e] = QS::raw_byte(qc);
      fv[e] = 0.f;
      continue;
    }
    float v = post[qc];
    if (res) v = __fadd_rn(v, QS::dec(r4 >> (8 * e), Q->z_r, Q->s_r));
    fv[e] = v;
    ov[e] = QS::store(v, Q);
  }
  if (mode == 2) *reinterpret_cast<f32x4*>(static_cast<float*>(a.dst) + obase + n0) = f32x4{fv[0], fv[1], fv[2], fv[3]};
  else *reinterpret_cast<int*>(static_cast<i8*>(a.dst) + obase + n0) = pack4(ov);
}

// ------------------------------------------------------------------------------------------------ streaming
template <int KIND, int KS, int PX, bool F8>
__global__ __launch_bounds__(256) void conv_stream_i8(const ConvArgs a) {
  constexpr int KP = KS * 64;   // Kpad (bytes per weight row)
  // LDS row pitch KP + 32 bytes (4·KS + 2 16-byte slots): the 16-row fragment reads hit distinct slots in each of
  // ds_read_b128's non-contiguous lane groups (MI355X_MICROARCH §LDS); a +16 pitch is 2-way there
  constexpr int LDW = KP + 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int NP = (a.N + 15) & ~15;
  float* post = reinterpret_cast<float*>(smem);  // [256] activation LUT, then per channel: sasw, bias, biasi
  float* ssa = post + 256;
  float* sbf = ssa + NP;
  int* sbi = reinterpret_cast<int*>(sbf + NP);
  i8* ws = reinterpret_cast<i8*>(sbi + NP);      // [NP][LDW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const QRec* Q = a.q;
  const i8* W = static_cast<const i8*>(a.w);
  for (int i0 = tid; i0 < NP * (KP / 16); i0 += 256 * 8) {  // 8 loads in flight per thread and round
    i8x16 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + 256 * u, n = i / (KP / 16), c = i - n * (KP / 16);
      v[u] = (i < NP * (KP / 16) && n < a.N) ? *reinterpret_cast<const i8x16*>(W + (size_t)n * KP + 16 * c)
                                              : __builtin_bit_cast(i8x16, i32x4{0, 0, 0, 0});
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + 256 * u, n = i / (KP / 16), c = i - n * (KP / 16);
      if (i < NP * (KP / 16)) *reinterpret_cast<i8x16*>(ws + n * LDW + 16 * c) = v[u];
    }
  }
  post[tid] = Q->post[tid];
  for (int i = tid; i < NP; i += 256) {
    const bool v = i < a.N;
    ssa[i] = v ? a.sasw[i] : 0.f;
    sbf[i] = v ? a.bias[i] : 0.f;
    sbi[i] = v ? a.biasi[i] : 0;
  }
  const int HW = a.Ho * a.Wo;
  const int G = (a.M + 15) >> 4;
  // XCD-contiguous group ranges (as csrc/ym_conv_stream.hip conv_stream)
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nwx = (nwg >> 3) + (xcd < (nwg & 7));
  const int v0 = xcd * (nwg >> 3) + (xcd < (nwg & 7) ? xcd : (nwg & 7));
  const int gend = (int)((long)G * (v0 + nwx) / nwg);
  const int step = nwx * 4 * PX;
  const unsigned c16m = (0x1000000u + a.Cin8 - 1) / a.Cin8;
  const int fb = Q8<F8>::pad_byte(Q);
  const int f4 = fb | (fb << 8) | (fb << 16) | (fb << 24);
  const i8x16 fill = __builtin_bit_cast(i8x16, i32x4{f4, f4, f4, f4});
  const i8* s0 = static_cast<const i8*>(a.src0) + a.s0_coff;
  auto load = [&](int gb, i8x16 (&bf)[PX][KS]) {
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int m = (gb + p) * 16 + col;
      const bool ok = gb + p < gend && m < a.M;
      const int mm = ok ? m : 0;
      const int b = ym_div(mm, a.fd_hw), rem = mm - b * HW;
      const int y = ym_div(rem, a.fd_w), x = rem - y * a.Wo;
      const i8* img = s0 + (size_t)b * a.s0_P * a.s0_ctot;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bf[p][ks] = gather<KIND>(a, img, ok, y, x, ks, g, c16m, fill);
    }
  };
  int gb = (int)((long)G * v0 / nwg) + (slot * 4 + wave) * PX;
  i8x16 cur[PX][KS], nxt[PX][KS];
  load(gb, cur);
  __syncthreads();
  const int mode = Q->mode;
  for (; gb < gend; gb += step) {
    if (gb + step < gend) load(gb + step, nxt);
    size_t ob[PX], rb[PX];
    bool okp[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int m = (gb + p) * 16 + col;
      const int b = ym_div(m, a.fd_hw), rem = m - b * HW;
      const int y = ym_div(rem, a.fd_w), x = rem - y * a.Wo;
      okp[p] = gb + p < gend && m < a.M;
      ob[p] = (size_t)(b * a.d_P + a.d_pixoff + y * a.d_W + x) * a.d_ctot + a.d_coff;
      rb[p] = (size_t)(b * a.r_P + y * a.Wo + x) * a.r_ctot + a.r_coff;
    }
    for (int nb = 0; nb < NP / 16; ++nb) {
      i8x16 af[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[ks] = *reinterpret_cast<const i8x16*>(ws + (16 * nb + col) * LDW + 64 * ks + 16 * g);
      const int n0 = 16 * nb + 4 * g;
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        typename Q8<F8>::acc4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = mfma16(af[ks], cur[p][ks], acc);
        if (!okp[p] || n0 >= a.N) continue;
        epilogue4<F8>(a, Q, mode, post, acc, sbi + n0, ssa + n0, sbf + n0, n0, ob[p], rb[p]);
      }
    }
#pragma unroll
    for (int p = 0; p < PX; ++p)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) cur[p][ks] = nxt[p][ks];
  }
}

template <int KIND, int KS, int PX, int CAP, bool F8>
hipError_t launch_stream(const ConvArgs& a, hipStream_t st) {
  if (a.Kpad != KS * 64 || a.k != KIND) return hipErrorInvalidValue;
  const int G = (a.M + 15) / 16;
  long wgs = (G + 4 * PX - 1) / (4 * PX);
  if (wgs > CAP) wgs = CAP;
  const int NP = (a.N + 15) & ~15;
  const size_t lds = 256 * 4 + (size_t)NP * 12 + (size_t)NP * (KS * 64 + 32);
  if (lds > kMaxLds) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_stream_i8<KIND, KS, PX, F8>), dim3(wgs), dim3(256), lds, st, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------ small M
template <int KIND, int KSW, int PXG, bool F8>
__global__ __launch_bounds__(256) void conv_small_i8(const ConvArgs a) {
  typedef typename Q8<F8>::acc4 A4;
  __shared__ A4 red[3][PXG][64];
  __shared__ float post[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const QRec* Q = a.q;
  post[tid] = Q->post[tid];
  const int ntn = (a.N + 15) >> 4;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // each XCD owns one contiguous run of pixel blocks
  const int tn = vb % ntn, tm = vb / ntn;
  const int KS = a.Kpad >> 6;
  const int HW = a.Ho * a.Wo;
  const unsigned c16m = (0x1000000u + a.Cin8 - 1) / a.Cin8;
  const int fb = Q8<F8>::pad_byte(Q);
  const int f4 = fb | (fb << 8) | (fb << 16) | (fb << 24);
  const i8x16 fill = __builtin_bit_cast(i8x16, i32x4{f4, f4, f4, f4});
  const i8x16 zero = __builtin_bit_cast(i8x16, i32x4{0, 0, 0, 0});
  const int nrow = 16 * tn + col;
  const i8* wr = static_cast<const i8*>(a.w) + (size_t)(nrow < a.N ? nrow : 0) * a.Kpad + 16 * g;
  i8x16 af[KSW];
#pragma unroll
  for (int j = 0; j < KSW; ++j) {
    const int ks = wave + 4 * j;
    af[j] = (ks < KS && nrow < a.N) ? *reinterpret_cast<const i8x16*>(wr + 64 * ks) : zero;
  }
  const int nq = 16 * tn + 4 * g < a.N ? 16 * tn + 4 * g : 0;  // the epilogue's parameters, fetched up front
  const i32x4 bi = *reinterpret_cast<const i32x4*>(a.biasi + nq);
  const f32x4 sa = *reinterpret_cast<const f32x4*>(a.sasw + nq);
  const f32x4 bf = *reinterpret_cast<const f32x4*>(a.bias + nq);
  const i8* s0 = static_cast<const i8*>(a.src0) + a.s0_coff;
  i8x16 bfr[PXG][KSW];
  int b[PXG], y[PXG], x[PXG];
  bool ok[PXG];
#pragma unroll
  for (int p = 0; p < PXG; ++p) {
    const int m = (tm * PXG + p) * 16 + col;
    ok[p] = m < a.M;
    const int mm = ok[p] ? m : 0;
    b[p] = ym_div(mm, a.fd_hw);
    const int rem = mm - b[p] * HW;
    y[p] = ym_div(rem, a.fd_w);
    x[p] = rem - y[p] * a.Wo;
    const i8* img = s0 + (size_t)b[p] * a.s0_P * a.s0_ctot;
#pragma unroll
    for (int j = 0; j < KSW; ++j) {
      const int ks = wave + 4 * j;
      bfr[p][j] = ks < KS ? gather<KIND>(a, img, ok[p], y[p], x[p], ks, g, c16m, fill) : zero;
    }
  }
  A4 acc[PXG];
#pragma unroll
  for (int p = 0; p < PXG; ++p) {
    acc[p] = A4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < KSW; ++j) acc[p] = mfma16(af[j], bfr[p][j], acc[p]);
    if (wave > 0) red[wave - 1][p][lane] = acc[p];
  }
  __syncthreads();
  if (wave > 0) return;
  const int n0 = 16 * tn + 4 * g;
  if (n0 >= a.N) return;
  const int biv[4] = {bi[0], bi[1], bi[2], bi[3]};
  const float sav[4] = {sa[0], sa[1], sa[2], sa[3]}, bfv[4] = {bf[0], bf[1], bf[2], bf[3]};
  const int mode = Q->mode;
#pragma unroll
  for (int p = 0; p < PXG; ++p) {
    if (!ok[p]) continue;
    const A4 r = acc[p] + red[0][p][lane] + red[1][p][lane] + red[2][p][lane];
    const size_t ob = (size_t)(b[p] * a.d_P + a.d_pixoff + y[p] * a.d_W + x[p]) * a.d_ctot + a.d_coff;
    const size_t rb = (size_t)(b[p] * a.r_P + y[p] * a.Wo + x[p]) * a.r_ctot + a.r_coff;
    epilogue4<F8>(a, Q, mode, post, r, biv, sav, bfv, n0, ob, rb);
  }
}

template <int KIND, int KSW, int PXG, bool F8>
hipError_t launch_small(const ConvArgs& a, hipStream_t st) {
  if (a.k != KIND || a.Kpad > 256 * KSW) return hipErrorInvalidValue;
  const long wgs = (long)((a.M + 16 * PXG - 1) / (16 * PXG)) * ((a.N + 15) / 16);
  hipLaunchKernelGGL((conv_small_i8<KIND, KSW, PXG, F8>), dim3(wgs), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace

int ym_conv_i8_stream_num_cfgs() { return kNumStream + kNumSmall; }

// Host-side applicability: one plain source (int8 plans materialise concats and upsamples), no pixel shuffle,
// N % 4 == 0, 16-aligned channel slices, 1x1 stride 1 or 3x3 pad 1, LDS within 80 KB.
hipError_t ym_launch_conv_i8_stream(const ConvArgs& a, int i, hipStream_t st, bool f8) {
  if (i < 0 || i >= kNumStream + kNumSmall) return hipErrorInvalidValue;
  if (a.shuffle || a.src1 || a.up0 || !a.src0 || !a.q || !a.sasw || !a.biasi || (a.N & 3) || a.Kpad % 64)
    return hipErrorInvalidValue;
  if ((a.s0_ctot & 15) || (a.s0_coff & 15) || (a.d_ctot & 3) || (a.d_coff & 3) || (a.res && ((a.r_ctot & 3) || (a.r_coff & 3))))
    return hipErrorInvalidValue;
  if (a.k == 1 ? (a.s != 1) : (a.k != 3 || a.pad != 1 || a.Cin8 > 1024)) return hipErrorInvalidValue;
  switch (i) {
#define YM_X(id, kind, ks, px, cap) \
  case id: return f8 ? launch_stream<kind, ks, px, cap, true>(a, st) : launch_stream<kind, ks, px, cap, false>(a, st);
    YM_I8S_CFGS(YM_X)
#undef YM_X
  }
  switch (i - kNumStream) {
#define YM_X(id, kind, ksw, pxg) \
  case id: return f8 ? launch_small<kind, ksw, pxg, true>(a, st) : launch_small<kind, ksw, pxg, false>(a, st);
    YM_I8M_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}
