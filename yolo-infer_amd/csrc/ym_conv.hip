// Implicit-GEMM NHWC convolution for gfx950 (CDNA4) — the Conv (conv2d → folded BN → SiLU) hot path.
//
// Replaces the ATen conv2d + BN + SiLU + cat/upsample/add launches that Ultralytics' DetectionModel issues per
// `Conv` module under `YOLO11Model.predict` (/root/reference/core/model.py:133).
//
// GEMM orientation (transposed on purpose): D[n][m] = Σ_k W[n][k] · X[k][m] with
//   n = output channel (MFMA rows, A operand = packed weights [N][Kpad]),
//   m = output pixel   (MFMA cols, B operand = implicit im2col gathered straight from NHWC),
//   k = (ky, kx, c)    so every 8-element K chunk is 8 consecutive channels of ONE input pixel: one 16-byte load.
// With v_mfma_f32_32x32x16_f16 each lane then ends up holding 4 consecutive output channels of one pixel
// (rows (reg&3) + 8(reg>>2) + 4(lane>>5), col lane&31), so the epilogue writes 8-byte NHWC vectors without an LDS
// transpose.
//
// Structure (MI355X-specific choices):
//  * operands go global → VGPRs directly in MFMA fragment layout (A: W[n][8 k] 16 B, B: pixel's 8 channels 16 B),
//    double-buffered in registers: no LDS and no barrier in the main loop; latency is hidden by the next step's loads
//    in flight plus 4-8 waves per SIMD;
//  * intra-workgroup split-K: WK waves share one output tile and take interleaved K steps, then reduce their fp32
//    partial tiles once through LDS — this puts 4-8x more waves on the small-M deep layers (20x20, 40x40 maps);
//  * 1x1/stride-1 convs (half the launches) use a division-free gather: pixel row base + channel, with the two-source
//    concat (C3k2/C2PSA cv1/cv2 inputs) and the nearest-2x upsample (FPN) folded into the row base;
//  * epilogue: + bias (BN folded at pack time), SiLU, + residual (Bottleneck / PSA shortcut), store into a channel
//    slice of the destination buffer (zero-copy concat), fp32 into the anchor-major Detect buffer, or 2x2
//    pixel-shuffled (Segment Proto ConvTranspose2d(2,2)).
// f16 plans: v_mfma_f32_32x32x16_f16 (fp32 accumulate). f32 plans (parity mode): v_mfma_f32_32x32x2_f32 (exact f32).
#include <stdlib.h>

#include <type_traits>

#include "ym_common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

// Plan arithmetic modes: f16 (fp16 operands), float (exact-f32 MFMA) and x3_t (fp32 activations, weights packed as
// fp16 hi/lo planes, every K chunk as three f16 MFMAs on split operands; csrc/ym_common.h YM_DT_X3).
struct x3_t {};
template <typename M> struct Mode;
template <> struct Mode<f16> { typedef f16 act; typedef f16 wt; typedef f16x8 frag; };
template <> struct Mode<float> { typedef float act; typedef float wt; typedef f32x8 frag; };
template <> struct Mode<x3_t> { typedef P2 act; typedef f16 wt; typedef HL frag; };
// fp16 weight elements per logical 8-channel K chunk (x3: the [hi x8 | lo x8] pair)
template <typename M> constexpr int kWChunk = std::is_same<M, x3_t>::value ? 16 : 8;

// one lane's 8 consecutive K values of the weight operand (p: the chunk's first element)
template <typename M>
__device__ __forceinline__ typename Mode<M>::frag wload(const typename Mode<M>::wt* p) {
  if constexpr (std::is_same<M, x3_t>::value) return HL{Vec8<f16>::load(p), Vec8<f16>::load(p + 8)};
  else return Vec8<typename Mode<M>::wt>::load(p);
}
// one lane's 8 consecutive K values of the activation operand (p: a logical chunk start)
template <typename M>
__device__ __forceinline__ typename Mode<M>::frag xload(const typename Mode<M>::act* p) {
  if constexpr (std::is_same<M, x3_t>::value) return ym_load_hl(p);
  else return Vec8<typename Mode<M>::act>::load(p);
}
template <typename M>
__device__ __forceinline__ typename Mode<M>::frag xzero() {
  if constexpr (std::is_same<M, x3_t>::value) return HL{Vec8<f16>::zero(), Vec8<f16>::zero()};
  else return Vec8<typename Mode<M>::act>::zero();
}

template <typename M>
__device__ __forceinline__ void mma(const typename Mode<M>::frag& a, const typename Mode<M>::frag& b, f32x16& acc);

template <>
__device__ __forceinline__ void mma<f16>(const f16x8& a, const f16x8& b, f32x16& acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
}

// exact-f32: lane half h holds k = 8h..8h+7; MFMA s multiplies the pair {s, 8+s} (same k map on both operands)
template <>
__device__ __forceinline__ void mma<float>(const f32x8& a, const f32x8& b, f32x16& acc) {
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
}

// split f16: the small cross terms first, then hi·hi (lo·lo, below 2^-22 relative, is dropped)
template <>
__device__ __forceinline__ void mma<x3_t>(const HL& a, const HL& b, f32x16& acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.lo, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.hi, b.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.hi, b.hi, acc, 0, 0, 0);
}

template <typename OutT> struct Out4;
template <> struct Out4<P2> {
  static __device__ __forceinline__ void store(P2* p, const float* v) { ym_p2_store4(p, v); }
};
template <> struct Out4<f16> {
  static __device__ __forceinline__ void store(f16* p, const float* v) {
    *reinterpret_cast<f16x4*>(p) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
  }
};
template <> struct Out4<float> {
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  }
};

template <typename T>
__device__ __forceinline__ void load_res4(const T* p, float* v) {
  if constexpr (std::is_same<T, P2>::value) {
    float r[4];
    ym_p2_load4(p, r);
    v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3];
  } else if constexpr (sizeof(T) == 2) {
    const f16x4 r = *reinterpret_cast<const f16x4*>(p);
    v[0] += (float)r[0]; v[1] += (float)r[1]; v[2] += (float)r[2]; v[3] += (float)r[3];
  } else {
    const f32x4 r = *reinterpret_cast<const f32x4*>(p);
    v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3];
  }
}

// WTM: 32-pixel blocks per wave; WTN: 32-channel blocks per wave; WM x WN x WK waves per workgroup.
// KIND 1: 1x1 stride-1 (two sources, optional up-sampled first source); KIND 3: 3x3 (one source, stride a.s);
// KIND 0: the stem, a 3x3 whose source is the caller's NCHW fp32 batch (3 channels, /255 rule applied on load).
// One K step = 64 (4 MFMAs per block pair): 4x fewer dependent memory round trips than a 16-deep step.
constexpr int KSTEP = 64;
constexpr int KS64 = KSTEP / 16;

// XCD-aware tile map: workgroups are dealt round-robin over the 8 XCDs (bid % 8), so give every N tile of one pixel
// tile the same bid % 8 (the pixel rows they all read then sit in ONE XCD's L2), and give each XCD one contiguous run
// of pixel tiles (the rows a 3x3 tile shares with its neighbours too).  The grid is padded to a multiple of 8 pixel
// tiles; padding workgroups exit immediately.  (Placement only affects speed, never results.)
__device__ __forceinline__ bool xcd_tile(const ConvArgs& a, int BM, int& tm, int& tn) {
  const int bid = blockIdx.x;
  const int rest = bid >> 3;
  tn = rest % a.tiles_n;
  tm = (bid & 7) * (int)(gridDim.x / (8u * a.tiles_n)) + rest / a.tiles_n;
  return tm * BM < a.M;
}

template <typename M, typename OutT, int WTM, int WTN, int WM, int WN, int WK, int KIND>
__global__ __launch_bounds__(WM * WN * WK * 64) void conv_igemm(const ConvArgs a) {
  typedef typename Mode<M>::act T;
  typedef typename Mode<M>::wt WT;
  typedef typename Mode<M>::frag F;
  // K chunks of 16 per step: 4 (64-deep steps); x3 fragments are twice the registers, so 2 (32-deep steps) keep the
  // two register buffers of fragments within the VGPR budget
  constexpr int KS = std::is_same<M, x3_t>::value ? 2 : KS64;
  constexpr int BM = WM * WTM * 32, BN = WN * WTN * 32;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wk = wid % WK;
  const int wm = (wid / WK) % WM;
  const int wn = wid / (WK * WM);
  const int l32 = lane & 31, h = lane >> 5;
  int tm, tn;
  if (!xcd_tile(a, BM, tm, tn)) return;
  const int pbase = tm * BM + wm * WTM * 32;
  const int nbase = tn * BN + wn * WTN * 32;
  const int HWo = a.Ho * a.Wo;

  // ---- this lane's pixels (one per 32-pixel block)
  int pb[WTM], py[WTM], px[WTM], iy0[WTM], ix0[WTM];
  bool pv[WTM];
  const T* row0[WTM];  // KIND 1: row base in src0 (up-sample mapped); KIND 3: image base in src0
  const T* row1[WTM];  // KIND 1: row base in src1 (pre-offset by -C0)
#pragma unroll
  for (int i = 0; i < WTM; ++i) {
    const int m = pbase + i * 32 + l32;
    pv[i] = m < a.M;
    const int mm = pv[i] ? m : 0;
    pb[i] = mm / HWo;
    const int rem = mm - pb[i] * HWo;
    py[i] = rem / a.Wo;
    px[i] = rem - py[i] * a.Wo;
    if constexpr (KIND == 1) {
      const int sy = a.up0 ? (py[i] >> 1) : py[i];
      const int sx = a.up0 ? (px[i] >> 1) : px[i];
      row0[i] = static_cast<const T*>(a.src0) +
                ((size_t)(pb[i] * a.s0_P + sy * a.s0_W + sx) * a.s0_ctot + a.s0_coff);
      row1[i] = a.src1 ? static_cast<const T*>(a.src1) +
                             ((size_t)(pb[i] * a.s1_P + py[i] * a.Win + px[i]) * a.s1_ctot + a.s1_coff - a.C0)
                       : row0[i];
    } else {
      row0[i] = KIND == 3 ? static_cast<const T*>(a.src0) + ((size_t)pb[i] * a.s0_P * a.s0_ctot + a.s0_coff)
                          : nullptr;
      row1[i] = nullptr;
      iy0[i] = py[i] * a.s - 1;  // top-left input coordinate of the 3x3 window (pad 1)
      ix0[i] = px[i] * a.s - 1;
    }
  }
  const WT* wrow[WTN];
  // x3: Cin8 / Kc / Kpad count fp16 storage chunks; this kernel walks logical chunks (a [hi | lo] pair each)
  constexpr int XS = std::is_same<M, x3_t>::value ? 2 : 1;
  const int Cin8 = a.Cin8 / XS, Kc = a.Kc / XS;
#pragma unroll
  for (int j = 0; j < WTN; ++j) {
    const int n = nbase + j * 32 + l32;
    wrow[j] = static_cast<const WT*>(a.w) + (size_t)(n < a.N ? n : 0) * a.Kpad;
  }

  // ---- K walk. Step g (this wave: g = wk, wk+WK, ...) covers chunks [g*2KS, (g+1)*2KS); lane half h loads
  // chunks g*2KS + 2s + h, s < KS (chunk = 8 consecutive K = 8 channels of one tap).
  const int nsteps = a.Kpad / XS / (16 * KS);
  int g = wk;
  int tap0 = 0, cb0 = 0;  // KIND 3: tap / channel-block of chunk g*2KS + h
  if constexpr (KIND != 1) {
    const int c = g * 2 * KS + h;
    tap0 = c / Cin8;
    cb0 = c - tap0 * Cin8;
  }

  bool div255 = false;
  if constexpr (KIND == 0) div255 = ym_input_max(a.ctl) > 1.0f + a.eps;
  auto gather = [&](int i, int s) -> F {
    const int chunk = g * 2 * KS + 2 * s + h;
    if (!pv[i] || chunk >= Kc) return xzero<M>();
    if constexpr (KIND == 1) {
      const int c = chunk * 8;
      return xload<M>((c < a.C0 ? row0[i] : row1[i]) + c);
    } else if constexpr (KIND == 0) {  // Cin8 == 1: chunk = tap; channels 3..7 are zero padding
      const int ky = chunk / 3, kx = chunk - (chunk / 3) * 3;
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      if ((unsigned)iy >= (unsigned)a.Hin || (unsigned)ix >= (unsigned)a.Win) return Vec8<T>::zero();
      const size_t HW = (size_t)a.Hin * a.Win;
      const float* p = a.nchw + (size_t)pb[i] * 3 * HW + (size_t)iy * a.Win + ix;
      float x0 = p[0], x1 = p[HW], x2 = p[2 * HW];
      if (div255) { x0 = x0 / 255.0f; x1 = x1 / 255.0f; x2 = x2 / 255.0f; }
      F v = Vec8<T>::zero();
      v[0] = (T)x0; v[1] = (T)x1; v[2] = (T)x2;
      return v;
    } else {
      int cb = cb0 + 2 * s, t = tap0;
      while (cb >= Cin8) { cb -= Cin8; ++t; }
      const int ky = t / 3, kx = t - (t / 3) * 3;
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      if ((unsigned)iy >= (unsigned)a.Hin || (unsigned)ix >= (unsigned)a.Win) return xzero<M>();
      return xload<M>(row0[i] + (size_t)(iy * a.Win + ix) * a.s0_ctot + cb * 8);
    }
  };
  auto advance = [&]() {
    g += WK;
    if constexpr (KIND != 1) {
      cb0 += 2 * KS * WK;
      while (cb0 >= Cin8) { cb0 -= Cin8; ++tap0; }
    }
  };

  f32x16 acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  F fa0[KS][WTN], fb0[KS][WTM], fa1[KS][WTN], fb1[KS][WTM];
  auto load_step = [&](F (*fa)[WTN], F (*fb)[WTM]) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int j = 0; j < WTN; ++j) fa[s][j] = wload<M>(wrow[j] + (size_t)(g * 2 * KS + 2 * s + h) * kWChunk<M>);
#pragma unroll
      for (int i = 0; i < WTM; ++i) fb[s][i] = gather(i, s);
    }
  };
  auto compute = [&](F (*fa)[WTN], F (*fb)[WTM]) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j) mma<M>(fa[s][j], fb[s][i], acc[i][j]);
  };

  // epilogue operands (bias, residual) are fetched during the last step's MFMAs
  float bias[WTN][4][4];
  float resv[WTM][WTN][4][4];
  const T* res = static_cast<const T*>(a.res);
  auto load_epi = [&]() {
    if (wk != 0) return;
#pragma unroll
    for (int j = 0; j < WTN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nbase + j * 32 + 8 * q + 4 * h;
        const f32x4 b4 = n < a.N ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) bias[j][q][e] = b4[e];
      }
#pragma unroll
    for (int i = 0; i < WTM; ++i)
#pragma unroll
      for (int j = 0; j < WTN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) resv[i][j][q][e] = 0.f;
    if (res) {
#pragma unroll
      for (int i = 0; i < WTM; ++i) {
        if (!pv[i]) continue;
        const size_t rb = (size_t)(pb[i] * a.r_P + py[i] * a.Wo + px[i]) * a.r_ctot + a.r_coff;
#pragma unroll
        for (int j = 0; j < WTN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = nbase + j * 32 + 8 * q + 4 * h;
            if (n >= a.N) continue;
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            load_res4<T>(res + rb + n, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) resv[i][j][q][e] = v[e];
          }
      }
    }
  };

  if (g < nsteps) load_step(fa0, fb0);
  else load_epi();
  while (g < nsteps) {
    if (g + WK < nsteps) { advance(); load_step(fa1, fb1); } else { g += WK; load_epi(); }
    compute(fa0, fb0);
    if (g >= nsteps) break;
    if (g + WK < nsteps) { advance(); load_step(fa0, fb0); } else { g += WK; load_epi(); }
    compute(fa1, fb1);
  }

  // ---- split-K reduction through LDS (waves wk > 0 hand their partial tiles to wave wk == 0)
  if constexpr (WK > 1) {
    extern __shared__ float red[];  // [(WK-1)][WM*WN][WTM*WTN*16][64]
    constexpr int PER = WTM * WTN * 16;
    const int grp = wid / WK;
    if (wk > 0) {
      float* dst = red + ((size_t)((wk - 1) * (WM * WN) + grp) * PER) * 64 + lane;
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((i * WTN + j) * 16 + r) * 64] = acc[i][j][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll 1
    for (int q = 1; q < WK; ++q) {
      const float* src = red + ((size_t)((q - 1) * (WM * WN) + grp) * PER) * 64 + lane;
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += src[((i * WTN + j) * 16 + r) * 64];
    }
  }

  // ---- epilogue: lane owns channels nbase + 32j + 8q + 4h + {0..3} of pixel pbase + 32i + l32
  OutT* dst = static_cast<OutT*>(a.dst);
#pragma unroll
  for (int i = 0; i < WTM; ++i) {
    if (!pv[i]) continue;
    const int oy = py[i], ox = px[i];
    const int pix = a.shuffle ? (2 * oy) * a.d_W + 2 * ox : oy * a.d_W + ox;
    const size_t obase = (size_t)(pb[i] * a.d_P + a.d_pixoff + pix) * a.d_ctot + a.d_coff;
#pragma unroll
    for (int j = 0; j < WTN; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nbase + j * 32 + 8 * q + 4 * h;
        if (n >= a.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = std::is_same<M, x3_t>::value ? ym_x3_pre(acc[i][j][4 * q + e], a.wsc, bias[j][q][e])
                                                       : acc[i][j][4 * q + e] + bias[j][q][e];
          // f16 plans: the fp16-rounded output does not see the fast SiLU's ~1 ulp (fp32) error
          v[e] = (a.act ? (sizeof(OutT) == 2 ? ym_silu_fast(x)
                                             : (std::is_same<M, x3_t>::value ? ym_silu_x3(x) : ym_silu(x)))
                        : x) + resv[i][j][q][e];
          if (a.raw) a.raw[(size_t)(pbase + i * 32 + l32) * a.N + n + e] = x;  // f32 calibration run
        }
        if (a.shuffle) {
          const int sub = n / a.npr;
          const int ch = n - sub * a.npr;
          Out4<OutT>::store(dst + obase + (size_t)((sub >> 1) * a.d_W + (sub & 1)) * a.d_ctot + ch, v);
        } else {
          Out4<OutT>::store(dst + obase + n, v);
        }
      }
    }
  }
}

struct Cfg {
  int wtm, wtn, wm, wn, wk;
};

template <typename M, typename OutT, int WTM, int WTN, int WM, int WN, int WK>
hipError_t launch_cfg(ConvArgs a, int kind, hipStream_t st) {
  constexpr int BM = WM * WTM * 32, BN = WN * WTN * 32, NT = WM * WN * WK * 64;
  const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
  a.tiles_n = (a.N + BN - 1) / BN;
  const size_t lds = WK > 1 ? (size_t)(WK - 1) * WM * WN * WTM * WTN * 16 * 64 * sizeof(float) : 0;
  const dim3 grid(tiles_m8 * a.tiles_n);
  if (kind == 1)
    hipLaunchKernelGGL((conv_igemm<M, OutT, WTM, WTN, WM, WN, WK, 1>), grid, dim3(NT), lds, st, a);
  else
    hipLaunchKernelGGL((conv_igemm<M, OutT, WTM, WTN, WM, WN, WK, 3>), grid, dim3(NT), lds, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------------
// LDS-staged variant for the MFMA-dense layers (large K): one BM x BN tile per 256-thread workgroup (2x2 waves),
// 64-deep K stages double-buffered in LDS.  Every operand byte is loaded from global ONCE per workgroup with
// coalesced 16-byte row loads (8 lanes cover a 128-byte row), stored XOR-swizzled (chunk c of row r at c ^ ((r >> 1) & 7): conflict-free for ds_read_b128's non-contiguous lane groups)
// so the MFMA fragment reads (ds_read_b128, 32 rows at one K offset) do not pile onto one bank group; the next
// stage's global loads are in flight while the current stage's MFMAs run; one barrier per stage.
// x3 plans (M = x3_t): the [hi | lo] chunk pairs of activations and weights are staged as separate fp16 hi / lo
// planes; the fragment reads then feed the three MFMAs of mma<x3_t>.
template <typename M, typename OutT, int BM, int BN, int KIND>
__global__ __launch_bounds__(256) void conv_lds(const ConvArgs a) {
  typedef typename Mode<M>::act T;
  typedef typename Mode<M>::wt WT;
  constexpr bool X3 = std::is_same<M, x3_t>::value;
  constexpr int NP = X3 ? 2 : 1;   // fp16 planes per operand in LDS
  constexpr int BK = 64;
  constexpr int RB = BM * 8 / 256;  // pixel-row chunks per thread per stage
  constexpr int RA = BN * 8 / 256;  // weight-row chunks per thread per stage
  constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 blocks per wave (2x2 waves)
  typedef typename Vec8<T>::type V;
  typedef typename Mode<M>::frag WF;
  __shared__ __attribute__((aligned(16))) f16 sA[2][NP][BN * BK];
  __shared__ __attribute__((aligned(16))) f16 sB[2][NP][BM * BK];
  int tm, tn;
  if (!xcd_tile(a, BM, tm, tn)) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid & 1, wn = wid >> 1;
  const int l32 = lane & 31, h = lane >> 5;
  const int HWo = a.Ho * a.Wo;
  const int kc = tid & 7;  // this thread's chunk inside every 64-deep stage
  // pixel rows this thread stages
  const T* prow0[RB];
  const T* prow1[RB];
  int piy[RB], pix0[RB];
  bool pok[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int m = tm * BM + r;
    pok[i] = m < a.M;
    const int mm = pok[i] ? m : 0;
    const int b = mm / HWo, rem = mm - (mm / HWo) * HWo;
    const int oy = rem / a.Wo, ox = rem - (rem / a.Wo) * a.Wo;
    if constexpr (KIND == 1) {
      const int sy = a.up0 ? (oy >> 1) : oy, sx = a.up0 ? (ox >> 1) : ox;
      prow0[i] = static_cast<const T*>(a.src0) + ((size_t)(b * a.s0_P + sy * a.s0_W + sx) * a.s0_ctot + a.s0_coff);
      prow1[i] = a.src1 ? static_cast<const T*>(a.src1) +
                              ((size_t)(b * a.s1_P + oy * a.Win + ox) * a.s1_ctot + a.s1_coff - a.C0)
                        : prow0[i];
      piy[i] = pix0[i] = 0;
    } else {
      prow0[i] = static_cast<const T*>(a.src0) + ((size_t)b * a.s0_P * a.s0_ctot + a.s0_coff);
      prow1[i] = nullptr;
      piy[i] = oy * a.s - 1;
      pix0[i] = ox * a.s - 1;
    }
  }
  const WT* wrow[RA];
  constexpr int XS = X3 ? 2 : 1;  // x3: Cin8 / Kc / Kpad count fp16 storage chunks, a logical chunk is a pair
  const int Cin8 = a.Cin8 / XS, Kc = a.Kc / XS;
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int n = tn * BN + (tid >> 3) + 32 * i;
    wrow[i] = static_cast<const WT*>(a.w) + (size_t)(n < a.N ? n : 0) * a.Kpad;
  }
  int tap = 0, cb = kc;  // KIND 3: tap / channel block of chunk kt*8 + kc
  if constexpr (KIND == 3) {
    tap = kc / Cin8;
    cb = kc - tap * Cin8;
  }
  WF ra[RB];
  WF rw[RA];
  int kt = 0;
  auto load = [&]() {
    const int chunk = kt * 8 + kc;
#pragma unroll
    for (int i = 0; i < RA; ++i) rw[i] = wload<M>(wrow[i] + (size_t)chunk * kWChunk<M>);
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      WF v = xzero<M>();
      if (pok[i] && chunk < Kc) {
        if constexpr (KIND == 1) {
          const int c = chunk * 8;
          v = xload<M>((c < a.C0 ? prow0[i] : prow1[i]) + c);
        } else {
          const int ky = tap / 3, kx = tap - (tap / 3) * 3;
          const int iy = piy[i] + ky, ix = pix0[i] + kx;
          if ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win)
            v = xload<M>(prow0[i] + (size_t)(iy * a.Win + ix) * a.s0_ctot + cb * 8);
        }
      }
      ra[i] = v;
    }
    if constexpr (KIND == 3) {  // advance this thread's chunk by one stage (8 chunks)
      cb += 8;
      while (cb >= Cin8) { cb -= Cin8; ++tap; }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int r = (tid >> 3) + 32 * i;
      const int o = r * BK + ((kc ^ ((r >> 1) & 7)) * 8);
      if constexpr (X3) {
        *reinterpret_cast<f16x8*>(&sA[buf][0][o]) = rw[i].hi;
        *reinterpret_cast<f16x8*>(&sA[buf][1][o]) = rw[i].lo;
      } else {
        *reinterpret_cast<f16x8*>(&sA[buf][0][o]) = rw[i];
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = (tid >> 3) + 32 * i;
      const int o = r * BK + ((kc ^ ((r >> 1) & 7)) * 8);
      if constexpr (X3) {
        *reinterpret_cast<f16x8*>(&sB[buf][0][o]) = ra[i].hi;
        *reinterpret_cast<f16x8*>(&sB[buf][1][o]) = ra[i].lo;
      } else {
        *reinterpret_cast<f16x8*>(&sB[buf][0][o]) = ra[i];
      }
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = a.Kpad / XS / BK;
  load();
  store(0);
  __syncthreads();
  for (kt = 0; kt < nk;) {
    const int cur = kt & 1;
    ++kt;
    if (kt < nk) load();  // stage kt+1's global loads fly under this stage's MFMAs
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int cc = 2 * s + h;
      WF fa[TN], fb[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * (BN / 2) + j * 32 + l32;
        const int o = r * BK + ((cc ^ ((r >> 1) & 7)) * 8);
        if constexpr (X3) fa[j] = HL{*reinterpret_cast<const f16x8*>(&sA[cur][0][o]),
                                     *reinterpret_cast<const f16x8*>(&sA[cur][1][o])};
        else fa[j] = *reinterpret_cast<const f16x8*>(&sA[cur][0][o]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * (BM / 2) + i * 32 + l32;
        const int o = r * BK + ((cc ^ ((r >> 1) & 7)) * 8);
        if constexpr (X3) fb[i] = HL{*reinterpret_cast<const f16x8*>(&sB[cur][0][o]),
                                     *reinterpret_cast<const f16x8*>(&sB[cur][1][o])};
        else fb[i] = *reinterpret_cast<const f16x8*>(&sB[cur][0][o]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mma<M>(fa[j], fb[i], acc[i][j]);
    }
    if (kt < nk) store(cur ^ 1);
    __syncthreads();
  }
  // epilogue (same register layout as conv_igemm): lane owns channels n..n+3 of one pixel per (i, j, q)
  OutT* dst = static_cast<OutT*>(a.dst);
  const T* res = static_cast<const T*>(a.res);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = tm * BM + wm * (BM / 2) + i * 32 + l32;
    if (m >= a.M) continue;
    const int b = m / HWo, rem = m - (m / HWo) * HWo;
    const int oy = rem / a.Wo, ox = rem - (rem / a.Wo) * a.Wo;
    const int pix = a.shuffle ? (2 * oy) * a.d_W + 2 * ox : oy * a.d_W + ox;
    const size_t obase = (size_t)(b * a.d_P + a.d_pixoff + pix) * a.d_ctot + a.d_coff;
    const size_t rbase = res ? (size_t)(b * a.r_P + pix) * a.r_ctot + a.r_coff : 0;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = tn * BN + wn * (BN / 2) + j * 32 + 8 * q + 4 * h;
        if (n >= a.N) continue;
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bias + n);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = X3 ? ym_x3_pre(acc[i][j][4 * q + e], a.wsc, b4[e]) : acc[i][j][4 * q + e] + b4[e];
          v[e] = a.act ? (X3 ? ym_silu_x3(x) : ym_silu_fast(x)) : x;  // fast SiLU where the output is rounded to fp16
        }
        if (a.shuffle) {
          const int sub = n / a.npr;
          const int ch = n - sub * a.npr;
          Out4<OutT>::store(dst + obase + (size_t)((sub >> 1) * a.d_W + (sub & 1)) * a.d_ctot + ch, v);
        } else {
          if (res) load_res4<T>(res + rbase + n, v);
          Out4<OutT>::store(dst + obase + n, v);
        }
      }
    }
  }
}

template <typename M, typename OutT, int BM, int BN>
hipError_t launch_lds(ConvArgs a, int kind, hipStream_t st) {
  // x3: the 64-deep logical stage needs a storage Kpad of a multiple of 128 (pair-chunk rows are padded to 64)
  if (std::is_same<M, x3_t>::value && a.Kpad % 128) return hipErrorInvalidValue;
  const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
  a.tiles_n = (a.N + BN - 1) / BN;
  const dim3 grid(tiles_m8 * a.tiles_n);
  if (kind == 1) hipLaunchKernelGGL((conv_lds<M, OutT, BM, BN, 1>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((conv_lds<M, OutT, BM, BN, 3>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

// LDS-variant tile configurations (f16 and x3 plans): (id, BM, BN)
#define YM_LDS_CFGS(X) \
  X(12, 128, 128)      \
  X(13, 128, 64)       \
  X(14, 64, 128)       \
  X(15, 64, 64)        \
  X(16, 256, 64)

// The instantiated tile configurations: (id, WTM, WTN, WM, WN, WK).
#define YM_CONV_CFGS(X) \
  X(0, 2, 2, 2, 2, 1)   \
  X(1, 2, 2, 4, 1, 1)   \
  X(2, 2, 1, 4, 1, 1)   \
  X(3, 1, 2, 1, 1, 4)   \
  X(4, 1, 2, 1, 2, 4)   \
  X(5, 1, 2, 4, 1, 1)   \
  X(6, 2, 2, 1, 2, 2)   \
  X(7, 1, 1, 1, 1, 8)   \
  X(8, 1, 2, 2, 1, 2)   \
  X(9, 1, 1, 4, 1, 1)   \
  X(10, 1, 2, 2, 2, 1)  \
  X(11, 1, 1, 1, 1, 4)

constexpr int kNumCfg = 12;
constexpr Cfg kCfgs[kNumCfg] = {
#define YM_X(id, a, b, c, d, e) {a, b, c, d, e},
    YM_CONV_CFGS(YM_X)
#undef YM_X
};

constexpr int kNumAllCfg = 17;

template <typename M, typename OutT>
hipError_t launch_id(int id, const ConvArgs& a, int kind, hipStream_t st) {
  switch (id) {
#define YM_X(cid, A, B, C, D, E) \
  case cid: return launch_cfg<M, OutT, A, B, C, D, E>(a, kind, st);
    YM_CONV_CFGS(YM_X)
#undef YM_X
  }
  if constexpr (!std::is_same<M, float>::value) {
    switch (id) {
#define YM_X(cid, BM_, BN_) \
  case cid: return launch_lds<M, OutT, BM_, BN_>(a, kind, st);
      YM_LDS_CFGS(YM_X)
#undef YM_X
    }
  }
  return hipErrorInvalidValue;
}

// Default tile choice when no autotuned choice is given: fill the 256 CUs before making tiles big.
int choose_cfg(const ConvArgs& a) {
  const int id = ym_debug_get(9) - 1;  // YM_DBG_CONV_CFG (value + 1): a forced tile configuration (tools/tune)
  if (id >= 0 && id < kNumCfg) return id;
  const long M = a.M, N = a.N;
  const int steps = a.Kpad / KSTEP;
  auto waves = [&](int id) {
    const Cfg& c = kCfgs[id];
    const long BM = c.wm * c.wtm * 32, BN = c.wn * c.wtn * 32;
    return ((M + BM - 1) / BM) * ((N + BN - 1) / BN) * c.wm * c.wn * c.wk;
  };
  if (N <= 32) return waves(2) >= 2048 ? 2 : (steps >= 4 ? 7 : 9);
  if (N <= 64) {
    if (waves(1) >= 2048) return 1;
    if (waves(5) >= 2048) return 5;
    return steps >= 4 ? 3 : 8;
  }
  if (waves(0) >= 2048) return 0;
  if (waves(10) >= 2048) return 10;
  return steps >= 4 ? 4 : 6;
}

}  // namespace

// ids [0, 17): first-generation kernels above; [17, 17 + ym_conv_dma_num_cfgs()): LDS-DMA / split-K kernels;
// then ym_conv_stream_num_cfgs() streaming / small-M kernels (csrc/ym_conv_stream.hip), then
// ym_conv_halo_num_cfgs() halo-tile 3x3 kernels (csrc/ym_conv_halo.hip), then ym_conv_bneck_num_cfgs() fused
// Bottleneck kernels (csrc/ym_conv_bneck.hip; fused pairs with a 3x3 successor only) — appended last so the ids of
// committed tables stay valid
int ym_conv_num_cfgs() {
  return kNumAllCfg + ym_conv_dma_num_cfgs() + ym_conv_stream_num_cfgs() + ym_conv_halo_num_cfgs() +
         ym_conv_bneck_num_cfgs();
}
// x3 plans: + the x3-only LDS-DMA configurations, appended (the f16 ids, and so the f16 tables, are unchanged)
int ym_conv_num_cfgs_dt(int dtype) {
  // int8: conv_i8 / streaming ids, then the LDS-DMA configurations in their Q8 mode (round 6); fp8: conv_i8 only
  if (dtype == YM_DT_I8) return ym_conv_i8_num_cfgs() + ym_conv_dma_num_cfgs();
  if (ym_dt_q8(dtype)) return ym_conv_i8_num_cfgs();
  return ym_conv_num_cfgs() + (dtype == YM_DT_X3 ? ym_conv_dma_x3_num_cfgs() + ym_conv_bneck_x3_num_cfgs() : 0);
}

hipError_t ym_launch_conv(int dtype, int out_f32, const ConvArgs& a, int cfg, hipStream_t st, bool strict) {
  // a depthwise-fused 1x1 (csrc/ym_conv_dwpw.hip) runs on its own kernel only: no other family computes the depthwise
  if (a.dw_w) return ym_launch_conv_dwpw(dtype, out_f32, a, cfg, st, strict);
  int kind;
  if (a.nchw) kind = (a.k == 3 && a.Cin8 == 1) ? 0 : -1;
  else if (a.k == 1 && a.s == 1) kind = 1;
  else if (a.k == 3 && !a.src1 && !a.up0) kind = 3;
  else kind = -1;
  if (kind < 0) return hipErrorInvalidValue;
  if (ym_dt_q8(dtype)) return ym_launch_conv_i8(a, cfg, st, strict, dtype == YM_DT_F8);  // csrc/ym_conv_i8.hip
  // (concat/upsample sources only feed 1x1 convs; YOLO11 has k in {1, 3})
  if (a.Kpad % KSTEP) return hipErrorInvalidValue;
  if (a.w2 && a.k2 == 3) {  // fused Bottleneck (3x3 -> 3x3): csrc/ym_conv_bneck.hip (f16 and x3 plans)
    if (dtype != YM_DT_F16 && dtype != YM_DT_X3) return hipErrorInvalidValue;
    const int bb = kNumAllCfg + ym_conv_dma_num_cfgs() + ym_conv_stream_num_cfgs() + ym_conv_halo_num_cfgs();
    const int nb = ym_conv_bneck_num_cfgs();
    const int xb = ym_conv_num_cfgs() + ym_conv_dma_x3_num_cfgs();  // x3-only Bottleneck ids
    if (cfg >= bb && cfg < bb + nb) {
      const hipError_t e = ym_launch_conv_bneck(out_f32, a, cfg - bb, st);
      if (e != hipErrorInvalidValue || strict) return e;
    } else if (dtype == YM_DT_X3 && cfg >= xb && cfg < xb + ym_conv_bneck_x3_num_cfgs()) {
      const hipError_t e = ym_launch_conv_bneck(out_f32, a, nb + cfg - xb, st);
      if (e != hipErrorInvalidValue || strict) return e;
    } else if (strict) {
      return hipErrorInvalidValue;
    }
    for (int i = 0; i < nb; ++i) {  // untuned: the first variant that takes the shape
      const hipError_t e = ym_launch_conv_bneck(out_f32, a, i, st);
      if (e != hipErrorInvalidValue) return e;
    }
    return hipErrorInvalidValue;
  }
  if (a.w2) {  // fused pair: the streaming kernels hold a whole N in one wave (csrc/ym_conv_stream.hip); a stride-2
    // 3x3 followed by a 1x1 can also take the band kernel of csrc/ym_conv_bneck.hip (f16 only)
    if (dtype != YM_DT_F16 && dtype != YM_DT_X3) return hipErrorInvalidValue;
    const int bb = kNumAllCfg + ym_conv_dma_num_cfgs() + ym_conv_stream_num_cfgs() + ym_conv_halo_num_cfgs();
    if (cfg >= bb && cfg < bb + ym_conv_bneck_num_cfgs()) {
      const hipError_t e = ym_launch_conv_bneck(out_f32, a, cfg - bb, st);
      if (e != hipErrorInvalidValue || strict) return e;
    }
    const int sbase = kNumAllCfg + ym_conv_dma_num_cfgs(), ns = ym_conv_stream_num_cfgs();
    if (dtype == YM_DT_X3 && a.k2 == 1 && cfg >= kNumAllCfg && cfg < sbase) {  // LDS-DMA ids: the fused-epilogue GEMM
      const hipError_t e = ym_launch_conv_dma_fuse(out_f32, a, cfg - kNumAllCfg, st);
      if (e != hipErrorInvalidValue || strict) return e;
    }
    if (cfg >= sbase && cfg < sbase + ns) {
      const hipError_t e = ym_launch_conv_stream(out_f32, a, cfg - sbase, st);
      if (e != hipErrorInvalidValue || strict) return e;
    } else if (strict) {
      return hipErrorInvalidValue;
    }
    for (int i = 0; i < ns; ++i) {  // untuned: the first streaming variant that takes the shape
      const hipError_t e = ym_launch_conv_stream(out_f32, a, i, st);
      if (e != hipErrorInvalidValue) return e;
    }
    return hipErrorInvalidValue;
  }
  if (dtype == YM_DT_X3 && cfg >= ym_conv_num_cfgs()) {  // the x3-only LDS-DMA configurations (and, past them, the
                                                          // x3-only Bottleneck ids: inapplicable to a single conv)
    const hipError_t e = ym_launch_conv_dma(out_f32, a, ym_conv_dma_num_cfgs() + cfg - ym_conv_num_cfgs(), st);
    if (e != hipErrorInvalidValue || strict) return e;
    cfg = -1;
  }
  if (cfg >= kNumAllCfg) {
    // a DMA config that does not apply to this op (checked before anything is launched): the tuner skips the
    // candidate (strict); a pinned table falls back to the heuristic
    const int ndma = ym_conv_dma_num_cfgs(), nstr = ym_conv_stream_num_cfgs();
    hipError_t e = hipErrorInvalidValue;
    if (dtype == YM_DT_F16 || (dtype == YM_DT_X3 && cfg - kNumAllCfg < ndma + nstr)) {  // x3: LDS-DMA, streaming
      const int i = cfg - kNumAllCfg;
      e = i < ndma ? ym_launch_conv_dma(out_f32, a, i, st)
                   : (i < ndma + nstr ? ym_launch_conv_stream(out_f32, a, i - ndma, st)
                                      : ym_launch_conv_halo(out_f32, a, i - ndma - nstr, st));
    }
    if (e != hipErrorInvalidValue || strict) return e;
    cfg = -1;
  }
  int id = (cfg >= 0 && cfg < kNumAllCfg) ? cfg : choose_cfg(a);
  if (id >= kNumCfg && dtype == YM_DT_F32) id = choose_cfg(a);  // LDS variants: f16 and x3 plans
  if (dtype == YM_DT_F16) return out_f32 ? launch_id<f16, float>(id, a, kind, st) : launch_id<f16, f16>(id, a, kind, st);
  if (dtype == YM_DT_X3) {
    auto go = [&](int i) { return out_f32 ? launch_id<x3_t, float>(i, a, kind, st) : launch_id<x3_t, P2>(i, a, kind, st); };
    const hipError_t e = go(id);
    // an LDS tile whose 64-deep stage does not divide this op's K: the tuner skips it (strict), a pinned table
    // falls back to the heuristic direct-to-register tile
    return (e == hipErrorInvalidValue && !strict && id >= kNumCfg) ? go(choose_cfg(a)) : e;
  }
  return launch_id<float, float>(id, a, kind, st);
}
