// Implicit-GEMM NHWC convolution for gfx950 (CDNA4) — the Conv (conv2d → folded BN → SiLU) hot path.
//
// Replaces the ATen conv2d + BN + SiLU + cat/upsample/add launches that Ultralytics' DetectionModel issues per
// `Conv` module under `YOLO11Model.predict` (/root/reference/core/model.py:133).
//
// GEMM view: M = B·Ho·Wo output pixels, N = Cout, K = k·k·Cin ordered (ky, kx, c) so that every 8-element K chunk
// is 8 consecutive channels of ONE input pixel = one 16-byte NHWC load (f16).  No im2col buffer: the A tile is
// gathered straight from the producer's NHWC buffer(s):
//   * two A sources split along K (concat fusion: channels [0, C0) from src0, [C0, C0+C1) from src1);
//   * src0 may be read at (y>>1, x>>1) (nearest 2x Upsample fused into the consumer's loader);
//   * channel-offset views (C2f chunk/split, SPPF/C3k2 concat slices) are just (ctot, coff) pairs.
// Epilogue: + bias (BN folded at pack time), SiLU, + residual (Bottleneck / PSA shortcut), store into a channel
// slice of the destination buffer, optionally fp32 into the anchor-major Detect buffer, or 2x2 pixel-shuffled
// (ConvTranspose2d(k=2,s=2) of the Segment Proto).
//
// Tiles: BM×BN output tile per 256-thread workgroup (4 waves as 2×2), BK = 32; A/B staged global → registers →
// LDS with the next K-step's global loads in flight during the current step's MFMAs.
//   f16 plans: v_mfma_f32_16x16x32_f16 (fp32 accumulate)
//   f32 plans: v_mfma_f32_16x16x4_f32  (exact-f32 MFMA: the parity mode)
#include "ym_common.h"

namespace {

constexpr int BK = 32;
constexpr int NT = 256;

template <typename T> struct LdsPad { static constexpr int v = 8; };
template <> struct LdsPad<float> { static constexpr int v = 1; };

template <typename T>
__device__ __forceinline__ typename Vec8<T>::type gather_a(const ConvArgs& a, int b, int iy0, int ix0, bool ok,
                                                           int tap, int cb) {
  if (!ok) return Vec8<T>::zero();
  int ky = 0, kx = tap;
  if (a.k != 1) { ky = tap / a.k; kx = tap - ky * a.k; } else { kx = 0; }
  const int iy = iy0 + ky, ix = ix0 + kx;
  if ((unsigned)iy >= (unsigned)a.Hin || (unsigned)ix >= (unsigned)a.Win) return Vec8<T>::zero();
  const int c = cb * 8;
  const T* p;
  if (c < a.C0) {
    const int sy = a.up0 ? (iy >> 1) : iy;
    const int sx = a.up0 ? (ix >> 1) : ix;
    p = static_cast<const T*>(a.src0) + ((size_t)(b * a.s0_P + sy * a.s0_W + sx) * a.s0_ctot + a.s0_coff + c);
  } else {
    p = static_cast<const T*>(a.src1) +
        ((size_t)(b * a.s1_P + iy * a.Win + ix) * a.s1_ctot + a.s1_coff + (c - a.C0));
  }
  return Vec8<T>::load(p);
}

template <typename T>
__device__ __forceinline__ void mma_step(const T* As, const T* Bs, int ldk, int lane, int arow, int bcol,
                                         f32x4& acc);

// f16: one 16x16x32 MFMA per (i, j) per K-step. Lane l holds A[row l&15][k 8(l>>4)..+8), B[k ..][col l&15].
template <>
__device__ __forceinline__ void mma_step<f16>(const f16* As, const f16* Bs, int ldk, int lane, int arow, int bcol,
                                              f32x4& acc) {
  const f16x8 av = *reinterpret_cast<const f16x8*>(As + (arow + (lane & 15)) * ldk + 8 * (lane >> 4));
  const f16x8 bv = *reinterpret_cast<const f16x8*>(Bs + (bcol + (lane & 15)) * ldk + 8 * (lane >> 4));
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
}

// f32: eight exact-f32 16x16x4 MFMAs per K-step. Lane l holds A[row l&15][k l>>4], B[k l>>4][col l&15].
template <>
__device__ __forceinline__ void mma_step<float>(const float* As, const float* Bs, int ldk, int lane, int arow,
                                                int bcol, f32x4& acc) {
#pragma unroll
  for (int kk = 0; kk < BK; kk += 4) {
    const float av = As[(arow + (lane & 15)) * ldk + kk + (lane >> 4)];
    const float bv = Bs[(bcol + (lane & 15)) * ldk + kk + (lane >> 4)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
  }
}

template <typename OutT> __device__ __forceinline__ OutT cvt_out(float x);
template <> __device__ __forceinline__ f16 cvt_out<f16>(float x) { return (f16)x; }
template <> __device__ __forceinline__ float cvt_out<float>(float x) { return x; }

template <typename T, typename OutT, int BM, int BN>
__global__ __launch_bounds__(NT) void conv_igemm_nhwc(const ConvArgs a) {
  constexpr int LDK = BK + LdsPad<T>::v;
  constexpr int NA = (BM * (BK / 8) + NT - 1) / NT;  // A chunks per thread
  constexpr int NB = (BN * (BK / 8) + NT - 1) / NT;  // B chunks per thread
  constexpr int TM = BM / 32, TN = BN / 32;           // 16x16 MFMA tiles per wave (2x2 waves)
  typedef typename Vec8<T>::type V;

  __shared__ T As[BM * LDK];
  __shared__ T Bs[BN * LDK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  const int bid = blockIdx.x;
  const int tn = bid % a.tiles_n;
  const int tm = bid / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int HWo = a.Ho * a.Wo;

  // per-thread A rows: fixed for the whole K loop
  int rb[NA], riy[NA], rix[NA];
  bool rok[NA];
  const int kc = tid & 3;  // this thread's 8-wide chunk inside a BK=32 step (same for every row it loads)
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r = (tid + i * NT) >> 2;
    const int m = m0 + r;
    rok[i] = (r < BM) && (m < a.M);
    const int mm = rok[i] ? m : 0;
    rb[i] = mm / HWo;
    const int rem = mm - rb[i] * HWo;
    const int oy = rem / a.Wo;
    const int ox = rem - oy * a.Wo;
    riy[i] = oy * a.s - a.pad;
    rix[i] = ox * a.s - a.pad;
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const T* W = static_cast<const T*>(a.w);
  V ra[NA], rbv[NB];
  const int nk = a.Kpad / BK;

  auto load_tiles = [&](int kt) {
    const int kchunk = kt * (BK / 8) + kc;
    const bool kok = kchunk < a.Kc;
    const int tap = kok ? kchunk / a.Cin8 : 0;
    const int cb = kchunk - tap * a.Cin8;
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = gather_a<T>(a, rb[i], riy[i], rix[i], rok[i] && kok, tap, cb);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * NT;
      const int n = n0 + (c >> 2);
      if ((c >> 2) < BN && n < a.N)
        rbv[i] = Vec8<T>::load(W + (size_t)n * a.Kpad + kt * BK + (c & 3) * 8);
      else
        rbv[i] = Vec8<T>::zero();
    }
  };

  load_tiles(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = (tid + i * NT) >> 2;
      if (r < BM) {
        T* dp = As + r * LDK + kc * 8;
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<V*>(dp) = ra[i];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) dp[e] = ra[i][e];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * NT;
      if ((c >> 2) < BN) {
        T* dp = Bs + (c >> 2) * LDK + (c & 3) * 8;
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<V*>(dp) = rbv[i];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) dp[e] = rbv[i][e];
        }
      }
    }
    __syncthreads();
    if (kt + 1 < nk) load_tiles(kt + 1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        mma_step<T>(As, Bs, LDK, lane, wr * (BM / 2) + i * 16, wc * (BN / 2) + j * 16, acc[i][j]);
  }

  // epilogue: bias, SiLU, residual, (shuffled) store into the destination channel slice
  OutT* dst = static_cast<OutT*>(a.dst);
  const T* res = static_cast<const T*>(a.res);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = m0 + wr * (BM / 2) + i * 16 + (lane >> 4) * 4 + v;
      if (row >= a.M) continue;
      const int b = row / HWo;
      const int rem = row - b * HWo;
      const int oy = rem / a.Wo;
      const int ox = rem - oy * a.Wo;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
        if (col >= a.N) continue;
        float x = acc[i][j][v] + a.bias[col];
        if (a.act) x = ym_silu(x);
        int pix, ch;
        if (a.shuffle) {
          const int sub = col / a.npr;
          ch = col - sub * a.npr;
          pix = (2 * oy + (sub >> 1)) * a.d_W + 2 * ox + (sub & 1);
        } else {
          ch = col;
          pix = oy * a.d_W + ox;
        }
        if (res) x += (float)res[(size_t)(b * a.r_P + pix) * a.r_ctot + a.r_coff + ch];
        dst[(size_t)(b * a.d_P + a.d_pixoff + pix) * a.d_ctot + a.d_coff + ch] = cvt_out<OutT>(x);
      }
    }
  }
}

template <typename T, typename OutT, int BM, int BN>
hipError_t launch(ConvArgs a, hipStream_t st) {
  const int tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  hipLaunchKernelGGL((conv_igemm_nhwc<T, OutT, BM, BN>), dim3(tiles_m * a.tiles_n), dim3(NT), 0, st, a);
  return hipGetLastError();
}

template <typename T, typename OutT>
hipError_t pick(const ConvArgs& a, hipStream_t st) {
  // tile choice: wide N tiles for wide layers, 128-pixel tiles when there are enough of them to fill 256 CUs
  const long tiles128 = (long)((a.M + 127) / 128) * ((a.N + 63) / 64);
  if (a.N <= 32) return launch<T, OutT, 128, 32>(a, st);
  if (tiles128 >= 512) return launch<T, OutT, 128, 64>(a, st);
  return launch<T, OutT, 64, 64>(a, st);
}

}  // namespace

hipError_t ym_launch_conv(int dtype, int out_f32, const ConvArgs& a, hipStream_t st) {
  if (dtype == YM_DT_F16) return out_f32 ? pick<f16, float>(a, st) : pick<f16, f16>(a, st);
  return pick<float, float>(a, st);
}
