// int8 (PTQ) kernels for gfx950: the quantized runtime behind the reference's PostTrainingQuantizer
// (/root/reference/optimization/quantization/quantizers.py:24-308; qconfig :124-131) — SURVEY §8a row a20, config 4.
//
// Numerics (pinned by oracle/quant.py, bit-exact apart from the float attention island):
//   activations are stored as int8 b = q - 128 (q = quint8 value, per-tensor affine), weights int8 symmetric;
//   a quantized conv accumulates Σ b·w with v_mfma_i32_32x32x32_i8 and adds the per-channel int32 correction
//   Σ_k (128 - z_in)·w, which makes acc = Σ (q - z_in)·w exactly (3x3 padding taps read the byte z_in - 128, i.e.
//   real zero); then y = float(acc)·(s_in·s_w) + bias, q_c = clamp(rint(y / s_out) + z_out), and the epilogue maps
//   q_c through the op's 256-entry `post` table (SiLU or plain dequant of the requantised output), adds the residual
//   ((q_r - z_r)·s_r), and quantizes into the stored tensor (or writes fp32 head rows).  Every float step rounds
//   once, as the oracle's separate torch fp32 ops do (ym_opaque keeps hipcc from fusing a multiply into an add).
//
// Kernels: conv_i8 (implicit GEMM over NHWC int8, same transposed orientation and tile structure as
// csrc/ym_conv.hip: MFMA A = weights [N][Kpad], B = im2col gathered straight from NHWC, one 16-byte K chunk = 16
// channels of one input pixel) — the int8 stem (the image's quantisation folded into the 3x3 s2 conv) is in
// csrc/ym_stem.hip —
// dwconv3x3_i8, attn_psa_i8 (float attention on dequantised q/k/v + int8 positional depthwise conv), requant (the
// materialised concats of an int8 plan).
#include <stdlib.h>

#include "ym_common.h"
#include "ym_quant.h"



namespace {

constexpr int KSTEP = 64;        // K bytes per step: two 32-deep MFMAs per 32x32 block pair
constexpr int KS = KSTEP / 32;

__device__ __forceinline__ i8x16 ld16(const i8* p) { return *reinterpret_cast<const i8x16*>(p); }

__device__ __forceinline__ bool xcd_tile(const ConvArgs& a, int BM, int& tm, int& tn) {
  const int bid = blockIdx.x;
  const int rest = bid >> 3;
  tn = rest % a.tiles_n;
  tm = (bid & 7) * (int)(gridDim.x / (8u * a.tiles_n)) + rest / a.tiles_n;  // one contiguous run per XCD
  return tm * BM < a.M;
}

// WTM x WTN 32x32 blocks per wave; WM x WN x WK waves (WK: intra-workgroup split-K, partial tiles summed through LDS
// — integer sums, so the result does not depend on the split).  KIND 1: 1x1 stride 1; KIND 3: 3x3 (stride a.s).
// a.Cin8 holds the number of 16-channel blocks per tap in int8 plans.
template <int WTM, int WTN, int WM, int WN, int WK, int KIND, bool F8>
__global__ __launch_bounds__(WM * WN * WK * 64) void conv_i8(const ConvArgs a) {
  typedef Q8<F8> QS;
  constexpr int BM = WM * WTM * 32, BN = WN * WTN * 32, NT = WM * WN * WK * 64;
  __shared__ float post[256];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wk = wid % WK;
  const int wm = (wid / WK) % WM;
  const int wn = wid / (WK * WM);
  const int l32 = lane & 31, h = lane >> 5;
  int tm, tn;
  if (!xcd_tile(a, BM, tm, tn)) return;
  const QRec* Q = a.q;
  for (int i = threadIdx.x; i < 256; i += NT) post[i] = Q->post[i];
  __syncthreads();
  const int pbase = tm * BM + wm * WTM * 32;
  const int nbase = tn * BN + wn * WTN * 32;
  const int HWo = a.Ho * a.Wo;

  int pb[WTM], py[WTM], px[WTM], iy0[WTM], ix0[WTM];
  bool pv[WTM];
  const i8* row0[WTM];
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
      row0[i] = static_cast<const i8*>(a.src0) + ((size_t)(pb[i] * a.s0_P + py[i] * a.s0_W + px[i]) * a.s0_ctot + a.s0_coff);
    } else {
      row0[i] = static_cast<const i8*>(a.src0) + ((size_t)pb[i] * a.s0_P * a.s0_ctot + a.s0_coff);
    }
    iy0[i] = py[i] * a.s - 1;
    ix0[i] = px[i] * a.s - 1;
  }
  const i8* wrow[WTN];
#pragma unroll
  for (int j = 0; j < WTN; ++j) {
    const int n = nbase + j * 32 + l32;
    wrow[j] = static_cast<const i8*>(a.w) + (size_t)(n < a.N ? n : 0) * a.Kpad;
  }

  const int nsteps = a.Kpad / KSTEP;
  int g = wk;
  int tap0 = 0, cb0 = 0;
  if constexpr (KIND == 3) {
    const int c = g * 2 * KS + h;
    tap0 = c / a.Cin8;
    cb0 = c - tap0 * a.Cin8;
  }
  const int fb = QS::pad_byte(Q);
  const int f4 = fb | (fb << 8) | (fb << 16) | (fb << 24);
  const i8x16 FILL = __builtin_bit_cast(i8x16, i32x4{f4, f4, f4, f4});
  const i8x16 ZERO = __builtin_bit_cast(i8x16, i32x4{0, 0, 0, 0});
  auto gather = [&](int i, int s) -> i8x16 {
    const int chunk = g * 2 * KS + 2 * s + h;
    if (!pv[i] || chunk >= a.Kc) return ZERO;
    if constexpr (KIND == 1) {
      return ld16(row0[i] + chunk * 16);
    } else {
      int cb = cb0 + 2 * s, t = tap0;
      while (cb >= a.Cin8) { cb -= a.Cin8; ++t; }
      const int ky = t / 3, kx = t - (t / 3) * 3;
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      if ((unsigned)iy >= (unsigned)a.Hin || (unsigned)ix >= (unsigned)a.Win) return FILL;
      return ld16(row0[i] + (size_t)(iy * a.Win + ix) * a.s0_ctot + cb * 16);
    }
  };
  auto advance = [&]() {
    g += WK;
    if constexpr (KIND == 3) {
      cb0 += 2 * KS * WK;
      while (cb0 >= a.Cin8) { cb0 -= a.Cin8; ++tap0; }
    }
  };

  typename QS::acc16 acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  i8x16 fa0[KS][WTN], fb0[KS][WTM], fa1[KS][WTN], fb1[KS][WTM];
  auto load_step = [&](i8x16 (*fa)[WTN], i8x16 (*fbv)[WTM]) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int j = 0; j < WTN; ++j) fa[s][j] = ld16(wrow[j] + (size_t)(g * 2 * KS + 2 * s + h) * 16);
#pragma unroll
      for (int i = 0; i < WTM; ++i) fbv[s][i] = gather(i, s);
    }
  };
  auto compute = [&](i8x16 (*fa)[WTN], i8x16 (*fbv)[WTM]) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j)
          acc[i][j] = mfma32(fa[s][j], fbv[s][i], acc[i][j]);
  };

  if (g < nsteps) load_step(fa0, fb0);
  while (g < nsteps) {
    if (g + WK < nsteps) { advance(); load_step(fa1, fb1); } else { g += WK; }
    compute(fa0, fb0);
    if (g >= nsteps) break;
    if (g + WK < nsteps) { advance(); load_step(fa0, fb0); } else { g += WK; }
    compute(fa1, fb1);
  }

  if constexpr (WK > 1) {
    extern __shared__ int red_raw[];  // [(WK-1)][WM*WN][WTM*WTN*16][64]
    typename QS::acc_t* red = reinterpret_cast<typename QS::acc_t*>(red_raw);
    constexpr int PER = WTM * WTN * 16;
    const int grp = wid / WK;
    if (wk > 0) {
      typename QS::acc_t* dst = red + ((size_t)((wk - 1) * (WM * WN) + grp) * PER) * 64 + lane;
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
      const typename QS::acc_t* src = red + ((size_t)((q - 1) * (WM * WN) + grp) * PER) * 64 + lane;
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += src[((i * WTN + j) * 16 + r) * 64];
    }
  }

  // ---- epilogue: lane owns channels nbase + 32j + 8q + 4h + {0..3} of pixel pbase + 32i + l32
  const int mode = Q->mode;
  const i8* res = static_cast<const i8*>(a.res);
#pragma unroll
  for (int i = 0; i < WTM; ++i) {
    if (!pv[i]) continue;
    const int oy = py[i], ox = px[i];
    const int pix = a.shuffle ? (2 * oy) * a.d_W + 2 * ox : oy * a.d_W + ox;
    const size_t obase = (size_t)(pb[i] * a.d_P + a.d_pixoff + pix) * a.d_ctot + a.d_coff;
    const size_t rbase = res ? (size_t)(pb[i] * a.r_P + oy * a.Wo + ox) * a.r_ctot + a.r_coff : 0;
#pragma unroll
    for (int j = 0; j < WTN; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nbase + j * 32 + 8 * q + 4 * h;
        if (n >= a.N) continue;
        const i32x4 bi = F8 ? i32x4{0, 0, 0, 0} : *reinterpret_cast<const i32x4*>(a.biasi + n);
        const f32x4 sa = *reinterpret_cast<const f32x4*>(a.sasw + n);
        const f32x4 bf = *reinterpret_cast<const f32x4*>(a.bias + n);
        const int r4 = res ? *reinterpret_cast<const int*>(res + rbase + n) : 0;
        int ov[4];
        float fv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int qc = QS::code(acc[i][j][4 * q + e], bi[e], sa[e], bf[e], Q);
          if (mode == 1) {
            ov[e] = QS::raw_byte(qc);
            continue;
          }
          float v = post[qc];
          if (res) v = __fadd_rn(v, QS::dec(r4 >> (8 * e), Q->z_r, Q->s_r));
          fv[e] = v;
          ov[e] = QS::store(v, Q);
        }
        size_t off = obase + n;
        if (a.shuffle) {
          const int sub = n / a.npr;
          const int ch = n - sub * a.npr;
          off = obase + (size_t)((sub >> 1) * a.d_W + (sub & 1)) * a.d_ctot + ch;
        }
        if (mode == 2) *reinterpret_cast<f32x4*>(static_cast<float*>(a.dst) + off) = f32x4{fv[0], fv[1], fv[2], fv[3]};
        else *reinterpret_cast<int*>(static_cast<i8*>(a.dst) + off) = pack4(ov);
      }
    }
  }
}

template <int WTM, int WTN, int WM, int WN, int WK, bool F8>
hipError_t launch_cfg(ConvArgs a, int kind, hipStream_t st) {
  constexpr int BM = WM * WTM * 32, BN = WN * WTN * 32, NT = WM * WN * WK * 64;
  const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
  a.tiles_n = (a.N + BN - 1) / BN;
  const size_t lds = WK > 1 ? (size_t)(WK - 1) * WM * WN * WTM * WTN * 16 * 64 * sizeof(int) : 0;
  const dim3 grid(tiles_m8 * a.tiles_n);
  if (kind == 1)
    hipLaunchKernelGGL((conv_i8<WTM, WTN, WM, WN, WK, 1, F8>), grid, dim3(NT), lds, st, a);
  else
    hipLaunchKernelGGL((conv_i8<WTM, WTN, WM, WN, WK, 3, F8>), grid, dim3(NT), lds, st, a);
  return hipGetLastError();
}

// (id, WTM, WTN, WM, WN, WK) — the same tile family as the f16/f32 conv_igemm configs
#define YM_I8_CFGS(X) \
  X(0, 2, 2, 2, 2, 1)  \
  X(1, 2, 2, 4, 1, 1)  \
  X(2, 2, 1, 4, 1, 1)  \
  X(3, 1, 2, 1, 1, 4)  \
  X(4, 1, 2, 1, 2, 4)  \
  X(5, 1, 2, 4, 1, 1)  \
  X(6, 2, 2, 1, 2, 2)  \
  X(7, 1, 1, 1, 1, 8)  \
  X(8, 1, 2, 2, 1, 2)  \
  X(9, 1, 1, 4, 1, 1)  \
  X(10, 1, 2, 2, 2, 1) \
  X(11, 1, 1, 1, 1, 4)

struct Cfg {
  int wtm, wtn, wm, wn, wk;
};
constexpr Cfg kCfgs[] = {
#define YM_X(id, a, b, c, d, e) {a, b, c, d, e},
    YM_I8_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumCfg = sizeof(kCfgs) / sizeof(kCfgs[0]);

hipError_t launch_id(int id, const ConvArgs& a, int kind, hipStream_t st, bool f8) {
  switch (id) {
#define YM_X(cid, A, B, C, D, E) \
  case cid: return f8 ? launch_cfg<A, B, C, D, E, true>(a, kind, st) : launch_cfg<A, B, C, D, E, false>(a, kind, st);
    YM_I8_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

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

// ------------------------------------------------------------------------------------------------- depthwise
// DWConv 3x3 (Detect cv3): one thread = 8 channels of one pixel; acc = Σ over in-image taps (q - z_in)·w, then the
// quantized-conv epilogue (mode 0).  fp8: the 9 products of e4m3 values are summed in float64 (exact: 8-bit
// significands) and rounded to fp32 once, as the oracle's float64 conv does.
template <bool F8>
__global__ __launch_bounds__(256) void dwconv3x3_i8(const DwArgs a) {
  typedef Q8<F8> QS;
  __shared__ float post[256];
  const QRec* Q = a.q;
  post[threadIdx.x] = Q->post[threadIdx.x];
  __syncthreads();
  const int C8 = a.C >> 3;
  // 32-bit index math (checked < 2^31 on the host); one contiguous run of blocks per XCD (shared tap rows)
  const int idx = ym_xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int total = a.B * a.H * a.W * C8;
  if (idx >= total) return;
  const int pix = idx / C8;
  const int cg = idx - pix * C8;
  const int HW = a.H * a.W;
  const int b = pix / HW;
  const int p = pix - b * HW;
  const int y = p / a.W, x = p - (p / a.W) * a.W;
  const int c0 = cg * 8;
  const i8* src = static_cast<const i8*>(a.src);
  typedef Vec8<i8>::type V;
  V v[9], w[9];
  bool ok[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
    ok[t] = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    v[t] = ok[t] ? Vec8<i8>::load(src + (size_t)(b * a.s_P + iy * a.W + ix) * a.s_ctot + a.s_coff + c0)
                 : Vec8<i8>::zero();
    w[t] = Vec8<i8>::load(a.wq + t * a.C + c0);
  }
  const int zi = Q->z_in;
  const f32x4 sa0 = *reinterpret_cast<const f32x4*>(a.sasw + c0), sa1 = *reinterpret_cast<const f32x4*>(a.sasw + c0 + 4);
  const f32x4 bb0 = *reinterpret_cast<const f32x4*>(a.bias + c0), bb1 = *reinterpret_cast<const f32x4*>(a.bias + c0 + 4);
  const float sav[8] = {sa0[0], sa0[1], sa0[2], sa0[3], sa1[0], sa1[1], sa1[2], sa1[3]};
  const float bbv[8] = {bb0[0], bb0[1], bb0[2], bb0[3], bb1[0], bb1[1], bb1[2], bb1[3]};
  V o;
  if constexpr (F8) {
    double acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.0;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if (ok[t]) {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fma((double)f8_dec(v[t][e]), (double)f8_dec(w[t][e]), acc[e]);
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (i8)QS::store(post[QS::code((float)acc[e], 0, sav[e], bbv[e], Q)], Q);
  } else {
    int acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if (ok[t]) {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += ((int)v[t][e] + 128 - zi) * (int)w[t][e];
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (i8)QS::store(post[QS::code(acc[e], 0, sav[e], bbv[e], Q)], Q);
  }
  Vec8<i8>::store(static_cast<i8*>(a.dst) + (size_t)(b * a.d_P + p) * a.d_ctot + a.d_coff + c0, o);
}

// ------------------------------------------------------------------------------------------------- attention
// C2PSA Attention on the int8 qkv tensor (stored in the qkv conv's own output quantisation): q, k, v dequantised to
// fp32 ((q - z)·s), then S = q·kᵀ·scale, softmax and O = P·V evaluated in float64 and rounded to fp32 once (the
// oracle's definition of the int8 model's float island, oracle/quant.py:_psablock: f64 results agree far below one
// fp32 ulp whatever the summation order, so the int8 outputs are bit-reproducible); + pe(v) as a quantized depthwise
// conv (int MACs on the stored v bytes, requantised, dequantised); the sum is quantized into attn.x.
//
// One workgroup = 16 queries of one (image, head); its 4 waves each take every 4th 16-key block and run a flash-style
// pass on v_mfma_f64_16x16x4_f64 (A/B one f64 per lane: A[l&15][k=l>>4], B[k=l>>4][l&15]; D col l&15, row
// (l>>4)+4r): Sᵀ = K·Qᵀ (8 MFMAs over kd = 32), running max / sum per query column, and Oᵀ += Vᵀ·Pᵀ (4 d-blocks x 4
// MFMAs) — the Pᵀ operand of key step s is exactly D register r = s of Sᵀ, so P never leaves registers.  The four
// partial (max, sum, Oᵀ) meet in LDS.
constexpr int AKD = 32, AHD = 64;
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <bool F8>
__global__ __launch_bounds__(256) void attn_psa_i8(const AttnArgs a) {
  typedef Q8<F8> QS;
  __shared__ float post[256];
  __shared__ double cm[4][16], cl[4][16];
  __shared__ double co[4][AHD][17];  // Oᵀ partials [wave][d][q] (odd pitch: the column reads below)
  const QRec* Qr = a.q;
  post[threadIdx.x] = Qr->post[threadIdx.x];
  const int N = a.N, nqb = (N + 15) >> 4, nkb = nqb;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // the query blocks of one (image, head) on one XCD
  const int qb = vb % nqb, bh = vb / nqb;
  const int h = bh % a.nh, b = bh / a.nh;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lc = lane & 15, lg = lane >> 4;
  const i8* qkv = static_cast<const i8*>(a.qkv);
  const size_t img = (size_t)b * a.q_P;
  const int hq = a.q_coff + h * (2 * AKD + AHD);
  const float s_in = Qr->s_in;
  const int z_in = Qr->z_in;
  const double scale = (double)a.scale;
  auto dq = [&](unsigned word, int byte) {  // stored byte of a little-endian word -> f64 of its dequantised value
    return (double)QS::dec((int)(word >> (8 * byte)), z_in, s_in);
  };
  // Qᵀ operand: Qᵀ[c = 4s + lg][q = lc]
  double qf[8];
  {
    const int qn = qb * 16 + lc;
    const i32x4* qp = reinterpret_cast<const i32x4*>(qkv + (img + (qn < N ? qn : 0)) * a.q_ctot + hq);
    const i32x4 u0 = qp[0], u1 = qp[1];
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = qn < N ? dq((unsigned)(s < 4 ? u0[s] : u1[s - 4]), lg) : 0.0;
  }
  double m = -INFINITY, l = 0.0;
  f64x4 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f64x4{0.0, 0.0, 0.0, 0.0};
  // the K row and V words of key block kb, one block ahead (each block's loads would otherwise be a full L2 round
  // trip on the wave's serial path)
  auto fetch = [&](int kb, i32x4& k0, i32x4& k1, unsigned (&vw)[4][4]) {
    // Sᵀ = K·Qᵀ: A = K[key = 16 kb + lc][c = 4s + lg]
    const int key = kb * 16 + lc;
    const i32x4* kp = reinterpret_cast<const i32x4*>(qkv + (img + (key < N ? key : 0)) * a.q_ctot + hq + AKD);
    k0 = kp[0];
    k1 = kp[1];
    // Vᵀ operand words: V[16 kb + 4s + lg][16 db + lc] is byte lc & 3 of word (lc >> 2) + 4 db of that key's v row
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int vk = kb * 16 + 4 * s + lg;
      const unsigned* vp = reinterpret_cast<const unsigned*>(qkv + (img + (vk < N ? vk : 0)) * a.q_ctot + hq + 2 * AKD);
#pragma unroll
      for (int db = 0; db < 4; ++db) vw[s][db] = vp[(lc >> 2) + 4 * db];
    }
  };
  i32x4 k0, k1, nk0, nk1;
  unsigned vw[4][4], nvw[4][4];
  if (w < nkb) fetch(w, k0, k1, vw);
  for (int kb = w; kb < nkb; kb += 4) {
    if (kb + 4 < nkb) fetch(kb + 4, nk0, nk1, nvw);
    const int key = kb * 16 + lc;
    f64x4 st = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 8; ++s)
      st = __builtin_amdgcn_mfma_f64_16x16x4f64(key < N ? dq((unsigned)(s < 4 ? k0[s] : k1[s - 4]), lg) : 0.0, qf[s],
                                                st, 0, 0, 0);
    double sv[4], mb = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // row = key 16 kb + lg + 4 r, column = query lc
      sv[r] = kb * 16 + lg + 4 * r < N ? st[r] * scale : -INFINITY;
      mb = fmax(mb, sv[r]);
    }
    mb = fmax(mb, __shfl_xor(mb, 16));
    mb = fmax(mb, __shfl_xor(mb, 32));
    const double mn = fmax(m, mb);
    const double alpha = exp(m - mn);  // m = -inf on the first block: 0
    double p[4], ps = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = exp(sv[r] - mn);
      ps += p[r];
    }
    ps += __shfl_xor(ps, 16);
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      o[db] *= alpha;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        o[db] = __builtin_amdgcn_mfma_f64_16x16x4f64(dq(vw[s][db], lc & 3), p[s], o[db], 0, 0, 0);
    }
    k0 = nk0;
    k1 = nk1;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int db = 0; db < 4; ++db) vw[s][db] = nvw[s][db];
  }
  if (lg == 0) {
    cm[w][lc] = m;
    cl[w][lc] = l;
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) co[w][16 * db + lg + 4 * r][lc] = o[db][r];
  __syncthreads();

  // combine the four partials; + pe(v); quantize into attn.x
  const int q = tid & 15, n = qb * 16 + q;
  if (n >= N) return;
  double M = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i) M = fmax(M, cm[i][q]);
  double f[4], L = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = exp(cm[i][q] - M);  // a wave without keys: exp(-inf) = 0
    L += cl[i][q] * f[i];
  }
  // thread = (query q, 4 consecutive channels 4 dg .. 4 dg + 3): pe's 3x3 taps are 9 dword loads of v bytes and 9 of
  // weight bytes, all issued before any arithmetic (borders: clamped address, zero weight)
  const int y = n / a.W, x = n - y * a.W;
  const int dg = tid >> 4, ch0 = h * AHD + 4 * dg;
  const i8* vimg = qkv + img * a.q_ctot + hq + 2 * AKD + 4 * dg;
  unsigned vt[9], wt[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
    const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    vt[t] = *reinterpret_cast<const unsigned*>(vimg + (size_t)(ok ? iy * a.W + ix : n) * a.q_ctot);
    wt[t] = ok ? *reinterpret_cast<const unsigned*>(a.pe_wq + t * a.C + ch0) : 0u;
  }
  const f32x4 sa4 = *reinterpret_cast<const f32x4*>(a.pe_sasw + ch0), pb4 = *reinterpret_cast<const f32x4*>(a.pe_b + ch0);
  int ov[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int d = 4 * dg + e;
    double od = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) od += co[i][d][q] * f[i];
    int qc;
    if constexpr (F8) {  // pe on e4m3 values: float64 sum of exact products, one rounding (as dwconv3x3_i8)
      double acc = 0.0;
#pragma unroll
      for (int t = 0; t < 9; ++t)
        acc = fma((double)f8_dec((int)(vt[t] >> (8 * e))), (double)f8_dec((int)(wt[t] >> (8 * e))), acc);
      qc = QS::code((float)acc, 0, sa4[e], pb4[e], Qr);
    } else {
      int acc = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t)
        acc += (((int)((vt[t] >> (8 * e)) & 0xFFu) ^ 0x80) - z_in) * (int)(signed char)(wt[t] >> (8 * e));
      qc = QS::code(acc, 0, sa4[e], pb4[e], Qr);
    }
    ov[e] = QS::store(__fadd_rn((float)(od / L), post[qc]), Qr);
  }
  *reinterpret_cast<int*>(static_cast<i8*>(a.dst) + ((size_t)b * a.d_P + n) * a.d_ctot + a.d_coff + ch0) = pack4(ov);
}

// ------------------------------------------------------------------------------------------------- requant
// dst[p, coff + c] = quantize(dequantize(src[p' , c])) with p' = p or (y/2, x/2): 16 channels per thread.
template <bool F8>
__global__ __launch_bounds__(256) void requant_copy(const ReqArgs a) {
  typedef Q8<F8> QS;
  const int C16 = a.C >> 4;
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)a.B * a.H * a.W * C16;
  if (idx >= total) return;
  const int cg = idx % C16;
  const long pix = idx / C16;
  const int HW = a.H * a.W;
  const int b = pix / HW;
  const int p = pix - (long)b * HW;
  const int y = p / a.W, x = p - (p / a.W) * a.W;
  const int sy = a.up ? (y >> 1) : y, sx = a.up ? (x >> 1) : x;
  const QRec* Q = a.q;
  const i8x16 v = ld16(a.src + (size_t)(b * a.s_P + sy * a.s_W + sx) * a.s_ctot + a.s_coff + cg * 16);
  int ov[16];
#pragma unroll
  for (int e = 0; e < 16; ++e)
    ov[e] = QS::store(QS::dec(v[e], Q->z_in, Q->s_in), Q);
  const i32x4 o{pack4(ov), pack4(ov + 4), pack4(ov + 8), pack4(ov + 12)};
  *reinterpret_cast<i32x4*>(a.dst + (size_t)(b * a.d_P + p) * a.d_ctot + a.d_coff + cg * 16) = o;
}

}  // namespace

// ids [0, kNumCfg): conv_i8 above; then the streaming / small-M int8 kernels (csrc/ym_conv_i8_stream.hip)
int ym_conv_i8_num_cfgs() { return kNumCfg + ym_conv_i8_stream_num_cfgs(); }

// fp8 plans: one K chain per output (WK = 1), so the oracle's restated fp8 MFMA accumulation (oracle/quant.py
// mfma_f8_conv) follows the kernel's order; the heuristic's choice among those configurations
int choose_cfg_f8(const ConvArgs& a) {
  const long M = a.M, N = a.N;
  auto waves = [&](int id) {
    const Cfg& c = kCfgs[id];
    const long BM = c.wm * c.wtm * 32, BN = c.wn * c.wtn * 32;
    return ((M + BM - 1) / BM) * ((N + BN - 1) / BN) * c.wm * c.wn;
  };
  if (N <= 32) return waves(2) >= 1024 ? 2 : 9;
  if (N <= 64) return waves(1) >= 1024 ? 1 : (waves(5) >= 1024 ? 5 : 9);
  return waves(0) >= 1024 ? 0 : 10;
}

hipError_t ym_launch_conv_i8(const ConvArgs& a, int cfg, hipStream_t st, bool strict, bool f8) {
  int kind;
  if (a.k == 1 && a.s == 1 && !a.src1 && !a.up0) kind = 1;
  else if (a.k == 3 && !a.src1 && !a.up0) kind = 3;
  else return hipErrorInvalidValue;
  if (a.Kpad % KSTEP || !a.q || !a.sasw || !a.biasi || (a.N & 3) || (a.s0_ctot & 15) || (a.s0_coff & 15))
    return hipErrorInvalidValue;
  if (f8 && (cfg >= kNumCfg || (cfg >= 0 && kCfgs[cfg].wk != 1))) {  // fp8: conv_i8 with one K chain only
    if (strict) return hipErrorInvalidValue;
    cfg = -1;
  }
  if (!f8 && cfg >= ym_conv_i8_num_cfgs()) {  // int8: the LDS-DMA kernel's Q8 mode (csrc/ym_conv_dma.hip)
    const hipError_t e = ym_launch_conv_dma_i8(a, cfg - ym_conv_i8_num_cfgs(), st);
    if (e != hipErrorInvalidValue || strict) return e;
    cfg = -1;
  }
  if (cfg >= kNumCfg) {
    const hipError_t e = ym_launch_conv_i8_stream(a, cfg - kNumCfg, st, f8);
    if (e != hipErrorInvalidValue || strict) return e;
    cfg = -1;  // a pinned table entry that does not apply: the heuristic
  }
  return launch_id(cfg >= 0 ? cfg : (f8 ? choose_cfg_f8(a) : choose_cfg(a)), a, kind, st, f8);
}

hipError_t ym_launch_dwconv_i8(const DwArgs& a, hipStream_t st, bool f8) {
  if (a.C % 8 || !a.q || !a.wq) return hipErrorInvalidValue;
  const long total = (long)a.B * a.H * a.W * (a.C / 8);
  if (total >= 0x7FFFFFFFL - 256) return hipErrorInvalidValue;  // the kernel indexes in 32 bits
  if (f8) hipLaunchKernelGGL(dwconv3x3_i8<true>, dim3((total + 255) / 256), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(dwconv3x3_i8<false>, dim3((total + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_attn_i8(const AttnArgs& a, hipStream_t st, bool f8) {
  // the f64 MFMA kernel's fixed head geometry (YOLO11 C2PSA: head_dim 64, key_dim 32) and 16-byte q/k rows
  if (a.kd != AKD || a.hd != AHD || !a.q || !a.pe_wq || (a.q_ctot & 15) || (a.q_coff & 15) || a.N < 1 ||
      (a.d_ctot & 3) || (a.d_coff & 3) || (a.C & 3))
    return hipErrorInvalidValue;
  const dim3 grid(a.B * a.nh * ((a.N + 15) / 16));
  if (f8) hipLaunchKernelGGL(attn_psa_i8<true>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_psa_i8<false>, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_requant(const ReqArgs& a, hipStream_t st, bool f8) {
  if (a.C % 16 || a.s_coff % 16 || a.d_coff % 16 || a.s_ctot % 16 || a.d_ctot % 16 || !a.q) return hipErrorInvalidValue;
  const long total = (long)a.B * a.H * a.W * (a.C / 16);
  if (f8) hipLaunchKernelGGL(requant_copy<true>, dim3((total + 255) / 256), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(requant_copy<false>, dim3((total + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}
