// Streaming 1x1 / 3x3 conv for the large-M, small-K/N layers (f16 plans) — the HBM-bound half of the Conv launches
// (C3k2 cv1/cv2 and Bottleneck 3x3s at 160² and 80², the stride-2 downsamples, the FPN merges of the neck, the P3
// Detect-head convs).
//
// The first-generation and LDS-DMA kernels (csrc/ym_conv.hip, ym_conv_dma.hip) give each wave one small output tile
// and retire: on these layers a wave does a few MFMAs between a prologue (tile coordinates, weight rows, bias) and
// an epilogue, and its lifetime is one memory round trip.  Here a persistent grid of waves streams over the pixels:
//   * the whole weight matrix [N][Kpad] (<= 80 KB) is staged in LDS once per workgroup, rows padded by 16 bytes so
//     the MFMA A-fragment reads (ds_read_b128, 16 rows at one K offset) spread over the banks; bias in LDS too;
//   * a wave takes PX groups of 16 consecutive pixels per iteration; their B fragments (one 16-byte load = 8
//     channels of one pixel per lane; 1x1: concat sources and the nearest-2x upsample folded into the row address,
//     3x3: the im2col gather of tap (ky, kx) straight from NHWC, zero padding by predicate) for the NEXT iteration
//     are in flight while the current one computes — two iterations of loads per wave in flight;
//   * v_mfma_f32_16x16x32_f16 in the transposed orientation (A = weights): a lane ends with 4 consecutive output
//     channels of one pixel → + bias, SiLU, (+ residual), one 8-byte (fp16) or 16-byte (fp32 head buffer) store.
// Results are identical in kind to the other conv kernels (fp32 accumulation of fp16 products, one rounding to the
// output type); only the summation order differs.
#include <type_traits>

#include "ym_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

struct SCfg {
  int kind, ks, px, cap, nw;  // kind 1 = 1x1 s1, 3 = 3x3; K steps of 32 (Kpad / 32); 16-pixel groups per wave
};                            // iteration; workgroup cap of the persistent grid; waves per workgroup
// nw 8: two waves per SIMD share one LDS copy of the weights — for the matrices too large for two workgroups per CU
// (N 256 x K 192: 106 KB), where one wave per SIMD leaves the SIMD idle while that wave waits for its next pixels
#define YM_STREAM_CFGS(X)                                                                                          \
  X(0, 1, 2, 1, 1024, 4) X(1, 1, 2, 2, 1024, 4) X(2, 1, 2, 1, 4096, 4) X(3, 1, 4, 1, 1024, 4)                      \
  X(4, 1, 4, 2, 1024, 4) X(5, 1, 8, 1, 1024, 4) X(6, 1, 4, 1, 4096, 4) X(7, 3, 4, 1, 1024, 4)                      \
  X(8, 3, 6, 1, 1024, 4) X(9, 3, 10, 1, 1024, 4) X(10, 3, 18, 1, 1024, 4) X(11, 3, 4, 1, 4096, 4)                  \
  X(12, 3, 6, 1, 4096, 4) X(13, 3, 10, 1, 4096, 4) X(14, 3, 18, 1, 4096, 4) X(15, 1, 2, 2, 4096, 4)                \
  X(16, 1, 2, 4, 4096, 4) X(17, 1, 4, 2, 4096, 4) X(18, 3, 4, 2, 4096, 4) X(19, 3, 6, 2, 4096, 4)                  \
  X(20, 1, 6, 1, 4096, 4) X(21, 1, 6, 2, 4096, 4) X(22, 1, 6, 1, 1024, 4) X(23, 1, 4, 1, 4096, 8)                  \
  X(24, 1, 4, 2, 4096, 8) X(25, 1, 6, 1, 4096, 8) X(26, 1, 6, 2, 4096, 8) X(27, 1, 8, 1, 4096, 8)                  \
  X(28, 1, 2, 2, 4096, 8) X(29, 3, 10, 1, 4096, 8) X(30, 3, 4, 2, 4096, 8)
constexpr SCfg kStream[] = {
#define YM_X(id, kind, ks, px, cap, nw) {kind, ks, px, cap, nw},
    YM_STREAM_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumStream = sizeof(kStream) / sizeof(kStream[0]);
constexpr int kMaxWBytes = 144 * 1024;  // whole weight matrix in LDS (one workgroup per CU above ~75 KB: the KS 6 configs)
constexpr int kMaxFusedBytes = 112 * 1024;  // fused pairs: both weight matrices

// FUSE: the fused pair (ConvArgs::w2) — the first conv's activated output block nb (16 channels x 16 pixels, lane
// (g, col) holding channels 16 nb + 4 g .. + 3 of pixel col) is exactly the B operand of a 16x16x16 MFMA with K chunk
// nb, so the following 1x1 conv runs from registers: no LDS round trip, no HBM write/read of the intermediate, one
// launch fewer.  The intermediate is rounded to fp16 like the stored tensor of the unfused pair.
constexpr int kFuseMaxN = 128;  // first conv's N (= second conv's K) held in registers: 8 blocks of 16
constexpr int RB = 8;           // output-channel blocks of 16 whose residuals are prefetched with the fragments

// x3 plans (X3): activations in the pair layout, weights in pair-chunk rows (csrc/ym_common.h), both read as fp16
// tensors of twice the channels; a K step ks of 32 then holds the hi / lo halves of logical chunks 2ks, 2ks+1 (lane
// group g: storage chunk 4ks + g).  Per two steps three MFMAs form the split product: A = w_hi of the group's own
// logical chunk (storage chunk 4ks + 2(g>>1)) with the natural B, for ks and ks+1 (w_hi·x_hi + w_hi·x_lo), and
// A = w_lo of logical chunk 2ks + g (storage 4ks + 2g + 1) with B = x_hi of that chunk (storage 4ks + 2g, one extra
// 16-byte gather per lane and step pair) — w_lo·x_hi of all four chunks.
// x3 fused pairs: the first conv's activated fp32 output is split in registers exactly as its producer epilogue
// would store it (hi = fp16(v), lo = fp16(v - hi)), and the second GEMM runs three 16x16x16 MFMAs per K block
// (w2_lo·h_hi, w2_hi·h_lo, w2_hi·h_hi) with W2's hi and lo halves in two LDS planes: the same products as the unfused
// x3 pair, summed in another order.
template <typename T> struct SOut;  // 4 output channels of one pixel
template <> struct SOut<f16> {
  static __device__ __forceinline__ void st(f16* o, const float* v) {
    *reinterpret_cast<f16x4*>(o) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
  }
};
template <> struct SOut<float> {
  static __device__ __forceinline__ void st(float* o, const float* v) {
    *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
  }
};
template <> struct SOut<P2> {
  static __device__ __forceinline__ void st(P2* o, const float* v) { ym_p2_store4(o, v); }
};
// residual values of 4 channels (x3: hi + lo)
template <bool X3> struct SRes {
  typedef f16x4 type;
  static __device__ __forceinline__ type load(const void* p) { return *reinterpret_cast<const f16x4*>(p); }
  static __device__ __forceinline__ type zero() { return f16x4{0, 0, 0, 0}; }
};
template <> struct SRes<true> {
  typedef f32x4 type;
  static __device__ __forceinline__ type load(const void* p) {
    float v[4];
    ym_p2_load4(static_cast<const P2*>(p), v);
    return f32x4{v[0], v[1], v[2], v[3]};
  }
  static __device__ __forceinline__ type zero() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
};

template <typename OutT, int KIND, int KS, int PX, bool FUSE, int NWV, bool X3 = false>
__global__ __launch_bounds__(64 * NWV) void conv_stream(const ConvArgs a) {
  ym_warm_kernargs<sizeof(ConvArgs)>();  // one round trip for the whole argument block (ym_common.h)
  static_assert(!X3 || KS % 2 == 0, "x3: K steps in pairs");
  constexpr int XS = X3 ? 2 : 1;       // fp16 storage elements per logical channel
  constexpr int KX = X3 ? KS / 2 : 0;  // x3: the extra x_hi gather per step pair
  typedef typename SRes<X3>::type RV;
  constexpr int NT = 64 * NWV;     // threads per workgroup
  constexpr int KP = KS * 32;      // Kpad
  // LDS row pitch (halves) KP + 16 = 4·KS + 2 16-byte slots: the A-fragment reads (16 rows x one K chunk per lane
  // group kg) hit distinct slots in each of ds_read_b128's non-contiguous lane groups (MI355X_MICROARCH §LDS);
  // a +8 pitch is 2-way there
  constexpr int LDW = KP + 16;
  constexpr int NBF = FUSE ? kFuseMaxN / 16 : 1;
  extern __shared__ __attribute__((aligned(16))) f16 ws[];  // [N][LDW], then bias [N] f32 (FUSE: then W2, bias2)
  float* bs = reinterpret_cast<float*>(ws + ((a.N + 15) & ~15) * LDW);
  const int NB = (a.N + 15) >> 4;
  const int LDW2 = 16 * NB + 8;  // W2 row pitch (halves): the 8-byte A reads of 16 rows x 2 lane groups hit 32
                                 // distinct 8-byte slots of a ds_read_b64 half-wave (+4 was 2-way)
  f16* w2s = reinterpret_cast<f16*>(bs + 16 * NB);
  const int NB2 = FUSE ? (a.N2 + 15) >> 4 : 0;
  f16* w2l = w2s + (X3 ? 16 * NB2 * LDW2 : 0);  // x3: the lo plane of W2
  float* bs2 = reinterpret_cast<float*>(w2l + 16 * NB2 * LDW2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const f16* W = static_cast<const f16*>(a.w);
  const int NP = (a.N + 15) & ~15;  // rows padded to the 16-row MFMA block (zero weights, outputs not stored)
  for (int i0 = tid; i0 < NP * (KP / 8); i0 += NT * 8) {  // 8 loads in flight per thread and round
    f16x8 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + NT * u, n = i / (KP / 8), c = i - n * (KP / 8);
      v[u] = (i < NP * (KP / 8) && n < a.N) ? *reinterpret_cast<const f16x8*>(W + (size_t)n * KP + 8 * c)
                                             : Vec8<f16>::zero();
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + NT * u, n = i / (KP / 8), c = i - n * (KP / 8);
      if (i < NP * (KP / 8)) *reinterpret_cast<f16x8*>(ws + n * LDW + 8 * c) = v[u];
    }
  }
  for (int i = tid; i < NP; i += NT) bs[i] = i < a.N ? a.bias[i] : 0.f;
  if constexpr (FUSE) {  // W2 [16 NB2][LDW2]: row n2, K = first-conv channel (zero past N / N2)
    const f16* W2 = static_cast<const f16*>(a.w2);
    const int q4 = 4 * NB;  // 4-channel quads per row
    for (int i = tid; i < 16 * NB2 * q4; i += NT) {
      const int n = i / q4, c = 4 * (i - n * q4);
      f16x4 v = {0, 0, 0, 0}, vl = {0, 0, 0, 0};
      if (n < a.N2 && c < a.N) {
        if constexpr (X3) {  // pair-chunk row: logical channel c's hi half at 2 (c & ~7) + (c & 7), its lo 8 further
          const f16* q = W2 + (size_t)n * a.Kpad2 + 2 * (c & ~7) + (c & 7);
          v = *reinterpret_cast<const f16x4*>(q);
          vl = *reinterpret_cast<const f16x4*>(q + 8);
        } else {
          v = *reinterpret_cast<const f16x4*>(W2 + (size_t)n * a.Kpad2 + c);
        }
      }
      *reinterpret_cast<f16x4*>(w2s + n * LDW2 + c) = v;
      if constexpr (X3) *reinterpret_cast<f16x4*>(w2l + n * LDW2 + c) = vl;
    }
    for (int i = tid; i < 16 * NB2; i += NT) bs2[i] = i < a.N2 ? a.bias2[i] : 0.f;
  }

  const int HW = a.Ho * a.Wo;
  const int G = (a.M + 15) >> 4;  // 16-pixel groups
  const f16* s0 = static_cast<const f16*>(a.src0);
  const f16* s1 = static_cast<const f16*>(a.src1);
  const int s0_ctot = XS * a.s0_ctot, s0_coff = XS * a.s0_coff, s1_ctot = XS * a.s1_ctot, s1_coff = XS * a.s1_coff;
  const int C0s = XS * a.C0;
  const int K = XS * (a.C0 + a.C1);  // storage K of one pixel row (1x1)
  const unsigned c8m = (0x1000000u + a.Cin8 - 1) / a.Cin8;  // 3x3: tap = (chunk * c8m) >> 24 (chunk < 9 Cin8)

  // B fragments of the iteration starting at group gb: [PX][KS]; with a residual also the residual values of the
  // first RB output-channel blocks of its pixels, one iteration ahead like the fragments (a residual load placed
  // after the previous block's stores would make the compiler drain every outstanding load, the prefetch included)
  const f16* res = static_cast<const f16*>(a.res);
  const P2* resp = static_cast<const P2*>(a.res);
  auto res_at = [&](size_t e) -> const void* {  // residual element e (logical index)
    if constexpr (X3) return resp + e;
    else return res + e;
  };
  const int NR = FUSE ? a.N2 : a.N;
  // XCD-contiguous group ranges: workgroup bid runs on XCD bid % 8 (round-robin dispatch), and each XCD sweeps one
  // contiguous range of 16-pixel groups with all of its workgroups, so the neighbouring image rows a 3x3 tap reads
  // (and a C2f residual) are fetched into that XCD's L2 once instead of once per XCD (speed only: any mapping gives
  // the same results)
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nwx = (nwg >> 3) + (xcd < (nwg & 7));                   // workgroups on this XCD
  const int v0 = xcd * (nwg >> 3) + (xcd < (nwg & 7) ? xcd : (nwg & 7));  // workgroups on lower XCDs
  const int gend = (int)((long)G * (v0 + nwx) / nwg);
  auto load = [&](int gb, h8 (&bf)[PX][KS + KX], RV (&rr)[PX][RB]) {
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int m = (gb + p) * 16 + col;
      const bool ok = gb + p < gend && m < a.M;
      const int mm = ok ? m : 0;
      const int b = ym_div(mm, a.fd_hw), rem = mm - b * HW;
      const int y = ym_div(rem, a.fd_w), x = rem - y * a.Wo;
      if (res) {
        const size_t rp = (size_t)(b * a.r_P + y * a.Wo + x) * a.r_ctot + a.r_coff + 4 * g;
#pragma unroll
        for (int j = 0; j < RB; ++j)
          rr[p][j] = (ok && 16 * j + 4 * g < NR) ? SRes<X3>::load(res_at(rp + 16 * j)) : SRes<X3>::zero();
      }
      if constexpr (KIND == 1) {
        const size_t p0 = a.up0 ? (size_t)b * a.s0_P + (y >> 1) * a.s0_W + (x >> 1) : (size_t)b * a.s0_P + y * a.s0_W + x;
        const size_t p1 = (size_t)b * a.s1_P + y * a.Win + x;
#pragma unroll
        for (int ks = 0; ks < KS + KX; ++ks) {
          // ks >= KS (x3): x_hi of logical chunk 4 (ks - KS) + g, i.e. storage chunk 8 (ks - KS) + 2g
          const int k0 = ks < KS ? 32 * ks + 8 * g : 64 * (ks - KS) + 16 * g;
          h8 v = Vec8<f16>::zero();
          if (ok && k0 < K)
            v = k0 < C0s ? Vec8<f16>::load(s0 + p0 * s0_ctot + s0_coff + k0)
                         : Vec8<f16>::load(s1 + p1 * s1_ctot + s1_coff + (k0 - C0s));
          bf[p][ks] = v;
        }
      } else {  // 3x3, pad 1, stride a.s: chunk c = 4 ks + g is tap c / Cin8, channels 8 (c % Cin8) ..
        const f16* img = s0 + (size_t)b * a.s0_P * s0_ctot + s0_coff;
        const int iy0 = y * a.s - 1, ix0 = x * a.s - 1;
#pragma unroll
        for (int ks = 0; ks < KS + KX; ++ks) {
          const int c = ks < KS ? 4 * ks + g : 8 * (ks - KS) + 2 * g;  // storage chunk (x3 extra: the x_hi chunks)
          const int t = (int)(((unsigned)c * c8m) >> 24), cb = c - t * a.Cin8;
          const int ky = t >= 6 ? 2 : (t >= 3 ? 1 : 0), kx = t - 3 * ky;
          const int iy = iy0 + ky, ix = ix0 + kx;
          h8 v = Vec8<f16>::zero();
          if (ok && c < a.Kc && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win)
            v = Vec8<f16>::load(img + (size_t)(iy * a.Win + ix) * s0_ctot + 8 * cb);
          bf[p][ks] = v;
        }
      }
    }
  };

  const int step = nwx * NWV * PX;
  int gb = (int)((long)G * v0 / nwg) + (slot * NWV + wave) * PX;
  h8 cur[PX][KS + KX], nxt[PX][KS + KX];
  RV rcur[PX][RB], rnxt[PX][RB];
  load(gb, cur, rcur);
  __syncthreads();
  OutT* dst = static_cast<OutT*>(a.dst);
  // x3 pair-layout outputs: whole-chunk stores by lane pairs where every 8-channel chunk of the output slice is
  // written by one lane pair (8-aligned slice and channel count; uniform)
  constexpr bool PAIRST = X3 && std::is_same<OutT, P2>::value;
  const bool pair1 = (a.pst & 2) && ((a.N | a.d_coff | a.d_ctot) & 7) == 0;
  const bool pair2 = (a.pst & 2) && ((a.N2 | a.d_coff | a.d_ctot) & 7) == 0;
  for (; gb < gend; gb += step) {
    if (gb + step < gend) load(gb + step, nxt, rnxt);
    int ob[PX], rb[PX];  // output / residual pixel index of this lane's pixel in group p (ob -1: none)
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int m = (gb + p) * 16 + col;
      const int b = ym_div(m, a.fd_hw), rem = m - b * HW;
      const int y = ym_div(rem, a.fd_w), x = rem - y * a.Wo;
      ob[p] = (gb + p < gend && m < a.M) ? b * a.d_P + a.d_pixoff + y * a.d_W + x : -1;
      rb[p] = b * a.r_P + y * a.Wo + x;
    }
    if constexpr (FUSE) {
      f16x4 h[PX][NBF];  // the first conv's activated output, fp16, in registers (x3: its hi half)
      f16x4 hl[X3 ? PX : 1][X3 ? NBF : 1];  // x3: the lo half
#pragma unroll
      for (int nb = 0; nb < NBF; ++nb) {
        if (nb >= NB) break;
        h8 af[KS + KX];
#pragma unroll
        for (int ks = 0; ks < KS + KX; ++ks) {
          const int c = !X3 ? 4 * ks + g : (ks < KS ? 4 * ks + 2 * (g >> 1) : 8 * (ks - KS) + 2 * g + 1);
          af[ks] = *reinterpret_cast<const h8*>(ws + (16 * nb + col) * LDW + 8 * c);
        }
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bs + 16 * nb + 4 * g);
#pragma unroll
        for (int p = 0; p < PX; ++p) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < KS + KX; ++ks)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ks], cur[p][ks], acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xv = X3 ? ym_x3_pre(acc[r], a.wsc, b4[r]) : acc[r] + b4[r];
            if constexpr (X3) {
              const float v = a.act ? ym_silu_x3(xv) : xv;
              const f16 hi = (f16)v;
              h[p][nb][r] = hi;
              hl[p][nb][r] = (f16)(v - (float)hi);
            } else {
              h[p][nb][r] = (f16)(a.act ? ym_silu_fast(xv) : xv);
            }
          }
        }
      }
      for (int nb20 = 0; nb20 < NB2; nb20 += RB)
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int nb2 = nb20 + j;
        if (nb2 >= NB2) break;
        f16x4 a2[NBF], a2l[X3 ? NBF : 1];
#pragma unroll
        for (int nb = 0; nb < NBF; ++nb)
          if (nb < NB) {
            a2[nb] = *reinterpret_cast<const f16x4*>(w2s + (16 * nb2 + col) * LDW2 + 16 * nb + 4 * g);
            if constexpr (X3) a2l[nb] = *reinterpret_cast<const f16x4*>(w2l + (16 * nb2 + col) * LDW2 + 16 * nb + 4 * g);
          }
        const int n0 = 16 * nb2 + 4 * g;
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bs2 + n0);
#pragma unroll
        for (int p = 0; p < PX; ++p) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int nb = 0; nb < NBF; ++nb)
            if (nb < NB) {
              if constexpr (X3) {
                acc = __builtin_amdgcn_mfma_f32_16x16x16f16(a2l[nb], h[p][nb], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x16f16(a2[nb], hl[p][nb], acc, 0, 0, 0);
              }
              acc = __builtin_amdgcn_mfma_f32_16x16x16f16(a2[nb], h[p][nb], acc, 0, 0, 0);
            }
          if constexpr (PAIRST) {
            if (pair2) {  // lane pair (g, g ^ 1) of one pixel writes whole 32-byte chunks
              const bool okp = ob[p] >= 0 && n0 < a.N2;
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float xv = ym_x3_pre(acc[r], a.wsc2, b4[r]);
                v[r] = a.act2 ? ym_silu_x3(xv) : xv;
              }
              if (res && okp) {
                const RV rv = nb20 == 0 ? rcur[p][j] : SRes<X3>::load(res_at((size_t)rb[p] * a.r_ctot + a.r_coff + n0));
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
              }
              ym_p2_store4_pair<16>(dst + (size_t)(okp ? ob[p] : 0) * a.d_ctot + a.d_coff + n0, v, g & 1, okp, a.pst & 16);
              continue;
            }
          }
          if (ob[p] < 0 || n0 >= a.N2) continue;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xv = X3 ? ym_x3_pre(acc[r], a.wsc2, b4[r]) : acc[r] + b4[r];
            v[r] = a.act2 ? (X3 ? ym_silu_x3(xv) : ym_silu_fast(xv)) : xv;
          }
          if (res) {
            const RV rv = nb20 == 0 ? rcur[p][j] : SRes<X3>::load(res_at((size_t)rb[p] * a.r_ctot + a.r_coff + n0));
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
          }
          SOut<OutT>::st(dst + (size_t)ob[p] * a.d_ctot + a.d_coff + n0, v);
        }
      }
    } else
    for (int nb0 = 0; nb0 < NP / 16; nb0 += RB)
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int nb = nb0 + j;
      if (nb >= NP / 16) break;
      h8 af[KS + KX];  // x3: [0, KS) = w_hi of each group's logical chunk, [KS, KS + KX) = w_lo of chunk 4ks' + g
#pragma unroll
      for (int ks = 0; ks < KS + KX; ++ks) {
        const int c = !X3 ? 4 * ks + g : (ks < KS ? 4 * ks + 2 * (g >> 1) : 8 * (ks - KS) + 2 * g + 1);
        af[ks] = *reinterpret_cast<const h8*>(ws + (16 * nb + col) * LDW + 8 * c);
      }
      const int n0 = 16 * nb + 4 * g;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(bs + n0);
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS + KX; ++ks)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ks], cur[p][ks], acc, 0, 0, 0);
        if constexpr (PAIRST) {
          if (pair1) {  // lane pair (g, g ^ 1) of one pixel writes whole 32-byte chunks
            const bool okp = ob[p] >= 0 && n0 < a.N;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float xv = ym_x3_pre(acc[r], a.wsc, b4[r]);
              v[r] = a.act ? ym_silu_x3(xv) : xv;
            }
            if (res && okp) {
              const RV rv = nb0 == 0 ? rcur[p][j] : SRes<X3>::load(res_at((size_t)rb[p] * a.r_ctot + a.r_coff + n0));
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
            }
            ym_p2_store4_pair<16>(dst + (size_t)(okp ? ob[p] : 0) * a.d_ctot + a.d_coff + n0, v, g & 1, okp, a.pst & 16);
            continue;
          }
        }
        if (ob[p] < 0 || n0 >= a.N) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xv = X3 ? ym_x3_pre(acc[r], a.wsc, b4[r]) : acc[r] + b4[r];
          v[r] = a.act ? (X3 ? ym_silu_x3(xv) : ym_silu_fast(xv)) : xv;
        }
        if (res) {
          const RV rv = nb0 == 0 ? rcur[p][j] : SRes<X3>::load(res_at((size_t)rb[p] * a.r_ctot + a.r_coff + n0));
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
        }
        SOut<OutT>::st(dst + (size_t)ob[p] * a.d_ctot + a.d_coff + n0, v);
      }
    }
#pragma unroll
    for (int p = 0; p < PX; ++p) {
#pragma unroll
      for (int ks = 0; ks < KS + KX; ++ks) cur[p][ks] = nxt[p][ks];
#pragma unroll
      for (int j = 0; j < RB; ++j) rcur[p][j] = rnxt[p][j];
    }
  }
}

// ------------------------------------------------------------------------------------------------ small-M convs
// The 20x20 / 40x40 layers (M = B·400 … B·1600 pixels): too few output tiles to fill 256 CUs with whole-K tiles,
// so their time is one tile's dependent memory round trips.  conv_small puts one 16-pixel x 16-channel output
// block (PXG blocks along M) on a 4-wave workgroup that splits K four ways: every wave issues ALL of its A (weight
// rows, 16 B per lane) and B (im2col, 16 B per lane) fragments at once, runs its MFMAs, and the partial blocks meet
// in LDS — one memory latency per launch.  Grid = ceil(M / 16 PXG) x ceil(N / 16) workgroups.
#define YM_SMALL_CFGS(X)                                                                                          \
  X(0, 1, 2, 1) X(1, 1, 4, 1) X(2, 1, 8, 1) X(3, 1, 16, 1) X(4, 1, 2, 2) X(5, 1, 4, 2) X(6, 1, 8, 2)             \
  X(7, 3, 5, 1) X(8, 3, 9, 1) X(9, 3, 18, 1) X(10, 3, 5, 2) X(11, 3, 9, 2)
struct MCfg {
  int kind, ksw, pxg;  // 1x1 / 3x3; max K steps of 32 per wave (Kpad <= 128 KSW); 16-pixel blocks per workgroup
};
constexpr MCfg kSmall[] = {
#define YM_X(id, kind, ksw, pxg) {kind, ksw, pxg},
    YM_SMALL_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumSmall = sizeof(kSmall) / sizeof(kSmall[0]);

template <typename OutT, int KIND, int KSW, int PXG>
__global__ __launch_bounds__(256) void conv_small(const ConvArgs a) {
  ym_warm_kernargs<sizeof(ConvArgs)>();  // one round trip for the whole argument block (ym_common.h)
  __shared__ f32x4 red[3][PXG][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int ntn = (a.N + 15) >> 4;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // each XCD owns one contiguous run of pixel blocks
  const int tn = vb % ntn, tm = vb / ntn;
  const int KS = a.Kpad >> 5;
  const int HW = a.Ho * a.Wo;
  const f16* s0 = static_cast<const f16*>(a.src0);
  const f16* s1 = static_cast<const f16*>(a.src1);
  const int K = a.C0 + a.C1;
  const unsigned c8m = (0x1000000u + a.Cin8 - 1) / a.Cin8;
  const int nrow = 16 * tn + col;
  const f16* wr = static_cast<const f16*>(a.w) + (size_t)(nrow < a.N ? nrow : 0) * a.Kpad + 8 * g;
  h8 af[KSW];
#pragma unroll
  for (int j = 0; j < KSW; ++j) {
    const int ks = wave + 4 * j;
    af[j] = (ks < KS && nrow < a.N) ? Vec8<f16>::load(wr + 32 * ks) : Vec8<f16>::zero();
  }
  // the epilogue's bias, fetched with the operands (4-aligned n0 < N: in range; clamped otherwise)
  const int nb4 = 16 * tn + 4 * g < a.N ? 16 * tn + 4 * g : 0;
  const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bias + nb4);
  h8 bf[PXG][KSW];
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
    if constexpr (KIND == 1) {
      const size_t p0 = a.up0 ? (size_t)b[p] * a.s0_P + (y[p] >> 1) * a.s0_W + (x[p] >> 1)
                              : (size_t)b[p] * a.s0_P + y[p] * a.s0_W + x[p];
      const size_t p1 = (size_t)b[p] * a.s1_P + y[p] * a.Win + x[p];
#pragma unroll
      for (int j = 0; j < KSW; ++j) {
        const int k0 = 32 * (wave + 4 * j) + 8 * g;
        h8 v = Vec8<f16>::zero();
        if (ok[p] && k0 < K)
          v = k0 < a.C0 ? Vec8<f16>::load(s0 + p0 * a.s0_ctot + a.s0_coff + k0)
                        : Vec8<f16>::load(s1 + p1 * a.s1_ctot + a.s1_coff + (k0 - a.C0));
        bf[p][j] = v;
      }
    } else {
      const f16* img = s0 + (size_t)b[p] * a.s0_P * a.s0_ctot + a.s0_coff;
      const int iy0 = y[p] * a.s - 1, ix0 = x[p] * a.s - 1;
#pragma unroll
      for (int j = 0; j < KSW; ++j) {
        const int c = 4 * (wave + 4 * j) + g;
        const int t = (int)(((unsigned)c * c8m) >> 24), cb = c - t * a.Cin8;
        const int ky = t >= 6 ? 2 : (t >= 3 ? 1 : 0), kx = t - 3 * ky;
        const int iy = iy0 + ky, ix = ix0 + kx;
        h8 v = Vec8<f16>::zero();
        if (ok[p] && c < a.Kc && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win)
          v = Vec8<f16>::load(img + (size_t)(iy * a.Win + ix) * a.s0_ctot + 8 * cb);
        bf[p][j] = v;
      }
    }
  }
  f32x4 acc[PXG];
#pragma unroll
  for (int p = 0; p < PXG; ++p) {
    acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KSW; ++j) acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[j], bf[p][j], acc[p], 0, 0, 0);
    if (wave > 0) red[wave - 1][p][lane] = acc[p];
  }
  __syncthreads();
  if (wave > 0) return;
  const int n0 = 16 * tn + 4 * g;
  if (n0 >= a.N) return;
  OutT* dst = static_cast<OutT*>(a.dst);
  const f16* res = static_cast<const f16*>(a.res);
#pragma unroll
  for (int p = 0; p < PXG; ++p) {
    if (!ok[p]) continue;
    const f32x4 r = acc[p] + red[0][p][lane] + red[1][p][lane] + red[2][p][lane];
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xv = r[e] + b4[e];
      v[e] = a.act ? ym_silu_fast(xv) : xv;
    }
    if (res) {
      const f16x4 rv = *reinterpret_cast<const f16x4*>(
          res + (size_t)(b[p] * a.r_P + y[p] * a.Wo + x[p]) * a.r_ctot + a.r_coff + n0);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += (float)rv[e];
    }
    OutT* o = dst + (size_t)(b[p] * a.d_P + a.d_pixoff + y[p] * a.d_W + x[p]) * a.d_ctot + a.d_coff + n0;
    if constexpr (sizeof(OutT) == 2) *reinterpret_cast<f16x4*>(o) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
    else *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
  }
}

template <typename OutT, int KIND, int KSW, int PXG>
hipError_t launch_small(const ConvArgs& a, hipStream_t st) {
  if (a.w2) return hipErrorInvalidValue;  // one 16-channel block per workgroup: no fused pairs
  if (a.k != KIND || a.Kpad > 128 * KSW) return hipErrorInvalidValue;
  const long wgs = (long)((a.M + 16 * PXG - 1) / (16 * PXG)) * ((a.N + 15) / 16);
  hipLaunchKernelGGL((conv_small<OutT, KIND, KSW, PXG>), dim3(wgs), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <typename OutT, int KIND, int KS, int PX, int CAP, int NWV, bool X3 = false>
hipError_t launch(const ConvArgs& a, hipStream_t st) {
  if (a.Kpad != KS * 32 || a.k != KIND) return hipErrorInvalidValue;
  if constexpr (X3) {
    if (KS % 2) return hipErrorInvalidValue;
  }
  const int G = (a.M + 15) / 16;
  long wgs = (G + NWV * PX - 1) / (NWV * PX);
  if (wgs > CAP) wgs = CAP;  // the persistent grid: CAP workgroups, the rest streams through them
  const int NP = (a.N + 15) & ~15;
  size_t lds = (size_t)NP * (KS * 32 + 16) * sizeof(f16) + (size_t)NP * sizeof(float);
  if (lds > kMaxWBytes) return hipErrorInvalidValue;
  if (a.w2) {  // fused pair: + W2 [N2P][NP + 8] and bias2 (checked by ym_launch_conv_stream: N <= 128)
    const int N2P = (a.N2 + 15) & ~15;
    lds += (size_t)N2P * (NP + 8) * sizeof(f16) * (X3 ? 2 : 1) + (size_t)N2P * sizeof(float);
    if (lds > kMaxFusedBytes) return hipErrorInvalidValue;
    if constexpr (NWV == 8 && PX > 1) return hipErrorInvalidValue;  // 256 VGPRs per wave: the pair would spill
    else hipLaunchKernelGGL((conv_stream<OutT, KIND, KS, PX, true, NWV, X3>), dim3(wgs), dim3(64 * NWV), lds, st, a);
  } else {
    hipLaunchKernelGGL((conv_stream<OutT, KIND, KS, PX, false, NWV, X3>), dim3(wgs), dim3(64 * NWV), lds, st, a);
  }
  return hipGetLastError();
}

template <typename OutT, bool X3 = false>
hipError_t dispatch(const ConvArgs& a, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, kind, ks, px, cap, nw) \
  case id: return launch<OutT, kind, ks, px, cap, nw, X3>(a, st);
    YM_STREAM_CFGS(YM_X)
#undef YM_X
  }
  if constexpr (X3) return hipErrorInvalidValue;  // the small-M kernels split K four ways: no x3 pairing
  switch (i - kNumStream) {
#define YM_X(id, kind, ksw, pxg) \
  case id: return launch_small<OutT, kind, ksw, pxg>(a, st);
    YM_SMALL_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

}  // namespace

int ym_conv_stream_num_cfgs() { return kNumStream + kNumSmall; }

// Host-side applicability: f16 plans; 1x1 stride-1 convs without pixel shuffle (8-channel-aligned concat split) or
// 3x3 convs on one plain source; N % 4 == 0 and 4-aligned output channel slices
// (8/16-byte stores); weights + bias <= 80 KB of LDS.
hipError_t ym_launch_conv_stream(int out_f32, const ConvArgs& a, int i, hipStream_t st) {
  if (i < 0 || i >= kNumStream + kNumSmall) return hipErrorInvalidValue;
  if (a.shuffle || a.raw || a.nchw || !a.src0 || (a.N & 3) || a.Kpad % 32) return hipErrorInvalidValue;
  if (a.k == 1) {
    if (a.s != 1 || a.C0 % 8 || a.C1 % 8) return hipErrorInvalidValue;  // (logical channels; x3: pair chunks)
    if (a.src1 && (a.s1_coff % 8 || a.s1_ctot % 8)) return hipErrorInvalidValue;
  } else if (a.k == 3) {
    if (a.src1 || a.up0 || a.pad != 1 || a.Cin8 > 1024) return hipErrorInvalidValue;
  } else {
    return hipErrorInvalidValue;
  }
  if ((a.d_ctot & 3) || (a.d_coff & 3) || (a.res && ((a.r_ctot & 3) || (a.r_coff & 3)))) return hipErrorInvalidValue;
  if (a.s0_coff % 8 || a.s0_ctot % 8) return hipErrorInvalidValue;
  if (a.w2 && (a.N > kFuseMaxN || (a.N2 & 3) || a.Kpad2 < (a.x3 ? 2 : 1) * a.N || (a.Kpad2 & 3) || !a.bias2 || a.k2 != 1))
    return hipErrorInvalidValue;
  if (a.x3) return out_f32 ? dispatch<float, true>(a, i, st) : dispatch<P2, true>(a, i, st);
  return out_f32 ? dispatch<float>(a, i, st) : dispatch<f16>(a, i, st);
}
