// Fused YOLO11 Bottleneck for gfx950 (f16 plans): out = x + SiLU(BN2(conv3x3(SiLU(BN1(conv3x3(x)))))) in ONE launch
// (the C3k2 `m` Bottlenecks, reference core/model.py:118-133 -> Ultralytics
// nn/modules/block.py Bottleneck with k=(3,3), shortcut).  Planned by yolomi/arch.py fuse_pairs as a conv pair whose
// successor is a 3x3 (ConvArgs::k2 == 3); the tuner also times the pair as two launches and keeps the faster.
//
// Why: at 160x160 / 80x80 the Bottleneck convs have few channels (C = 16..64 in, C/2 mid), so per output pixel they
// move a few hundred bytes and do little math; the implicit-GEMM families gather every input pixel 9 times per conv
// from L2 and pay two launches plus a round trip of the mid tensor through HBM (yolo11s B=8: 85 us for three
// Bottlenecks whose HBM floor is ~15 us).  Here one workgroup owns a tile of RB output rows x TW columns (whole rows or
// half rows) of one image:
//   phase 0  the band's input rows + a 2-row / 1-column halo (RB+4 rows x TW+2 px x C) are read from HBM ONCE into
//            LDS, W1 and the biases are staged, W2 is prefetched into registers, the mid image is zeroed;
//   phase 1  cv1 for the RB+2 mid rows the band needs (rows outside the image stay zero: cv2's padding), implicit
//            im2col straight from the LDS image, v_mfma_f32_16x16x32_f16, bias + SiLU, rounded to fp16 (as the stored
//            mid tensor of the unfused pair) into the LDS mid image (RB+2 rows x W+2 px x Cm);
//   phase 2  W2 goes from registers into W1's LDS slot; cv2 from the mid image, bias + SiLU + the residual (the
//            input pixels, still in LDS), 8-byte NHWC stores into the output channel slice.
// Nothing but the input band, the weights and the output touches global memory.
//
// LDS images are pixel-major with C contiguous; a pixel's 16-byte chunk c sits at position c ^ f(p) (CH = C / 8
// chunks per pixel: f = (p >> 1) & 3 for CH 4, p & 7 for CH 8, 0 below).  ds_read_b128 is serviced in the
// non-contiguous 16-lane groups of MI355X_MICROARCH.md §LDS ({0-3,12-15,20-27}, ...), which mix two K chunks (lane
// groups kg of the 16x16x32 operand) of 8 + 8 pixels; these f make every group hit 16 distinct 16-byte slots for
// any pixel base and tap (checked exhaustively; a plain c ^ (p / (16 / CH)) swizzle is 2-way there).  Weight rows
// are pitched 64·KS + 32 bytes (4·KS + 2 slots), conflict-free for the same groups.
// Results: fp32 accumulation of fp16 products with one fp16 rounding of the mid tensor and of the output, like the
// unfused pair (only the summation order differs; f16-plan tolerance, tests/test_gpu_parity.py).
// x3 plans (X3): the input tile, the mid image and both weight matrices live in LDS as two planes each — the fp16 hi
// halves, then the lo halves, in the f16 layout (same swizzle, same conflict-free reads per plane) — and every K
// step runs three MFMAs (w_lo·x_hi, w_hi·x_lo, w_hi·x_hi).  The mid image holds the exact split of the activated
// fp32 value (hi = fp16(v), lo = fp16(v - hi)), as the unfused pair's stored pair-layout tensor; outputs are stored
// in the pair layout.  Twice the LDS of the f16 kernel: the geometry check keeps only the tiles that fit.
#include <stdlib.h>

#include "ym_common.h"

namespace {

template <int CH>
__device__ __forceinline__ int swz(int p) {
  if constexpr (CH == 4) return (p >> 1) & 3;
  else if constexpr (CH == 8) return p & 7;
  else return 0;  // 1 or 2 chunks per pixel: the plain layout is as good as any (CH 2 conflict-free, CH 1 2-way)
}

struct BneckGeom {
  int RB;          // output rows per tile
  int nbands;      // ceil(H / RB)
  int TW, ntx;     // tile width (pixels, a multiple of 16 or the map width) and tiles per row
  int C, Cm, N2;   // input (= residual) channels, mid channels, output channels
  int KS1, KS2;    // K steps of 32 per conv
  int P1, P2;      // weight row pitches (bytes)
  int MR, MC;      // mid tile rows / columns (K2 = 3: + 1-pixel halo)
  int XR, XC, XE;  // input tile rows / columns; S1 = 2: even columns first (XE of them), then the odd ones
  int offM, offW, offB;  // LDS byte offsets: mid image, weight slot, biases (input image at 0)
  int plW;               // x3: weight slot plane size (bytes)
  int lds;
  int dbg;  // tools/bneck_ablate.py timing ablations (YM_BNECK_DBG): 1 no input loads, 2 no cv1, 4 no cv2, 8 no stores
};

// one lane's 16-byte B fragment: pixel p (LDS image index), K chunk c (8 channels) of a CH-chunk image
template <int CH>
__device__ __forceinline__ f16x8 ld_px(const char* img, int p, int c) {
  return *reinterpret_cast<const f16x8*>(img + ((p * CH + (c ^ swz<CH>(p))) << 4));
}

// LDS pixel index of input-tile pixel (row, column xc).  Stride 2 keeps even and odd columns in separate half-rows,
// so the taps of 16 consecutive mid pixels (input columns 2j + kx) read 16 consecutive pixel slots.
template <int S1>
__device__ __forceinline__ int xpix(int row, int xc, int XC, int XE) {
  if constexpr (S1 == 1) return row * XC + xc;
  else return row * XC + ((xc & 1) ? XE + (xc >> 1) : (xc >> 1));
}

// S1: stride of the first 3x3 conv (1: Bottleneck, 2: a downsampling Conv); K2: kernel of the second conv (3: the
// Bottleneck's cv2 with its 1-pixel halo on the mid image; 1: a following 1x1 such as C3k2.cv1, no halo).
template <int C, int CM, int N2, int PX, int NW, int S1, int K2, bool X3>
__global__ __launch_bounds__(64 * NW) void conv_bneck(const ConvArgs a, const BneckGeom g) {
  ym_warm_kernargs<sizeof(ConvArgs)>();  // one round trip for the whole argument block (ym_common.h)
  constexpr int NT = 64 * NW;
  constexpr int XS = X3 ? 2 : 1;  // fp16 storage elements per logical channel (global pair layout)
  constexpr int CH = C / 8, CHM = CM / 8;
  constexpr int NB1 = (CM + 15) / 16, NB2 = N2 / 16;
  constexpr int KS1 = (9 * C + 31) / 32, KS2 = (K2 * K2 * CM + 31) / 32;
  constexpr int HM = K2 / 2;  // mid-tile halo
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sX = smem;
  char* sM = smem + g.offM;
  char* sW = smem + g.offW;
  float* sB1 = reinterpret_cast<float*>(smem + g.offB);
  float* sB2 = sB1 + 16 * NB1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kg = lane >> 4;
  const int W = a.Wo, H = a.Ho, TW = g.TW;  // mid (= output) map
  const int MR = g.MR, MC = g.MC, XR = g.XR, XC = g.XC, XE = g.XE;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // neighbouring tiles (shared halo rows) on one XCD
  const int tx = vb % g.ntx, band = (vb / g.ntx) % g.nbands, b = vb / (g.ntx * g.nbands);
  const int RB = g.RB, r0 = band * RB, x0 = tx * TW;  // the tile: rows r0 .. r0+RB-1, columns x0 .. x0+TW-1
  const int mr0 = r0 - HM, mc0 = x0 - HM;           // mid tile origin (map coordinates)
  const int xr0 = mr0 * S1 - 1, xc0 = mc0 * S1 - 1;  // input tile origin (input map coordinates)
  const f16* src = static_cast<const f16*>(a.src0);
  const f16* W1 = static_cast<const f16*>(a.w);
  const f16* W2 = static_cast<const f16*>(a.w2);
  // x3: byte distance from a hi plane to its lo plane (input tile, mid image, weight slot)
  const int plX = g.XR * g.XC * C * 2, plM = g.MR * g.MC * CM * 2, plW = g.plW;

  // ---- phase 0: W2 prefetch (registers), W1 + biases, input tile (zeros outside the input map), zeroed mid image
  constexpr int W2CH = N2 * KS2 * 4;  // 16-byte chunks of W2 rows [N2][KS2 * 32] (x3: per plane)
  constexpr int W2PT = (W2CH + NT - 1) / NT;
  f16x8 w2r[W2PT], w2l[X3 ? W2PT : 1];
#pragma unroll
  for (int u = 0; u < W2PT; ++u) {
    const int i = tid + NT * u;
    const int n = i / (KS2 * 4), c = i - n * (KS2 * 4);
    // (x3: the weight rows are pair chunks — logical chunk c's hi half at 16 c, its lo half 8 further; the K padding
    // chunks past 9 CM / 8 read zeros inside the padded row)
    const f16* q = W2 + (size_t)n * a.Kpad2 + 8 * XS * c;
    w2r[u] = i < W2CH ? *reinterpret_cast<const f16x8*>(q) : Vec8<f16>::zero();
    if constexpr (X3) w2l[u] = i < W2CH ? *reinterpret_cast<const f16x8*>(q + 8) : Vec8<f16>::zero();
  }
  for (int i = tid; i < 16 * NB1 * KS1 * 4; i += NT) {
    const int n = i / (KS1 * 4), c = i - n * (KS1 * 4);
    const f16* q = W1 + (size_t)n * a.Kpad + 8 * XS * c;
    const f16x8 v = n < CM ? *reinterpret_cast<const f16x8*>(q) : Vec8<f16>::zero();
    *reinterpret_cast<f16x8*>(sW + n * g.P1 + 16 * c) = v;
    if constexpr (X3) {
      const f16x8 vl = n < CM ? *reinterpret_cast<const f16x8*>(q + 8) : Vec8<f16>::zero();
      *reinterpret_cast<f16x8*>(sW + plW + n * g.P1 + 16 * c) = vl;
    }
  }
  for (int i = tid; i < 16 * NB1; i += NT) sB1[i] = i < CM ? a.bias[i] : 0.f;
  for (int i = tid; i < N2; i += NT) sB2[i] = a.bias2[i];
  {
    const int nx = XR * XC * CH;  // input tile chunks, in input-map order
    const size_t img = (size_t)b * a.s0_P;
    constexpr int UN = X3 ? 4 : 8;  // loads in flight per thread and round (x3: two 16-byte halves each)
    for (int i0 = tid; i0 < nx; i0 += NT * UN) {
      f16x8 v[UN], vl[X3 ? UN : 1];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int i = i0 + NT * u;
        const int q = i / CH, c = i - q * CH;
        const int row = q / XC, xc = q - row * XC;
        const int gy = xr0 + row, gx = xc0 + xc;
        const bool in = i < nx && !(g.dbg & 1) && (unsigned)gy < (unsigned)a.Hin && (unsigned)gx < (unsigned)a.Win;
        const f16* p = src + ((img + (size_t)gy * a.Win + gx) * a.s0_ctot + a.s0_coff + 8 * c) * XS;
        v[u] = in ? *reinterpret_cast<const f16x8*>(p) : Vec8<f16>::zero();
        if constexpr (X3) vl[u] = in ? *reinterpret_cast<const f16x8*>(p + 8) : Vec8<f16>::zero();
      }
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int i = i0 + NT * u;
        if (i < nx) {
          const int q = i / CH, c = i - q * CH;
          const int row = q / XC, xc = q - row * XC;
          const int p = xpix<S1>(row, xc, XC, XE);
          *reinterpret_cast<f16x8*>(sX + ((p * CH + (c ^ swz<CH>(p))) << 4)) = v[u];
          if constexpr (X3) *reinterpret_cast<f16x8*>(sX + plX + ((p * CH + (c ^ swz<CH>(p))) << 4)) = vl[u];
        }
      }
    }
    const int nm = MR * MC * CHM * XS;  // (x3: both planes, contiguous)
    for (int i = tid; i < nm; i += NT) *reinterpret_cast<f16x8*>(sM + (i << 4)) = Vec8<f16>::zero();
  }
  __syncthreads();

  // ---- phase 1: the first conv over the MR x MC mid tile, PX 16-pixel groups per work item (lanes past a row's end
  // compute but never store)
  {
    const int gpr = (MC + 15) / 16;
    const int ng = (g.dbg & 2) ? 0 : MR * gpr;
    for (int it = wave * PX; it < ng; it += NW * PX) {
      int prow[PX], pm[PX];  // mid row, this lane's mid column (tile coordinates)
      bool ok[PX];
#pragma unroll
      for (int q = 0; q < PX; ++q) {
        const int gi = it + q < ng ? it + q : ng - 1;  // a tail slot recomputes the last group, never stores it
        prow[q] = gi / gpr;
        pm[q] = (gi - prow[q] * gpr) * 16 + col;
        const int gm = mr0 + prow[q], xm = mc0 + pm[q];
        ok[q] = it + q < ng && pm[q] < MC && (unsigned)gm < (unsigned)H && (unsigned)xm < (unsigned)W;
        if (pm[q] >= MC) pm[q] = MC - 1;  // keep the reads inside the image rows
      }
      f32x4 acc[NB1][PX];
#pragma unroll
      for (int nb = 0; nb < NB1; ++nb)
#pragma unroll
        for (int q = 0; q < PX; ++q) acc[nb][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
      for (int s = 0; s < KS1; ++s) {
        const int K = 32 * s + 8 * kg;
        int tap = K / C;
        const int ch = (K - tap * C) >> 3;
        if (tap > 8) tap = 8;  // K padding: finite pixels times zero weights
        const int ky = tap / 3, kx = tap - 3 * ky;
        f16x8 wa[NB1], xb[PX], wl[X3 ? NB1 : 1], xl[X3 ? PX : 1];
#pragma unroll
        for (int nb = 0; nb < NB1; ++nb) {
          wa[nb] = *reinterpret_cast<const f16x8*>(sW + (16 * nb + col) * g.P1 + 2 * K);
          if constexpr (X3) wl[nb] = *reinterpret_cast<const f16x8*>(sW + plW + (16 * nb + col) * g.P1 + 2 * K);
        }
#pragma unroll
        for (int q = 0; q < PX; ++q) {
          const int px = xpix<S1>(prow[q] * S1 + ky, pm[q] * S1 + kx, XC, XE);
          xb[q] = ld_px<CH>(sX, px, ch);
          if constexpr (X3) xl[q] = ld_px<CH>(sX + plX, px, ch);
        }
#pragma unroll
        for (int nb = 0; nb < NB1; ++nb)
#pragma unroll
          for (int q = 0; q < PX; ++q) {
            if constexpr (X3) {
              acc[nb][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[nb], xb[q], acc[nb][q], 0, 0, 0);
              acc[nb][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nb], xl[q], acc[nb][q], 0, 0, 0);
            }
            acc[nb][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nb], xb[q], acc[nb][q], 0, 0, 0);
          }
      }
      // lane: channels 16 nb + 4 kg .. + 3 of its pixel -> 8 bytes of the mid image
#pragma unroll
      for (int q = 0; q < PX; ++q) {
        if (!ok[q]) continue;
        const int p = prow[q] * MC + pm[q];
#pragma unroll
        for (int nb = 0; nb < NB1; ++nb) {
          const int n0 = 16 * nb + 4 * kg;
          if (n0 >= CM) continue;
          f16x4 h, hl;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = X3 ? ym_x3_pre(acc[nb][q][r], a.wsc, sB1[n0 + r]) : acc[nb][q][r] + sB1[n0 + r];
            if constexpr (X3) {
              const float vv = a.act ? ym_silu_x3(v) : v;
              h[r] = (f16)vv;
              hl[r] = (f16)(vv - (float)h[r]);
            } else {
              h[r] = (f16)(a.act ? ym_silu_fast(v) : v);
            }
          }
          const int c = n0 >> 3;
          const int off = ((p * CHM + (c ^ swz<CHM>(p))) << 4) + ((n0 & 4) << 1);
          *reinterpret_cast<f16x4*>(sM + off) = h;
          if constexpr (X3) *reinterpret_cast<f16x4*>(sM + plM + off) = hl;
        }
      }
    }
  }
  __syncthreads();  // mid image complete; every wave is done with W1
#pragma unroll
  for (int u = 0; u < W2PT; ++u) {
    const int i = tid + NT * u;
    if (i < W2CH) {
      const int n = i / (KS2 * 4), c = i - n * (KS2 * 4);
      *reinterpret_cast<f16x8*>(sW + n * g.P2 + 16 * c) = w2r[u];
      if constexpr (X3) *reinterpret_cast<f16x8*>(sW + plW + n * g.P2 + 16 * c) = w2l[u];
    }
  }
  __syncthreads();

  // ---- phase 2: the second conv over the RB x TW output tile, + residual (S1 = 1, K2 = 3: the input pixels, still in
  // LDS), stores
  {
    const int rows = H - r0 < RB ? H - r0 : RB;
    const int xe = W - x0 < TW ? W - x0 : TW;  // tile columns inside the map
    const int gpr = (TW + 15) / 16;
    const int ng = (g.dbg & 4) ? 0 : rows * gpr;
    f16* dst = static_cast<f16*>(a.dst);
    P2* dstp = static_cast<P2*>(a.dst);
    const bool res = S1 == 1 && K2 == 3 && a.res != nullptr;
    for (int it = wave * PX; it < ng; it += NW * PX) {
      int prow[PX], pc[PX];  // output row, this lane's output column (both within the tile)
#pragma unroll
      for (int q = 0; q < PX; ++q) {
        const int gi = it + q < ng ? it + q : ng - 1;
        prow[q] = gi / gpr;
        pc[q] = (gi - prow[q] * gpr) * 16 + col;
        if (K2 == 1 && pc[q] >= MC) pc[q] = MC - 1;
      }
      f32x4 acc[NB2][PX];
#pragma unroll
      for (int nb = 0; nb < NB2; ++nb)
#pragma unroll
        for (int q = 0; q < PX; ++q) acc[nb][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
      for (int s = 0; s < KS2; ++s) {
        const int K = 32 * s + 8 * kg;
        int tap = K / CM;
        const int ch = (K - tap * CM) >> 3;
        if (tap > K2 * K2 - 1) tap = K2 * K2 - 1;
        const int ky = tap / 3, kx = tap - 3 * ky;
        f16x8 wa[NB2], xb[PX], wl[X3 ? NB2 : 1], xl[X3 ? PX : 1];
#pragma unroll
        for (int nb = 0; nb < NB2; ++nb) {
          wa[nb] = *reinterpret_cast<const f16x8*>(sW + (16 * nb + col) * g.P2 + 2 * K);
          if constexpr (X3) wl[nb] = *reinterpret_cast<const f16x8*>(sW + plW + (16 * nb + col) * g.P2 + 2 * K);
        }
#pragma unroll
        for (int q = 0; q < PX; ++q) {
          const int pm2 = (prow[q] + ky) * MC + pc[q] + kx;
          xb[q] = ld_px<CHM>(sM, pm2, ch);
          if constexpr (X3) xl[q] = ld_px<CHM>(sM + plM, pm2, ch);
        }
#pragma unroll
        for (int nb = 0; nb < NB2; ++nb)
#pragma unroll
          for (int q = 0; q < PX; ++q) {
            if constexpr (X3) {
              acc[nb][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[nb], xb[q], acc[nb][q], 0, 0, 0);
              acc[nb][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nb], xl[q], acc[nb][q], 0, 0, 0);
            }
            acc[nb][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nb], xb[q], acc[nb][q], 0, 0, 0);
          }
      }
#pragma unroll
      for (int q = 0; q < PX; ++q) {
        if (it + q >= ng || pc[q] >= xe) continue;
        const int y = r0 + prow[q], x = x0 + pc[q];
        const int px = xpix<S1>(prow[q] + 2, pc[q] + 2, XC, XE);  // the same pixel in the input tile (residual)
        const size_t obase = (size_t)(b * a.d_P + y * a.d_W + x) * a.d_ctot + a.d_coff;
#pragma unroll
        for (int nb = 0; nb < NB2; ++nb) {
          const int n0 = 16 * nb + 4 * kg;
          float rv[4] = {0.f, 0.f, 0.f, 0.f};
          if (res) {
            const int c = n0 >> 3;
            const int off = ((px * CH + (c ^ swz<CH>(px))) << 4) + ((n0 & 4) << 1);
            const f16x4 rh = *reinterpret_cast<const f16x4*>(sX + off);
#pragma unroll
            for (int r = 0; r < 4; ++r) rv[r] = (float)rh[r];
            if constexpr (X3) {
              const f16x4 rl = *reinterpret_cast<const f16x4*>(sX + plX + off);
#pragma unroll
              for (int r = 0; r < 4; ++r) rv[r] += (float)rl[r];
            }
          }
          if constexpr (X3) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = ym_x3_pre(acc[nb][q][r], a.wsc2, sB2[n0 + r]);
              o[r] = (a.act2 ? ym_silu_x3(v) : v) + rv[r];
            }
            // lanes (kg, kg ^ 1) of this pixel write whole 32-byte chunks where the output slice keeps them whole
            if ((a.pst & 8) && ((a.d_coff | a.d_ctot) & 7) == 0) ym_p2_store4_pair<16>(dstp + obase + n0, o, kg & 1, !(g.dbg & 8), a.pst & 16);
            else if (!(g.dbg & 8)) ym_p2_store4(dstp + obase + n0, o);
          } else {
            f16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = acc[nb][q][r] + sB2[n0 + r];
              o[r] = (f16)((a.act2 ? ym_silu_fast(v) : v) + rv[r]);
            }
            if (!(g.dbg & 8)) *reinterpret_cast<f16x4*>(dst + obase + n0) = o;
          }
        }
      }
    }
  }
}

// (id, RB, TW, PX, NW): output rows per tile, tile width (0: the whole row; else a multiple of 16), 16-pixel groups
// per work item, waves per workgroup.  Full-row tiles hold one workgroup per CU (NW / 4 waves per SIMD hide each
// other's LDS-read latency); the half-row tiles fit two, whose load / compute / store phases then overlap.
#define YM_BNECK_CFGS(X)                                                                                       \
  X(0, 2, 0, 4, 8) X(1, 4, 0, 4, 8) X(2, 5, 0, 4, 8) X(3, 8, 0, 4, 8) X(4, 4, 0, 2, 16) X(5, 5, 0, 2, 16)     \
  X(6, 8, 0, 2, 16) X(7, 2, 0, 2, 16) X(8, 4, 80, 2, 8) X(9, 5, 80, 2, 8) X(10, 8, 80, 2, 8) X(11, 4, 48, 2, 8) \
  X(12, 8, 48, 2, 8) X(13, 2, 80, 2, 8)
constexpr int kNumBneck = 14;
// x3-only variants (ids appended to the x3 id space): 2-row x 32-pixel tiles, the one geometry in which the 80²
// (64, 32, 64) Bottleneck's doubled LDS (hi / lo planes of input tile, mid image and weights: 151 KB) fits
#define YM_BNECK_X3_CFGS(X) X(14, 2, 32, 2, 8) X(15, 2, 32, 2, 4)
constexpr int kNumBneckX3 = 2;
constexpr int kMaxLds = 160 * 1024;

bool bneck_geom(const ConvArgs& a, int C, int CM, int N2, int S1, int K2, int RB, int TW, BneckGeom& g, int xs) {
  g.RB = RB;
  g.nbands = (a.Ho + RB - 1) / RB;
  if (TW >= a.Wo) TW = 0;
  g.TW = TW ? TW : a.Wo;
  g.ntx = (a.Wo + g.TW - 1) / g.TW;
  g.C = C; g.Cm = CM; g.N2 = N2;
  g.KS1 = (9 * C + 31) / 32;
  g.KS2 = (K2 * K2 * CM + 31) / 32;
  g.P1 = 64 * g.KS1 + 32;
  g.P2 = 64 * g.KS2 + 32;
  const int hm = K2 / 2;
  g.MR = RB + 2 * hm;
  g.MC = g.TW + 2 * hm;
  g.XR = (g.MR - 1) * S1 + 3;
  g.XC = (g.MC - 1) * S1 + 3;
  g.XE = (g.XC + 1) / 2;
  const int sx = g.XR * g.XC * C * 2 * xs, sm = g.MR * g.MC * CM * 2 * xs;  // (x3: hi and lo planes)
  const int nb1 = (CM + 15) / 16;
  const int w1 = 16 * nb1 * g.P1, w2 = N2 * g.P2;
  g.plW = w1 > w2 ? w1 : w2;
  g.offM = sx;
  g.offW = sx + sm;
  g.offB = g.offW + g.plW * xs;
  g.lds = g.offB + (16 * nb1 + N2) * 4;
  static const int dbg = [] {
    const char* e = getenv("YM_BNECK_DBG");
    return e ? atoi(e) : 0;
  }();
  g.dbg = dbg;
  return g.lds <= kMaxLds;
}

template <int C, int CM, int N2, int S1, int K2, int RB, int TW, int PX, int NW, bool X3>
hipError_t launch(const ConvArgs& a, hipStream_t st) {
  BneckGeom g;
  if ((TW && TW >= a.Wo) || !bneck_geom(a, C, CM, N2, S1, K2, RB, TW, g, X3 ? 2 : 1))
    return hipErrorInvalidValue;  // (TW: a real split)
  const int B = a.M / (a.Ho * a.Wo);
  hipLaunchKernelGGL((conv_bneck<C, CM, N2, PX, NW, S1, K2, X3>), dim3(B * g.nbands * g.ntx), dim3(64 * NW), g.lds, st,
                     a, g);
  return hipGetLastError();
}

template <int C, int CM, int N2, int S1, int K2, bool X3>
hipError_t dispatch_cfg(const ConvArgs& a, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, rb, tw, px, nw) \
  case id: return launch<C, CM, N2, S1, K2, rb, tw, px, nw, X3>(a, st);
    YM_BNECK_CFGS(YM_X)
#undef YM_X
  }
  if constexpr (X3) {
    switch (i) {
#define YM_X(id, rb, tw, px, nw) \
  case id: return launch<C, CM, N2, S1, K2, rb, tw, px, nw, true>(a, st);
      YM_BNECK_X3_CFGS(YM_X)
#undef YM_X
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace

int ym_conv_bneck_num_cfgs() { return kNumBneck; }
int ym_conv_bneck_x3_num_cfgs() { return kNumBneckX3; }

// Host-side applicability: a fused pair (w2) of a 3x3 / pad 1 conv on one plain source followed by either
//   * a 3x3 stride-1 conv (k2 == 3, first conv stride 1): a Bottleneck; the residual, if any, IS the input view, or
//   * a 1x1 conv (k2 == 1, first conv stride 2): a downsampling Conv and the next C3k2's cv1, no residual;
// (C, Cm, N2) one of the YOLO11 shapes instantiated below; fp16 output into a 4-aligned channel slice.
hipError_t ym_launch_conv_bneck(int out_f32, const ConvArgs& a, int i, hipStream_t st) {
  if (i < 0 || i >= kNumBneck + (a.x3 ? kNumBneckX3 : 0) || out_f32) return hipErrorInvalidValue;
  if (!a.w2 || a.k != 3 || a.pad != 1 || a.src1 || a.up0 || a.shuffle || a.raw || a.nchw) return hipErrorInvalidValue;
  const bool bneck = a.k2 == 3 && a.s == 1, down = a.k2 == 1 && a.s == 2;
  if (!bneck && !down) return hipErrorInvalidValue;
  if (a.Ho != (a.Hin - 1) / a.s + 1 || a.Wo != (a.Win - 1) / a.s + 1 || a.d_W != a.Wo || a.d_pixoff)
    return hipErrorInvalidValue;
  if ((a.s0_ctot & 7) || (a.s0_coff & 7) || (a.d_ctot & 3) || (a.d_coff & 3)) return hipErrorInvalidValue;
  if (a.res && (down || a.res != a.src0 || a.r_ctot != a.s0_ctot || a.r_coff != a.s0_coff || a.r_P != a.s0_P))
    return hipErrorInvalidValue;
  const int C = a.C0, CM = a.N, N2 = a.N2, K2 = a.k2;
  // x3: Cin8 / Kpad / Kpad2 count fp16 storage (the pair chunks); the kernel walks logical K chunks of 8 channels
  const int xs = a.x3 ? 2 : 1;
  if (xs * C != 8 * a.Cin8 || a.Kpad < xs * 32 * ((9 * C + 31) / 32) || a.Kpad2 < xs * 32 * ((K2 * K2 * CM + 31) / 32))
    return hipErrorInvalidValue;
  if (a.x3) {
    if (down) {  // the stride-2 "down" pairs: only the narrow tiles fit the doubled LDS (2 x 32 px: 136 KB for s model.1)
      if (C == 32 && CM == 64 && N2 == 64) return dispatch_cfg<32, 64, 64, 2, 1, true>(a, i, st);
      if (C == 16 && CM == 32 && N2 == 32) return dispatch_cfg<16, 32, 32, 2, 1, true>(a, i, st);
      return hipErrorInvalidValue;
    }
    if (C == 16 && CM == 8 && N2 == 16) return dispatch_cfg<16, 8, 16, 1, 3, true>(a, i, st);
    if (C == 32 && CM == 16 && N2 == 32) return dispatch_cfg<32, 16, 32, 1, 3, true>(a, i, st);
    if (C == 64 && CM == 32 && N2 == 64) return dispatch_cfg<64, 32, 64, 1, 3, true>(a, i, st);
    if (C == 32 && CM == 32 && N2 == 32) return dispatch_cfg<32, 32, 32, 1, 3, true>(a, i, st);
    if (C == 64 && CM == 64 && N2 == 64) return dispatch_cfg<64, 64, 64, 1, 3, true>(a, i, st);
    return hipErrorInvalidValue;
  }
  if (bneck) {
    if (C == 16 && CM == 8 && N2 == 16) return dispatch_cfg<16, 8, 16, 1, 3, false>(a, i, st);
    if (C == 32 && CM == 16 && N2 == 32) return dispatch_cfg<32, 16, 32, 1, 3, false>(a, i, st);
    if (C == 64 && CM == 32 && N2 == 64) return dispatch_cfg<64, 32, 64, 1, 3, false>(a, i, st);
    if (C == 32 && CM == 32 && N2 == 32) return dispatch_cfg<32, 32, 32, 1, 3, false>(a, i, st);
    if (C == 64 && CM == 64 && N2 == 64) return dispatch_cfg<64, 64, 64, 1, 3, false>(a, i, st);  // s: C3k at 40x40
  } else {
    if (C == 32 && CM == 64 && N2 == 64) return dispatch_cfg<32, 64, 64, 2, 1, false>(a, i, st);  // s model.1, n model.3
    if (C == 16 && CM == 32 && N2 == 32) return dispatch_cfg<16, 32, 32, 2, 1, false>(a, i, st);  // n model.1
  }
  return hipErrorInvalidValue;
}
