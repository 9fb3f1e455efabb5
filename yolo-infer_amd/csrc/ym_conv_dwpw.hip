// Depthwise 3x3 → 1x1 conv in one launch: the Detect head's classification chains (reference
// core/model.py → Ultralytics Detect.cv3[l] = Sequential(Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
// Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)), Conv2d(c3, nc, 1))).  yolomi/arch.py GraphBuilder.fuse_dw merges a
// depthwise op into the 1x1 conv that is the only reader of its output; the depthwise output never reaches HBM.
//
// A workgroup owns a TH x TW tile of output pixels of one image (TH·TW = 64: four 16-pixel groups, one per wave) and
// every output channel (N <= 128: 8 blocks of 16).  Per K block of 32 logical channels:
//   * staging: the (TH+2) x (TW+2) input window of the block's 4 channel chunks (zeros outside the image: buffer
//     loads at an out-of-range offset), the 1x1 weight rows of the block and its depthwise taps / bias go to LDS —
//     loaded into registers one block AHEAD, so the memory latency hides under the previous block's compute; each
//     window pixel is fetched once per workgroup instead of 9 times per output pixel;
//   * depthwise: lane (g, col) of wave w computes pixel 16 w + col (tile row-major), channels 32 kb + 8 g .. + 7 —
//     exactly its B operand of v_mfma_f32_16x16x32_f16 (k = 8 g .. 8 g + 7 of pixel col), in the arithmetic of
//     csrc/ym_misc.hip dwconv3x3* (acc = bias, fmaf over taps 0..8 on the stored values — x3: hi + lo in fp32 —,
//     SiLU (x3: ym_silu_x3, f16: ym_silu_fast), then x3: hi = fp16(v), lo = fp16(v - hi)): the same B operands the
//     unfused 1x1 would read back from the stored depthwise tensor;
//   * the 1x1: A fragments from the LDS weight rows (pitch 32·XS + 16 halves, conflict-free for the 16-row reads as
//     in csrc/ym_conv_stream.hip); x3 takes three MFMAs per block (w_lo·x_hi + w_hi·x_lo + w_hi·x_hi), f16 one;
//   * epilogue as the other x3 convs: fmaf(acc, 2^-s, bias), SiLU, lane-pair whole-chunk stores (x3) / fp16x4.
// The window is kept in two planes of 4 channels ([chunk][pixel] f32x4 for x3, f16x8 for f16), so the 16-byte reads of
// consecutive lanes (consecutive pixels) are consecutive in LDS.
// SPLIT > 1 (the P4 / P5 maps: 40², 20²): the K blocks of a tile are divided over SPLIT workgroups — a block's depthwise
// channels are its own, so the depthwise work splits with the GEMM's K.  Each workgroup publishes its fp32 partial tile
// write-through (sc1) into the stream's split-K slab, and the last to arrive at the tile's counter sums the SPLIT partials
// in split order (bitwise the same whichever arrives last) and runs the epilogue: the sc1 hand-off of
// csrc/ym_conv_dma.hip.  Without it the 20² maps had 80 workgroups, each a chain of 16 K blocks at ~2 µs.
#include <type_traits>

#include "ym_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// (id, tile width (the tile is 64 / tw rows high: 16 for 80² maps, 8 for 40², 4 for 20²), K split)
#define YM_DWPW_CFGS(X) X(0, 16, 1) X(1, 8, 1) X(2, 4, 1) X(3, 8, 2) X(4, 8, 4) X(5, 4, 2) X(6, 4, 4) X(7, 4, 8)
struct DwpwCfg {
  int tw, split;
};
constexpr DwpwCfg kDwpw[] = {
#define YM_X(id, tw, sp) {tw, sp},
    YM_DWPW_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumDwpw = sizeof(kDwpw) / sizeof(kDwpw[0]);
constexpr int kDwpwMaxC = 512;  // depthwise channels (the head's widest input)
constexpr int kDwpwNB = 8;      // output-channel blocks of 16 (N <= 128)
constexpr unsigned OOBX = 0x80000000u;

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

template <typename T, int TW, int SPLIT>
__global__ __launch_bounds__(256, 2) void conv_dwpw(const ConvArgs a) {
  ym_warm_kernargs<sizeof(ConvArgs)>();  // one round trip for the whole argument block (ym_common.h)
  constexpr bool X3 = std::is_same<T, P2>::value;
  constexpr int XS = X3 ? 2 : 1;            // fp16 storage elements per logical channel
  constexpr int TH = 64 / TW, IH = TH + 2, IW = TW + 2, NPIX = IH * IW;
  constexpr int NWIN = NPIX * 4;            // window items (pixel, 8-channel chunk)
  constexpr int WPT = (NWIN + 255) / 256;   // window items per thread
  constexpr int LDW = 32 * XS + 16;         // LDS pitch of a 1x1 weight row (halves)
  constexpr int WQ = 128 * 32 * XS / 8 / 256;  // 16-byte weight pieces per thread and block (x3 4, f16 2)
  // window planes: x3 [2][4 chunks][NPIX] f32x4 (channels 0-3 / 4-7 of each chunk as fp32 hi + lo); f16 [4][NPIX] f16x8
  __shared__ __attribute__((aligned(16))) u32x4 win[(X3 ? 2 : 1) * 4 * NPIX];
  __shared__ __attribute__((aligned(16))) f16 w1[128 * LDW];
  __shared__ __attribute__((aligned(16))) float dwk[10 * 32 + 4];  // the block's taps [9][32], bias [32], split flag
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int C = a.C0;
  const int ntx = (a.Wo + TW - 1) / TW, nty = (a.Ho + TH - 1) / TH;
  // neighbouring tiles (shared window rows) and a tile's K splits on one XCD
  int vb = ym_xcd_block(blockIdx.x, gridDim.x);
  const int sp = vb % SPLIT;
  vb /= SPLIT;
  const int tile = vb;
  const int tx = vb % ntx;
  vb /= ntx;
  const int ty = vb % nty, b = vb / nty;
  const int y0 = ty * TH, x0 = tx * TW;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.src0), 0,
                                                                      (int)(a.s0_elems * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0,
                                                                      (int)((long)a.N * a.Kpad * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dw_w), 0, 40 * C, 0x00020000);
  // per thread, fixed over the K loop: its window items' pixel offsets (logical elements; -1 outside the image)
  int woff[WPT];
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int i = tid + 256 * u, q = i >> 2;
    const int iy = y0 - 1 + q / IW, ix = x0 - 1 + q % IW;
    woff[u] = (i < NWIN && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win)
                  ? (b * a.s0_P + iy * a.s0_W + ix) * a.s0_ctot + a.s0_coff + 8 * (i & 3)
                  : -1;
  }
  // registers of the next block: window items (x3: hi and lo), weight pieces, one dw-weight float4
  struct Regs {
    u32x4 win[WPT][XS], w1[WQ], dk;
  };
  auto load = [&](Regs& r, int kb) {
    const int c0 = 32 * kb;
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const bool ok = woff[u] >= 0 && c0 + 8 * ((tid + 256 * u) & 3) < C;
      const unsigned off = (unsigned)(woff[u] + c0) * (2u * XS);
      r.win[u][0] = bld(rs, ok ? off : OOBX);
      if constexpr (X3) r.win[u][1] = bld(rs, ok ? off + 16u : OOBX);
    }
#pragma unroll
    for (int q = 0; q < WQ; ++q) {  // piece i: row n = i / (4 XS), 16-byte piece j of the row's block
      const int i = tid + 256 * q, n = i / (4 * XS), j = i % (4 * XS);
      const bool ok = n < a.N && c0 * XS + 8 * j < a.Kpad;
      r.w1[q] = bld(rw, ok ? (unsigned)(n * a.Kpad + c0 * XS + 8 * j) * 2u : OOBX);
    }
    if (tid < 80) {  // taps t < 9: dw_w[t][c0 + 4 v]; t == 9: the bias (dw_b follows dw_w: one buffer)
      const int t = tid >> 3, v = tid & 7;
      const bool ok = c0 + 4 * v < C;
      r.dk = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, ok ? (unsigned)((t * C + c0 + 4 * v) * 4) : OOBX, 0, 0));
    }
  };
  auto store = [&](const Regs& r) {
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const int i = tid + 256 * u;
      if (i >= NWIN) continue;
      const int pix = i >> 2, ch = i & 3;
      if constexpr (X3) {
        const f16x8 hv = __builtin_bit_cast(f16x8, r.win[u][0]), lv = __builtin_bit_cast(f16x8, r.win[u][1]);
        f32x4 p0, p1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          p0[e] = (float)hv[e] + (float)lv[e];
          p1[e] = (float)hv[4 + e] + (float)lv[4 + e];
        }
        win[ch * NPIX + pix] = __builtin_bit_cast(u32x4, p0);
        win[(4 + ch) * NPIX + pix] = __builtin_bit_cast(u32x4, p1);
      } else {
        win[ch * NPIX + pix] = r.win[u][0];
      }
    }
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int i = tid + 256 * q, n = i / (4 * XS), j = i % (4 * XS);
      *reinterpret_cast<u32x4*>(w1 + n * LDW + 8 * j) = r.w1[q];
    }
    if (tid < 80) *reinterpret_cast<u32x4*>(dwk + 4 * tid) = r.dk;
  };

  // this lane's output pixel
  const int p = 16 * wave + col, py = p / TW, px = p % TW;
  const int y = y0 + py, x = x0 + px;
  const bool okm = y < a.Ho && x < a.Wo;
  const int NB = (a.N + 15) >> 4;
  const int nkb = (C + 31) >> 5;
  const int kb_lo = nkb * sp / SPLIT, kb_hi = nkb * (sp + 1) / SPLIT;  // this split's K blocks (launch: nkb >= SPLIT)
  f32x4 acc[kDwpwNB];
#pragma unroll
  for (int nb = 0; nb < kDwpwNB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the depthwise of block kb from LDS (lane (g, col): pixel p, chunk g), then its 1x1 MFMAs
  auto compute = [&](int kb) {
    const bool kc = 32 * kb + 8 * g < C;
    float v[8];
    {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(dwk + 9 * 32 + 8 * g),
                  b1 = *reinterpret_cast<const f32x4*>(dwk + 9 * 32 + 8 * g + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = b0[e]; v[4 + e] = b1[e]; }
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int q = (py + t / 3) * IW + px + t % 3;
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(dwk + t * 32 + 8 * g),
                  w1v = *reinterpret_cast<const f32x4*>(dwk + t * 32 + 8 * g + 4);
      if constexpr (X3) {
        const f32x4 x0v = __builtin_bit_cast(f32x4, win[g * NPIX + q]), x1v = __builtin_bit_cast(f32x4, win[(4 + g) * NPIX + q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = fmaf(x0v[e], w0[e], v[e]);
          v[4 + e] = fmaf(x1v[e], w1v[e], v[4 + e]);
        }
      } else {
        const f16x8 xv = __builtin_bit_cast(f16x8, win[g * NPIX + q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = fmaf((float)xv[e], w0[e], v[e]);
          v[4 + e] = fmaf((float)xv[4 + e], w1v[e], v[4 + e]);
        }
      }
    }
    h8 xh, xl;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float sv = a.dw_act ? (X3 ? ym_silu_x3(v[e]) : ym_silu_fast(v[e])) : v[e];
      sv = kc ? sv : 0.f;  // channels past C: a zero operand (their weights are zero-padded too)
      xh[e] = (f16)sv;
      if constexpr (X3) xl[e] = (f16)(sv - (float)xh[e]);
    }
#pragma unroll
    for (int nb = 0; nb < kDwpwNB; ++nb) {
      if (nb >= NB) break;
      const f16* wr = w1 + (16 * nb + col) * LDW + 8 * XS * g;  // x3: [hi x8 | lo x8] of the lane's chunk
      const h8 wa = *reinterpret_cast<const h8*>(wr);
      if constexpr (X3) {
        const h8 wb = *reinterpret_cast<const h8*>(wr + 8);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb, xh, acc[nb], 0, 0, 0);
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, xl, acc[nb], 0, 0, 0);
      }
      acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, xh, acc[nb], 0, 0, 0);
    }
  };
  // one block ahead (a second register set, block kb + 2 in flight during block kb, spilled ~100 VGPRs: the x3 kernel
  // already holds 248, the compiler hoisting a block's depthwise taps and window reads together)
  Regs ra;
  load(ra, kb_lo);
  for (int kb = kb_lo; kb < kb_hi; ++kb) {
    store(ra);
    __syncthreads();
    if (kb + 1 < kb_hi) load(ra, kb + 1);
    compute(kb);
    __syncthreads();  // every wave is done with the block's LDS before the next store
  }

  if constexpr (SPLIT > 1) {
    // publish this split's partial tile write-through; the last arriver sums all SPLIT partials in split order
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
        a.slab, 0, (int)(a.slab_cap < 0x7FFFFFF0L ? a.slab_cap : 0x7FFFFFF0L), 0x00020000);
    constexpr int SC1 = 16;  // cache-policy aux bit: sc1 (write-through stores / L1-bypassing loads)
    constexpr unsigned PART = 256u * kDwpwNB * 16u;  // bytes of one split's partial tile
#pragma unroll
    for (int nb = 0; nb < kDwpwNB; ++nb)
      if (nb < NB)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[nb]), rsl,
                                               (unsigned)(tile * SPLIT + sp) * PART + (unsigned)(nb * 256 + tid) * 16u,
                                               0, SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(dwk + 10 * 32);
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == SPLIT - 1;
      if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below the ticket
    // four splits' loads in flight at a time (registers), summed in split order
    constexpr int CH = SPLIT < 4 ? SPLIT : 4;
#pragma unroll
    for (int s0 = 0; s0 < SPLIT; s0 += CH) {
      f32x4 part[CH][kDwpwNB];
#pragma unroll
      for (int s2 = 0; s2 < CH; ++s2)
#pragma unroll
        for (int nb = 0; nb < kDwpwNB; ++nb)
          if (nb < NB)
            part[s2][nb] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                           rsl, (unsigned)(tile * SPLIT + s0 + s2) * PART + (unsigned)(nb * 256 + tid) * 16u, 0, SC1));
#pragma unroll
      for (int s2 = 0; s2 < CH; ++s2)
#pragma unroll
        for (int nb = 0; nb < kDwpwNB; ++nb)
          if (nb < NB) acc[nb] = (s0 + s2 == 0) ? part[s2][nb] : acc[nb] + part[s2][nb];
    }
  }

  // epilogue: lane (g, col) holds channels 16 nb + 4 g .. + 3 of pixel (y, x)
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

template <typename T, int TW, int SPLIT>
hipError_t launch(const ConvArgs& a, hipStream_t st) {
  constexpr int TH = 64 / TW;
  const int tiles = (a.M / (a.Ho * a.Wo)) * ((a.Ho + TH - 1) / TH) * ((a.Wo + TW - 1) / TW);
  if (SPLIT > 1) {  // every split owns >= 1 K block; the partial tiles fit the stream's slab, the tiles its counters
    if ((a.C0 + 31) / 32 < SPLIT || !a.slab || !a.cnt || tiles > a.cnt_cap ||
        (long)tiles * SPLIT * 256 * kDwpwNB * 16 > a.slab_cap)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL((conv_dwpw<T, TW, SPLIT>), dim3(tiles * SPLIT), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_cfg(const ConvArgs& a, int cfg, hipStream_t st) {
  switch (cfg) {
#define YM_X(id, tw, sp) \
  case id: return launch<T, tw, sp>(a, st);
    YM_DWPW_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
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
  const bool x3 = dtype == YM_DT_X3;
  if (cfg >= 0 && cfg < kNumDwpw) {
    const hipError_t e = x3 ? launch_cfg<P2>(a, cfg, st) : launch_cfg<f16>(a, cfg, st);
    if (e != hipErrorInvalidValue || strict) return e;  // (not strict: a split this shape cannot take → heuristic)
  } else if (strict) {
    return hipErrorInvalidValue;
  }
  cfg = a.Wo % 16 == 0 ? 0 : (a.Wo % 8 == 0 ? 1 : 2);  // a tile width that divides the map, no K split
  return x3 ? launch_cfg<P2>(a, cfg, st) : launch_cfg<f16>(a, cfg, st);
}
