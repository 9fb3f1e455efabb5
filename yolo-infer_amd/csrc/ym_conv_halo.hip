// Halo-tile 3x3 convolution for gfx950 (f16 plans) — the third conv generation, for the 3x3 Conv launches that
// dominate a YOLO11 forward (stride-2 downsamples model.1/3/5/7/17/20, Bottleneck 3x3s, the Detect box / mask
// branches).
//
// The implicit-GEMM kernels (csrc/ym_conv.hip, ym_conv_dma.hip, ym_conv_stream.hip) gather im2col rows straight
// from NHWC: every input pixel is fetched once per tap that reads it — 9x at stride 1, 2.25x at stride 2 — and
// the weights once per 64..128-pixel tile.  Here a workgroup owns TH FULL output rows of one image (160 or 320
// pixels) and walks Cin in chunks of CC channels; per chunk it stages
//   * the input rows of the tile plus the 3x3 halo, ONCE, into LDS (stride 2: even and odd input columns in two
//     half-rows, so every tap of consecutive output pixels reads consecutive LDS slots), and
//   * the 9 taps x BN output channels x CC input channels of weights,
// both with LDS-DMA (`buffer_load … lds`, 16 B per lane, out-of-image halo and K padding as out-of-range offsets =
// zeros), double-buffered so chunk c+1 streams in while chunk c computes.  All 9 taps then read the staged input:
// L2→LDS traffic drops to ~1.3 input reads per output pixel (stride 1) and one weight read per 160-320 pixels.
//
// LDS image: per stage, the weights [tap][output channel] and the input [pixel slot] as items of CC*2 bytes (CC/8
// 16-byte chunks = CC channels).  An item's chunk c sits at position c ^ h(item) (h = bits 2-3 of the item index for
// 4 chunks, bit 3 for 2), applied on the DMA source side: the lanes of one `buffer_load … lds` then read an item's
// CC*2 contiguous global bytes (full 64- / 32-byte segments), and the 16-lane groups of every ds_read_b128 operand
// read of v_mfma_f32_32x32x16_f16 — 16 of 32 consecutive items, one chunk — hit 16 distinct bank groups
// (checked exhaustively for every base offset).  Input slots: input row * pitch + column with pitch ≡ Wo (mod 16)
// (stride 2: even/odd column half-rows, 4·pitch ≡ Wo), so consecutive output pixels are consecutive slots mod 16
// across row wraps too.
//
// MFMA: v_mfma_f32_32x32x16_f16 in the transposed orientation of the other kernels (A = weights: 32 output channels
// x 16 K; B = pixels: 16 K x 32 pixels), one K step = one tap x 16 channels, so a lane ends with 4 groups of 4
// consecutive output channels of one pixel → bias, SiLU, residual, 8-byte NHWC stores into a channel slice.
// Waves: WM along pixels x WN along channels (WM·WN = 4); a wave holds MB 32-pixel x NB 32-channel blocks.
// Results are identical in kind to the other conv kernels (fp32 accumulation of fp16 products, one rounding to the
// output type); only the summation order differs.
#include <stdlib.h>

#include "ym_common.h"

typedef __attribute__((address_space(3))) void lds_void_t;
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr unsigned OOB = 0x80000000u;  // byte offset past num_records: the DMA deposits zeros

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// vmcnt(0) as the builtin, not inline asm: the compiler's wait-count pass then knows every earlier load (the
// prefetched residuals) has landed and inserts no drains of its own in the epilogue
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

struct HaloGeom {
  int TH;        // output rows per tile
  int tiles_y;   // ceil(Ho / TH)
  int pitch;     // stride 1: slots per input row; stride 2: slots per half-row (even / odd input columns)
  int nslot;     // real input slots
  int npad;      // slots padded so the input DMA is whole wave-instructions
  int wbytes;    // weight bytes per stage
  int stage;     // bytes per stage (weights + input)
  int tab;       // byte offset of the slot → source-offset table (after the two stages)
  int B;         // images
  int dbg;       // tools/halo_ablate.py timing ablations (YM_HALO_DBG): bit 0 no DMA, bit 1 no MFMA; 0 in production
};

template <int S>
__device__ __forceinline__ int tap_off(int tap, int pitch) {
  const int ky = tap / 3, kx = tap - 3 * ky;
  if constexpr (S == 1) return ky * pitch + kx;
  else return ky * 2 * pitch + (kx == 1 ? pitch : (kx >> 1));  // kx 0: even column x, 1: odd column x, 2: even x + 1
}

// chunk position swizzle of an item (see the header comment)
template <int CC8>
__device__ __forceinline__ int swz(int item) {
  if constexpr (CC8 == 4) return (item >> 2) & 3;
  else return (item >> 3) & 1;
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (a scalar jump table; vmcnt takes an immediate)
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
template <int N = 0>
__device__ __forceinline__ void wait_vm_rt(int n) {
  if constexpr (N < 32) {
    if (n == N) {
      wait_vm<N>();
      return;
    }
    wait_vm_rt<N + 1>(n);
  } else {
    wait_vm<0>();  // beyond the table: drain everything (correct, only slower)
  }
}

constexpr int MAXI = 16;  // input DMA wave-instructions per wave and stage (geometries beyond are not launched)

template <typename OutT, int S, int WM, int MB, int WN, int NB, int CC, int NBUF>
__global__ __launch_bounds__(256) void conv_halo(const ConvArgs a, const HaloGeom g) {
  static_assert(WM * WN == 4, "four waves");
  constexpr int CC8 = CC / 8;          // 16-byte chunks per item
  constexpr int BN = WN * NB * 32;     // output channels per workgroup
  constexpr int TMP = WM * MB * 32;    // output pixel slots per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (g.dbg & 96) return;  // ablation 32 / 64: empty kernel with no / the full LDS allocation (launch cost)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hl = lane >> 5;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // neighbouring row tiles (shared halo rows) on one XCD
  const int tn = vb % a.tiles_n;
  const int rest = vb / a.tiles_n;
  const int ty = rest % g.tiles_y, b = rest / g.tiles_y;
  const int r0 = ty * g.TH;
  const int Cin = a.C0;
  (void)TMP;

  // ---- epilogue operands first (their latency hides behind the K loop)
  f32x4 bias4[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = tn * BN + wn * (NB * 32) + nb * 32 + 8 * q + 4 * hl;
      bias4[nb][q] = n < a.N ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // this lane's pixel of each 32-pixel block: tap-(0,0) input slot, output position
  int pslot[MB], oy[MB], ox[MB];
  bool pok[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int p = 32 * (wm * MB + mb) + l32;
    const int t = ym_div(p, a.fd_w), x = p - t * a.Wo;
    oy[mb] = r0 + t;
    ox[mb] = x;
    pok[mb] = t < g.TH && r0 + t < a.Ho;
    pslot[mb] = pok[mb] ? (S == 1 ? t * g.pitch + x : 4 * t * g.pitch + x) : 0;
  }

  // residual (Bottleneck shortcut) operands, also loaded before the K loop; zeros without a residual
  f16x4 res4[MB][NB][4];
  const f16* res = static_cast<const f16*>(a.res);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const size_t rbase = (size_t)(b * a.r_P + oy[mb] * a.Wo + ox[mb]) * a.r_ctot + a.r_coff;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = tn * BN + wn * (NB * 32) + nb * 32 + 8 * q + 4 * hl;
        res4[mb][nb][q] = (res && pok[mb] && n0 < a.N) ? *reinterpret_cast<const f16x4*>(res + rbase + n0)
                                                       : f16x4{0, 0, 0, 0};
      }
  }

  // ---- slot → source element offset table of this tile's input rows (-1: halo / padding = zeros)
  int* tab = reinterpret_cast<int*>(smem + g.tab);
  const int iy0 = r0 * S - 1;
  for (int s = tid; s < g.npad; s += 256) {
    int off = -1;
    if (s < g.nslot && !(g.dbg & 4)) {
      int i, ix;
      if constexpr (S == 1) {
        i = s / g.pitch;
        ix = s - i * g.pitch - 1;
      } else {
        i = s / (2 * g.pitch);
        const int rem = s - i * 2 * g.pitch;
        ix = rem < g.pitch ? 2 * rem - 1 : 2 * (rem - g.pitch);
      }
      const int iy = iy0 + i;
      if ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win)
        off = (b * a.s0_P + iy * a.Win + ix) * a.s0_ctot + a.s0_coff;
    }
    tab[s] = off;
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.src0), 0,
                                                                       (int)(a.s0_elems * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0,
                                                                      (int)((long)a.N * a.Kpad * 2), 0x00020000);
  // This wave's DMA wave-instructions of a stage (k = wave, wave + 4, ...) and their source byte offsets at channel
  // 0 — the same for every stage up to + 2·c0 — computed once, so a stage's DMAs issue back to back.
  const int ID = g.npad * CC8 / 64;      // input DMA wave-instructions per stage
  constexpr int WD = 9 * BN * CC8 / 64;  // weight DMA wave-instructions per stage
  constexpr int NWW = (WD + 3) / 4;      // per wave (the last ones of some waves are absent)
  const int cl = lane % CC8;             // this lane's stored chunk position
  unsigned woff[NWW], xoff[MAXI];
#pragma unroll
  for (int u = 0; u < NWW; ++u) {
    const int k = wave + 4 * u;
    const int item = (k * 64 + lane) / CC8;  // tap * BN + n
    const int tap = item / BN, n = item % BN;
    const int nn = tn * BN + n;
    woff[u] = (k < WD && nn < a.N) ? (unsigned)(nn * a.Kpad + tap * Cin + 8 * (cl ^ swz<CC8>(n))) * 2u : OOB;
  }
#pragma unroll
  for (int u = 0; u < MAXI; ++u) {
    const int k = wave + 4 * u;
    const int p = (k * 64 + lane) / CC8;
    const int t = k < ID ? tab[p] : -1;
    xoff[u] = t >= 0 ? (unsigned)(t + 8 * (cl ^ swz<CC8>(p))) * 2u : OOB;
  }
  const int nw_w = (WD - wave + 3) / 4, nw_x = (ID - wave + 3) / 4;  // this wave's counts
  // DMA v of this wave's per-stage list (weights first, then input), for stage st into buffer buf
  auto issue_one = [&](int v, int st, int buf) {
    if (g.dbg & 1) return;
    char* sw = smem + buf * g.stage;
    const unsigned c2 = 2u * st * CC;
    if (v < NWW) {
      if (v < nw_w) dma16(rw, sw + (wave + 4 * v) * 1024, woff[v] == OOB ? OOB : woff[v] + c2);
    } else {
      const int u = v - NWW;
      if (u < nw_x) dma16(rs0, sw + g.wbytes + (wave + 4 * u) * 1024, xoff[u] == OOB ? OOB : xoff[u] + c2);
    }
  };
  constexpr int NV = NWW + MAXI;
  auto issue = [&](int st, int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) issue_one(v, st, buf);
  };
  const int ndma = nw_w + nw_x;  // DMA wave-instructions this wave issues per stage

  f32x16 acc[MB][NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][nb][r] = 0.f;

  // the MFMAs of one stage; the next stage's DMAs (st2 >= 0) are issued between the taps, PV per tap, so their
  // issue cost overlaps the matrix pipe instead of preceding it
  constexpr int PV = (NV + 8) / 9;
  auto compute = [&](int buf, int st2, int buf2) {
    const char* sw = smem + buf * g.stage;
    const char* sx = sw + g.wbytes;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = tap_off<S>(tap, g.pitch);
      if (g.dbg & 2) {  // ablation: no LDS reads / MFMAs (the DMAs of the next stage still issue)
        if (st2 >= 0)
          for (int i = 0; i < PV; ++i)
            if (tap * PV + i < NV) issue_one(tap * PV + i, st2, buf2);
        continue;
      }
#pragma unroll
      for (int k2 = 0; k2 < CC8 / 2; ++k2) {
        const int c = 2 * k2 + hl;
        f16x8 xb[MB], wa[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const int n = wn * (NB * 32) + nb * 32 + l32;
          wa[nb] = *reinterpret_cast<const f16x8*>(sw + ((tap * BN + n) * CC8 + (c ^ swz<CC8>(n))) * 16);
        }
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          const int ps = pslot[mb] + toff;
          xb[mb] = *reinterpret_cast<const f16x8*>(sx + (ps * CC8 + (c ^ swz<CC8>(ps))) * 16);
        }
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[nb], xb[mb], acc[mb][nb], 0, 0, 0);
      }
      if (st2 >= 0) {
#pragma unroll
        for (int i = 0; i < PV; ++i)
          if (tap * PV + i < NV) issue_one(tap * PV + i, st2, buf2);
      }
    }
  };

  const int nst = (g.dbg & 16) ? 0 : Cin / CC;  // ablation 16: no K loop at all
  if constexpr (NBUF == 2) {
    issue(0, 0);
    for (int st = 0; st < nst; ++st) {
      wait_vm0();     // this wave's DMAs of stage st have landed ...
      raw_barrier();  // ... and every wave's; every wave is done reading the buffer stage st+1 refills
      compute(st & 1, st + 1 < nst ? st + 1 : -1, (st + 1) & 1);
    }
  } else {  // three buffers: two stages of DMAs in flight behind the MFMAs
    issue(0, 0);
    if (nst > 1) issue(1, 1);
    for (int st = 0; st < nst; ++st) {
      if (st + 1 < nst) wait_vm_rt(ndma);  // stage st landed: only stage st+1's DMAs still outstanding
      else wait_vm0();
      raw_barrier();  // every wave's stage st landed; every wave is done with compute(st - 1)
      compute(st % 3, st + 2 < nst ? st + 2 : -1, (st + 2) % 3);
    }
  }

  // ---- epilogue: lane holds channels nbase + 8q + 4hl + {0..3} (q = 0..3) of pixel (oy, ox) per block; stores
  // only (the residuals were loaded before the K loop: a load after a store to a possibly aliasing address would
  // make the compiler drain every store)
  OutT* __restrict__ dst = static_cast<OutT*>(a.dst);
  wait_vm0();  // (already true after the last stage; tells the compiler so on every path)
  if (g.dbg & 8) return;  // ablation: no epilogue stores
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    if (!pok[mb]) continue;
    const size_t obase = (size_t)(b * a.d_P + a.d_pixoff + oy[mb] * a.d_W + ox[mb]) * a.d_ctot + a.d_coff;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = tn * BN + wn * (NB * 32) + nb * 32 + 8 * q + 4 * hl;
        if (n0 >= a.N) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = acc[mb][nb][4 * q + r] + bias4[nb][q][r];
          v[r] = (a.act ? ym_silu_fast(x) : x) + (float)res4[mb][nb][q][r];
        }
        if constexpr (sizeof(OutT) == 2)
          *reinterpret_cast<f16x4*>(dst + obase + n0) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
        else
          *reinterpret_cast<f32x4*>(dst + obase + n0) = f32x4{v[0], v[1], v[2], v[3]};
      }
  }
}

// (id, S, WM, MB, WN, NB, CC, NBUF): ids 0.. of this family, appended to the conv config space of csrc/ym_conv.hip.
// Tile = WM·MB·32 pixel slots (TH = that / Wo full output rows) x WN·NB·32 output channels; NBUF LDS stages.
#define YM_HALO_CFGS(X)                                                                                       \
  X(0, 1, 2, 5, 2, 1, 32, 2) X(1, 1, 1, 5, 4, 1, 16, 3) X(2, 1, 2, 5, 2, 2, 16, 2) X(3, 1, 2, 4, 2, 1, 16, 3)  \
  X(4, 1, 4, 2, 1, 1, 32, 3) X(5, 1, 4, 5, 1, 1, 16, 3) X(6, 1, 2, 5, 2, 1, 16, 3) X(7, 1, 4, 5, 1, 1, 32, 2)  \
  X(8, 2, 1, 5, 4, 1, 16, 2) X(9, 2, 2, 5, 2, 1, 16, 3) X(10, 2, 4, 5, 1, 1, 16, 3) X(11, 2, 2, 4, 2, 1, 16, 3)
constexpr int kNumHalo = 12;

constexpr int kMaxLds = 160 * 1024;

// Tile geometry of a launch, or false when the shape does not fit this variant.
bool halo_geom(const ConvArgs& a, int S, int TMP, int BN, int CC, int NBUF, HaloGeom& g) {
  int TH = TMP / a.Wo;
  if (TH < 1) return false;
  if (TH > a.Ho) TH = a.Ho;
  g.TH = TH;
  g.tiles_y = (a.Ho + TH - 1) / TH;
  const int rows = (TH - 1) * S + 3;
  if (S == 1) {
    g.pitch = a.Wo + 16;  // ≡ Wo (mod 16), >= Win + 2
    g.nslot = rows * g.pitch;
  } else {
    int p = a.Wo + 1;  // >= Wo + 1 (even column x + 1), 4 p ≡ Wo (mod 16) when possible
    if (a.Wo % 4 == 0)
      while ((4 * p - a.Wo) % 16) ++p;
    g.pitch = p;
    g.nslot = rows * 2 * p;
  }
  const int CC8 = CC / 8, per = 64 / CC8;  // slots per DMA wave-instruction
  g.npad = (g.nslot + per - 1) / per * per;
  g.wbytes = 9 * BN * CC * 2;
  g.stage = g.wbytes + g.npad * CC * 2;
  g.tab = NBUF * g.stage;
  g.B = a.M / (a.Ho * a.Wo);
  static const int dbg = [] {
    const char* e = getenv("YM_HALO_DBG");
    return e ? atoi(e) : 0;
  }();
  g.dbg = dbg;
  if (g.npad * CC8 / 64 > 4 * MAXI) return false;  // more input DMAs per wave than the kernel holds offsets for
  return g.tab + g.npad * 4 <= kMaxLds;
}

template <typename OutT, int S, int WM, int MB, int WN, int NB, int CC, int NBUF>
hipError_t launch(ConvArgs a, hipStream_t st) {
  if (a.s != S || a.C0 % CC) return hipErrorInvalidValue;
  HaloGeom g;
  constexpr int BN = WN * NB * 32;
  if (!halo_geom(a, S, WM * MB * 32, BN, CC, NBUF, g)) return hipErrorInvalidValue;
  a.tiles_n = (a.N + BN - 1) / BN;
  const long grid = (long)g.B * g.tiles_y * a.tiles_n;
  // a K loop shorter than the ring touches only its first stages: allocate those (more workgroups per CU)
  const int nst = a.C0 / CC, used = nst < NBUF ? nst : NBUF;
  if (used < NBUF) {
    g.tab = used * g.stage;
  }
  const size_t lds = (g.dbg & 32) ? 0 : (size_t)g.tab + (size_t)g.npad * 4;
  hipLaunchKernelGGL((conv_halo<OutT, S, WM, MB, WN, NB, CC, NBUF>), dim3(grid), dim3(256), lds, st, a, g);
  return hipGetLastError();
}

template <typename OutT>
hipError_t dispatch(const ConvArgs& a, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, s, wm, mb, wn, nb, cc, nbuf) \
  case id: return launch<OutT, s, wm, mb, wn, nb, cc, nbuf>(a, st);
    YM_HALO_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

}  // namespace

int ym_conv_halo_num_cfgs() { return kNumHalo; }

// Host-side applicability: f16 plans; 3x3, pad 1, stride 1 or 2, one plain source (no concat / upsample), Cin a
// multiple of the chunk, 4-aligned output channel slices (8-byte stores), element offsets < 2^30 (byte offsets of
// the buffer descriptors stay < 2^31).
hipError_t ym_launch_conv_halo(int out_f32, const ConvArgs& a, int i, hipStream_t st) {
  if (i < 0 || i >= kNumHalo) return hipErrorInvalidValue;
  if (a.k != 3 || a.pad != 1 || a.src1 || a.up0 || a.w2 || a.shuffle || a.raw || a.nchw || !a.src0)
    return hipErrorInvalidValue;
  if ((a.N & 3) || (a.d_ctot & 3) || (a.d_coff & 3) || (a.s0_ctot & 7) || (a.s0_coff & 7)) return hipErrorInvalidValue;
  if (a.res && ((a.r_ctot & 3) || (a.r_coff & 3))) return hipErrorInvalidValue;
  if (a.Kpad < 9 * a.C0 || a.C0 != 8 * a.Cin8) return hipErrorInvalidValue;
  const long lim = 0x3FFFFFF0L;
  if ((long)a.N * a.Kpad > lim || a.s0_elems > lim) return hipErrorInvalidValue;
  return out_f32 ? dispatch<float>(a, i, st) : dispatch<f16>(a, i, st);
}
