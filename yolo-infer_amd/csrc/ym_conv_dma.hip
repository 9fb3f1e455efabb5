// LDS-DMA implicit-GEMM convolution for gfx950 with in-launch split-K — the fp16 conv hot path, second generation.
//
// Same GEMM as csrc/ym_conv.hip (D[n][m] = Σ_k W[n][k]·X[k][m], n = output channel on the MFMA rows, m = output pixel on
// the columns, k = (ky, kx, c) so an 8-element K chunk is 8 channels of one input pixel), built for the two regimes
// that cost the first-generation kernels most on YOLO11 shapes:
//  * operands stream global → LDS with `buffer_load_dwordx4 … lds` (LDS-DMA: no VGPR staging, no ds_write pass)
//    into a 4-deep ring of 64-deep K stages, one raw barrier per stage and a counted `s_waitcnt vmcnt`, so three
//    stages of loads are in flight behind the MFMAs (a stage's load latency, not its MFMAs, sets the pace here).  The implicit-im2col gather is per lane (each lane
//    computes its own pixel/tap byte offset); 3x3 zero padding, K tails and M/N tails are out-of-range buffer offsets,
//    which the DMA turns into zeros in LDS — no branches in the load path;
//  * LDS image: row = one pixel (or one weight row) × 64 K = 128 B; chunk c of row r sits at slot c ^ ((r >> 1) & 7),
//    which makes the 16-lane groups of every ds_read_b128 fragment read hit 16 distinct 16-byte bank groups;
//    the swizzle is applied on the SOURCE side (the DMA destination is lane-linear);
//  * small-M deep layers (20x20 / 40x40 maps: a few hundred pixels per image, K up to 4608) are bound by the serial
//    chain of K stages, not by MFMA or HBM: SPLIT workgroups share one output tile, each takes a contiguous K range,
//    writes its fp32 partial tile (a "slab") with write-through (sc1) stores, and the last to arrive at the tile's
//    counter sums the slabs (sc1 loads) and runs the epilogue — the sc1 hand-off of cdna_hip_programming.md §6
//    Guideline 16: no release fence, whose L2 write-back (the previous layers' dirty activations) cost ~2 µs per
//    workgroup, and no L1 invalidate.
// Epilogue as in ym_conv.hip: + folded-BN bias, SiLU, + residual, channel-slice store (zero-copy concat), fp32
// anchor-major Detect rows, 2x2 pixel shuffle (Proto ConvTranspose2d).
#include <type_traits>

#include "ym_common.h"
#include "ym_quant.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifdef YM_DMA_STAMPS  // tools/dma_probe.hip: cycle stamps of workgroup 0, wave 0 (never built into the library)
__device__ unsigned long long* ym_dma_stamps;
#define YM_STAMP(i)                                                                          \
  do {                                                                                       \
    if (blockIdx.x == 0 && threadIdx.x == 0) ym_dma_stamps[(i)] = __builtin_readcyclecounter(); \
  } while (0)
#else
#define YM_STAMP(i) \
  do {              \
  } while (0)
#endif

namespace {

constexpr int DK = 64;                    // K per stage
typedef Q8<false> Q8S;                    // the int8 scheme of csrc/ym_quant.h (Q8 mode of conv_dma_body)
constexpr unsigned OOB = 0x80000000u;     // byte offset past num_records: the DMA deposits zeros

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// a DMA byte offset, or OOB (the DMA deposits zeros) where !ok: branch-free bit select — a ?: here compiled to an
// exec-mask branch around the address arithmetic before every DMA instruction
__device__ __forceinline__ unsigned oob_sel(bool ok, unsigned off) {
  const unsigned m = 0u - (unsigned)ok;
  return (off & m) | (OOB & ~m);
}

__device__ __forceinline__ void raw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, 0, 0, 0);
}

template <typename OutT> struct Store4;
template <> struct Store4<f16> {
  static __device__ __forceinline__ void st(f16* p, const float* v) {
    *reinterpret_cast<f16x4*>(p) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
  }
};
template <> struct Store4<float> {
  static __device__ __forceinline__ void st(float* p, const float* v) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  }
};
template <> struct Store4<P2> {
  static __device__ __forceinline__ void st(P2* p, const float* v) { ym_p2_store4(p, v); }
};

// A workgroup = KG groups of 2x2 waves (256·KG threads).  Every wave group covers the whole BM x BN tile — a wave
// owns (BM/2) pixels x (BN/2) channels = TM x TN blocks of 32x32 — and takes 4/KG of each stage's four 16-deep k
// sub-steps; the groups' partial tiles are summed once through LDS after the K loop.  KG = 2 puts two waves on every
// SIMD, so one wave's LDS reads, barrier and DMA issue overlap the other's MFMAs (the small-M layers are latency-bound
// with one wave per SIMD: tools/dma_probe.hip).
// KIND 1: 1x1 stride 1 (two sources, upsampled first source); KIND 3: 3x3, any Cin (per-lane tap walk);
// KIND 4: 3x3 with Cin % 64 == 0 — every 64-deep stage is ONE tap, so the tap, its pixel offset and the channel
// block are wave-uniform scalars and a DMA address is one add onto a per-row base, validity one bit of a 9-bit
// per-row tap mask.
// NSTAGE: LDS ring depth (NSTAGE - 1 stages of loads in flight); 3 for the 256 x 128 tiles (48 KB per stage), 2
// (double buffer) for the 256-deep stages.
// SUB: 64-deep K sub-stages per stage (one barrier, one LDS-read latency and one wait per SUB x 64 of K): the small-M
// layers' K loops are chains of per-stage fixed costs, which SUB 2 halves; launched only where every split's K range
// is whole stages (no partial stage: every stage issues exactly NL DMA instructions, tools/check_dma_asm.py)
// X3 (x3 plans): activations in the pair layout and weights in pair-chunk rows, both fetched by the same DMA as fp16
// tensors of twice the channels (storage chunk 2j = hi of logical chunk j, 2j + 1 = its lo), so a 16-deep k sub-step
// s holds hi_s (lane half 0) and lo_s (lane half 1) of one logical chunk.  Per two sub-steps (s, s+1) three MFMAs
// form the split product hi·hi + hi·lo + lo·hi of both chunks: A = [w_hi_s | w_hi_s] with the natural B (w_hi·x_hi +
// w_hi·x_lo), the same for s+1, and A = [w_lo_s | w_lo_s+1] with B = [x_hi_s | x_hi_s+1] (w_lo·x_hi of both) — only
// the chunk each lane half reads from LDS changes, the swizzle stays conflict-free.
// FUSE (x3 plans; a fused conv -> 1x1 pair, ConvArgs::w2 with k2 == 1, yolomi/arch.py fuse_pairs): the tile holds
// every output channel of the first conv (N <= BN), so after its K loop the activated tile is split hi / lo exactly as
// its stored pair-layout tensor would be and written into the idle stage ring in the staging layout of the pixel
// operand; W2 (prefetched into registers at the start, its latency hidden by the K loop) goes into an LDS slot in the
// weight-operand layout, and the second GEMM (K = the first conv's N) runs as extra ring stages — the same fragment
// reads and split MFMAs — before the epilogue stores the second conv's output.  The intermediate never reaches HBM and
// the pair is one launch (the split pair wrote and read it back: model.1+cv1, the Detect cv2.l.1 -> cv2.l.2 chains).
// The workgroup body (output tile `bid` of the launch's tile map; LDS from the caller) — the conv_dma kernel below, or
// one work item of the persistent chain kernel conv_dma_chain.  Returns true when this workgroup stored the tile's
// final output (false: a padding workgroup, or a split-K partial that another workgroup of the tile reduced); the
// value is the same in every wave.  SC1OUT: the epilogue stores write through (sc1), for a consumer in the same launch.
template <int NSTAGE, int SB, int BN, int KS2, bool Q8 = false>
struct DmaSmem {
  static constexpr int ring = NSTAGE * SB + 16 + 256 + (Q8 ? 1024 : 0);  // Q8: + the 256-entry post table
  static constexpr int w2 = KS2 ? KS2 * BN * 128 : 16;
};
// Q8 (round 6): the int8 PTQ plan on the same kernel — an int8 tensor is staged as the fp16 tensor of half its
// channels (a 16-byte chunk = 16 int8 channels, the same fragment bytes per lane), every 16-deep fp16 sub-step is one
// v_mfma_i32_32x32x32_i8 with exact int32 sums (so tiles, K splits and wave groups never change the result), and the
// epilogue is conv_i8's quantized one (csrc/ym_conv_i8.hip; + the padding-tap correction of ConvArgs::wtap).
template <typename OutT, int BM, int BN, int KIND, int SPLIT, int KG, int NSTAGE, int SUB, bool X3 = false,
          bool FUSE = false, bool SC1OUT = false, bool Q8 = false>
__device__ __forceinline__ bool conv_dma_body(const ConvArgs& a, const int bid, char* smem, char* w2s) {
  static_assert(!Q8 || (!X3 && !FUSE && !SC1OUT), "int8: the plain GEMM only");
  typedef typename std::conditional<Q8, i32x16, f32x16>::type ACC;
  constexpr int NW = 4 * KG;
  constexpr int TM = BM / 64, TN = BN / 64;
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "DMA groups must divide over the waves");
  constexpr int GB = BM / 8 / NW, GA = BN / 8 / NW;  // DMA wave-instructions per stage per wave (8 rows x 128 B)
  constexpr int NL = (GA + GB) * SUB;                // DMA wave-instructions per stage per wave
  constexpr int SBS = (BM + BN) * 128;               // bytes per 64-deep sub-stage
  constexpr int SB = SUB * SBS;                      // bytes per stage
  constexpr int NREG = TM * TN * 16;
  constexpr int SPW = 4 / KG;                        // 16-deep k sub-steps per wave per stage
  constexpr int NACC = TM * TN == 1 && SPW >= 2 ? 2 : 1;  // one 32x32 block per wave: alternate two accumulators
  // smem: NSTAGE * SB ring bytes + split-K flag, L2 warm-up scratch
  // FUSE: the second GEMM's K (the first conv's BN channels) in 64-deep storage sub-stages, W2 [KS2][BN rows][128 B]
  constexpr int KS2 = FUSE ? (X3 ? 2 : 1) * BN / 64 : 0;
  static_assert(!FUSE || (SPLIT == 1 && NSTAGE * SB >= KS2 * BM * 128), "fused pair: whole-K tiles, T fits the ring");
  constexpr int W2P = FUSE ? KS2 * BN * 8 / (256 * KG) : 1;  // 16-byte W2 pieces per thread
  static_assert(!FUSE || (KS2 * BN * 8) % (256 * KG) == 0, "W2 pieces divide over the threads");
  // BN 128: W2 is 64 KB, 16 pieces per thread — too many registers to hold through the K loop; loaded after it
  constexpr bool W2LATE = W2P > 8;

  YM_STAMP(0);
  // wid in an SGPR (uniform per wave): every LDS-DMA destination (M0) derived from it is then scalar arithmetic,
  // not a VALU address moved to M0 by v_readfirstlane before each DMA instruction
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wid >> 2, wq = wid & 3;
  const int wm = wq & 1, wn = wq >> 1;
  const int l32 = lane & 31, h = lane >> 5;
  // tile map: every N tile and every K split of pixel tile tm share bid % 8 = one XCD (its L2 holds the pixels and
  // the split's slabs), and each XCD owns one contiguous run of pixel tiles, so the image rows a 3x3 tile shares with
  // its neighbours are fetched into one L2; padding workgroups (tm beyond M) exit before touching a counter
  int rest = bid >> 3;
  const int sp = rest % SPLIT;
  rest /= SPLIT;
  const int rq = ym_div(rest, a.fd_tn);  // rest / tiles_n
  const int tn = rest - rq * a.tiles_n;
  const int tm = (bid & 7) * a.tm_per_xcd + rq;  // (a.tm_per_xcd = gridDim.x / (8 SPLIT tiles_n))
  if (tm * BM >= a.M) return false;

  // ---- epilogue operands first (bias, residual; wave group 0 runs the epilogue): their latency hides behind the
  // K loop.  They are older than every DMA, so the counted vmcnt waits below stay exact (loads retire in order).
  int ep_m[TM];
  size_t ep_obase[TM];
  f32x4 bias4[TN][4];
  typedef typename std::conditional<X3, f32x4, f16x4>::type RV;  // residual (x3: hi + lo)
  RV res4[TM][TN][4];
  const f16* res = static_cast<const f16*>(a.res);
  const P2* resp = static_cast<const P2*>(a.res);
  constexpr int XS = X3 ? 2 : 1;  // fp16 storage elements per logical channel
  const int s0_ctot = XS * a.s0_ctot, s0_coff = XS * a.s0_coff, s1_ctot = XS * a.s1_ctot, s1_coff = XS * a.s1_coff;
  const int C0s = XS * a.C0;
  // FUSE: the epilogue writes the SECOND conv (N2 channels, bias2); bias4a holds the first conv's bias for the tile T
  const int NOUT = FUSE ? a.N2 : a.N;
  f32x4 bias4a[FUSE ? TN : 1][4];
  u32x4 w2r[W2LATE ? 1 : W2P];
  if constexpr (FUSE && !W2LATE) {
#pragma unroll
    for (int u = 0; u < W2P; ++u) {  // piece p: row n2 = p / (8 KS2), storage chunk cs = p % (8 KS2) of W2's K
      const int p = tid + 256 * KG * u, n2 = p / (8 * KS2), cs = p % (8 * KS2);
      const bool ok = n2 < a.N2 && 8 * cs < a.Kpad2;
      // (unconditional load of a clamped address; the out-of-range pieces are zeroed when they go to LDS, after the
      // K loop: a select here would make the compiler wait for the load on the spot)
      w2r[u] = ym_gld<u32x4>(static_cast<const f16*>(a.w2) + (ok ? (size_t)n2 * a.Kpad2 + 8 * cs : 0));
    }
  }
  if constexpr (Q8) {  // the epilogue's requantisation table, staged once (the K loop's barriers order it)
    float* post = reinterpret_cast<float*>(smem + NSTAGE * SB + 16 + 256);
    for (int i = tid; i < 256; i += 256 * KG) post[i] = a.q->post[i];
  }
  if (kg == 0 && !Q8) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = tn * BN + wn * (BN / 2) + 32 * j + 8 * q + 4 * h;
        const float* bsrc = FUSE ? a.bias2 : a.bias;
        bias4[j][q] = n < NOUT ? *reinterpret_cast<const f32x4*>(bsrc + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (FUSE)
          bias4a[j][q] = n < a.N ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = tm * BM + wm * (BM / 2) + 32 * i + l32;
      ep_m[i] = m;
      const int mm = m < a.M ? m : 0;
      const int b = ym_div(mm, a.fd_hw), rem = mm - b * (a.Ho * a.Wo);
      const int oy = ym_div(rem, a.fd_w), ox = rem - oy * a.Wo;
      const int pix = a.shuffle ? (2 * oy) * a.d_W + 2 * ox : oy * a.d_W + ox;
      ep_obase[i] = (size_t)(b * a.d_P + a.d_pixoff + pix) * a.d_ctot + a.d_coff;
      const size_t rbase = res ? (size_t)(b * a.r_P + oy * a.Wo + ox) * a.r_ctot + a.r_coff : 0;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = tn * BN + wn * (BN / 2) + 32 * j + 8 * q + 4 * h;
          if constexpr (X3) {
            float rv[4] = {0.f, 0.f, 0.f, 0.f};
            if (res && m < a.M && n < a.N) ym_p2_load4(resp + rbase + n, rv);
            res4[i][j][q] = f32x4{rv[0], rv[1], rv[2], rv[3]};
          } else {
            res4[i][j][q] = (res && m < a.M && n < a.N) ? *reinterpret_cast<const f16x4*>(res + rbase + n)
                                                         : f16x4{0, 0, 0, 0};
          }
        }
    }
  }

  // ---- DMA lanes: instruction-row rr = lane >> 3, LDS slot lane & 7, so this lane fetches chunk c of its row with
  // c = slot ^ ((row >> 1) & 7); rows of wave wid's groups are (wid + NW gi) * 8 + rr, hence (row >> 1) & 7 =
  // ((wid & 1) << 2) | (rr >> 1) for every group of this wave (NW even): one chunk index per lane.
  const int rr = lane >> 3;
  const int c = (lane & 7) ^ (((wid & 1) << 2) | (rr >> 1));
  // exact extents: a K-tail chunk past the end of a buffer reads zeros, inside it a finite activation (times a
  // zero-padded weight) — so no per-lane K-tail test is needed, and none may be added: a per-lane condition around
  // the DMA lets the compiler split it into two instructions for mixed waves, which breaks the counted vmcnt below
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.src0), 0,
                                                                       (int)(a.s0_elems * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.src1 ? a.src1 : a.src0), 0, (int)((a.src1 ? a.s1_elems : a.s0_elems) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0,
                                                                      (int)((long)a.N * a.Kpad * 2), 0x00020000);
  // pixel rows of this lane's B groups
  int pbase0[GB], pbase1[GB], piy[GB], pix[GB];
  unsigned tmask[GB];  // KIND 4: bit t = tap t of the 3x3 window lies inside the image (0 for an M-tail row)
#pragma unroll
  for (int gi = 0; gi < GB; ++gi) {
    const int m = tm * BM + (wid + NW * gi) * 8 + rr;
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    const int b = ym_div(mm, a.fd_hw), rem = mm - b * (a.Ho * a.Wo);
    const int oy = ym_div(rem, a.fd_w), ox = rem - oy * a.Wo;
    tmask[gi] = 0;
    if constexpr (KIND == 1) {
      const int sy = a.up0 ? (oy >> 1) : oy, sx = a.up0 ? (ox >> 1) : ox;
      pbase0[gi] = ok ? (b * a.s0_P + sy * a.s0_W + sx) * s0_ctot + s0_coff : -1;
      // (row bases stay >= 0 for valid rows: -1 marks an M-tail row, so the -C0 of the second source's channel
      // index is applied per stage, not folded in here)
      pbase1[gi] = ok && a.src1 ? (b * a.s1_P + oy * a.Win + ox) * s1_ctot + s1_coff : -1;
      piy[gi] = pix[gi] = 0;
    } else if constexpr (KIND == 3) {
      pbase0[gi] = ok ? b * a.s0_P : -1;  // image pixel base
      pbase1[gi] = 0;
      piy[gi] = oy * a.s - 1;
      pix[gi] = ox * a.s - 1;
    } else {
      const int iy0 = oy * a.s - 1, ix0 = ox * a.s - 1;
      // element offset of this lane's chunk at the window's top-left pixel (may be negative: only in-image taps
      // are ever added to it)
      pbase0[gi] = (b * a.s0_P + iy0 * a.Win + ix0) * s0_ctot + s0_coff + c * 8;
      pbase1[gi] = 0;
      piy[gi] = pix[gi] = 0;
      unsigned mk = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int iy = iy0 + t / 3, ix = ix0 + t % 3;
        mk |= ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win) ? (1u << t) : 0u;
      }
      tmask[gi] = ok ? mk : 0u;
    }
  }
  int wbase[GA];
#pragma unroll
  for (int gi = 0; gi < GA; ++gi) {
    const int n = tn * BN + (wid + NW * gi) * 8 + rr;
    wbase[gi] = n < a.N ? n * a.Kpad + c * 8 : -1;
  }

  const int nst = a.Kpad / DK;
  const int k_lo = (nst * sp) / SPLIT, k_hi = (nst * (sp + 1)) / SPLIT;
  const int nk = (k_hi - k_lo) / SUB;  // stages (launch_dma: a multiple of SUB sub-stages)
  // KIND 3: tap / channel block of this lane's chunk at stage k_lo (chunk index k*8 + c);
  // KIND 4: the stage's tap (ky, kx) and channel block cb (wave-uniform)
  int tap = 0, cb = 0, ky = 0, kx = 0;
  if constexpr (KIND == 3) {
    const int idx = k_lo * 8 + c;
    tap = ym_div(idx, a.fd_cin8);
    cb = idx - tap * a.Cin8;
  } else if constexpr (KIND == 4) {
    tap = ym_div(k_lo * 8, a.fd_cin8);
    cb = k_lo * 8 - tap * a.Cin8;
    ky = tap / 3;
    kx = tap - ky * 3;
  }
  int kcur = k_lo;  // stage whose loads are issued next

  auto issue_sub = [&](char* sbase) {
    const int chunk = kcur * 8 + c;
    // B: pixels
    if constexpr (KIND == 1) {
      const bool second = a.src1 && kcur * DK >= C0s;  // wave-uniform (C0 % 64 == 0 when src1 is used)
#pragma unroll
      for (int gi = 0; gi < GB; ++gi) {
        const int pb = second ? pbase1[gi] : pbase0[gi];
        const unsigned off = oob_sel(pb >= 0, (unsigned)(pb + chunk * 8 - (second ? C0s : 0)) * 2u);
        dma16(second ? rs1 : rs0, sbase + (wid + NW * gi) * 1024, off);
      }
    } else if constexpr (KIND == 3) {
      const int ty = tap / 3, tx = tap - (tap / 3) * 3;
#pragma unroll
      for (int gi = 0; gi < GB; ++gi) {
        const int iy = piy[gi] + ty, ix = pix[gi] + tx;
        const bool ok = pbase0[gi] >= 0 && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        const unsigned off = oob_sel(ok, (unsigned)((pbase0[gi] + iy * a.Win + ix) * s0_ctot + s0_coff + cb * 8) * 2u);
        dma16(rs0, sbase + (wid + NW * gi) * 1024, off);
      }
      cb += 8;
      while (cb >= a.Cin8) { cb -= a.Cin8; ++tap; }
    } else {
      const int S = (ky * a.Win + kx) * s0_ctot + cb * 8;  // uniform
#pragma unroll
      for (int gi = 0; gi < GB; ++gi) {
        const unsigned off = oob_sel((tmask[gi] >> tap) & 1u, (unsigned)(pbase0[gi] + S) * 2u);
        dma16(rs0, sbase + (wid + NW * gi) * 1024, off);
      }
      cb += 8;
      if (cb == a.Cin8) {
        cb = 0;
        ++tap;
        if (++kx == 3) { kx = 0; ++ky; }
      }
    }
    // A: weights
#pragma unroll
    for (int gi = 0; gi < GA; ++gi) {
      const unsigned off = oob_sel(wbase[gi] >= 0, (unsigned)(wbase[gi] + kcur * DK) * 2u);
      dma16(rw, sbase + BM * 128 + (wid + NW * gi) * 1024, off);
    }
    ++kcur;
  };
  auto issue = [&](int slot) {
#pragma unroll
    for (int u = 0; u < SUB; ++u) issue_sub(smem + slot * SB + u * SBS);
  };
  // L2 warm-up (ConvArgs::pf, the latency-bound small-M layers): every line this workgroup's K range will stage is
  // requested ONCE up front by a 4-byte LDS-DMA into a scratch slot (the same per-lane addresses as the ring, so the
  // same zero-fill rules; no VGPR destination, so no compiler waits), all in flight together; the ring's stages then
  // find their lines in L2.  The counted vmcnt waits stay exact: these requests are older than every ring stage.
  if (a.pf) {
    const int s_tap = tap, s_cb = cb, s_ky = ky, s_kx = kx, s_k = kcur;
    char* scratch = smem + NSTAGE * SB + 16;
    for (int st = 0; st < nk * SUB; ++st) {
      const int chunk = kcur * 8 + c;
      if constexpr (KIND == 1) {
        const bool second = a.src1 && kcur * DK >= C0s;
#pragma unroll
        for (int gi = 0; gi < GB; ++gi) {
          const int pb = second ? pbase1[gi] : pbase0[gi];
          const unsigned off = pb >= 0 ? (unsigned)(pb + chunk * 8 - (second ? C0s : 0)) * 2u : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? rs1 : rs0, (lds_void_t*)scratch, 4, off, 0, 0, 0);
        }
      } else if constexpr (KIND == 3) {
        const int ty = tap / 3, tx = tap - (tap / 3) * 3;
#pragma unroll
        for (int gi = 0; gi < GB; ++gi) {
          const int iy = piy[gi] + ty, ix = pix[gi] + tx;
          const bool ok = pbase0[gi] >= 0 && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
          const unsigned off =
              ok ? (unsigned)((pbase0[gi] + iy * a.Win + ix) * s0_ctot + s0_coff + cb * 8) * 2u : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs0, (lds_void_t*)scratch, 4, off, 0, 0, 0);
        }
        cb += 8;
        while (cb >= a.Cin8) { cb -= a.Cin8; ++tap; }
      } else {
        const int S = (ky * a.Win + kx) * s0_ctot + cb * 8;
#pragma unroll
        for (int gi = 0; gi < GB; ++gi) {
          const unsigned off = (tmask[gi] >> tap) & 1u ? (unsigned)(pbase0[gi] + S) * 2u : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs0, (lds_void_t*)scratch, 4, off, 0, 0, 0);
        }
        cb += 8;
        if (cb == a.Cin8) {
          cb = 0;
          ++tap;
          if (++kx == 3) { kx = 0; ++ky; }
        }
      }
#pragma unroll
      for (int gi = 0; gi < GA; ++gi) {
        const unsigned off = wbase[gi] >= 0 ? (unsigned)(wbase[gi] + kcur * DK) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void_t*)scratch, 4, off, 0, 0, 0);
      }
      ++kcur;
    }
    tap = s_tap; cb = s_cb; ky = s_ky; kx = s_kx; kcur = s_k;
  }

  ACC acc[NACC][TM][TN];
#pragma unroll
  for (int u = 0; u < NACC; ++u)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[u][i][j][r] = 0;

  const int key = (l32 >> 1) & 7;
  // this wave's k sub-steps of the stage: fragment reads first, then the MFMAs (one LDS latency per stage)
  auto compute = [&](int slot) {
    if constexpr (X3) {
      static_assert(SPW % 2 == 0, "x3: a wave's k sub-steps come in pairs");
      // per sub-step pair (s, s+1): A'_s = w_hi_s on both lane halves, B_s natural; the same for s+1; A'' =
      // [w_lo_s | w_lo_s+1], B'' = [x_hi_s | x_hi_s+1]
      f16x8 fb[SUB][SPW / 2][3][TM], fa[SUB][SPW / 2][3][TN];
#pragma unroll
      for (int su = 0; su < SUB; ++su) {
        const char* sb = smem + slot * SB + su * SBS;
        const char* sa = sb + BM * 128;
#pragma unroll
        for (int u = 0; u < SPW / 2; ++u) {
          const int s = kg * SPW + 2 * u;
          const int ca[3] = {2 * s, 2 * s + 2, 2 * (s + h) + 1}, cbx[3] = {2 * s + h, 2 * s + 2 + h, 2 * (s + h)};
#pragma unroll
          for (int v = 0; v < 3; ++v) {
            const int offa = ((ca[v] ^ key) << 4) + l32 * 128, offb = ((cbx[v] ^ key) << 4) + l32 * 128;
#pragma unroll
            for (int i = 0; i < TM; ++i)
              fb[su][u][v][i] = *reinterpret_cast<const f16x8*>(sb + (wm * (BM / 2) + 32 * i) * 128 + offb);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              fa[su][u][v][j] = *reinterpret_cast<const f16x8*>(sa + (wn * (BN / 2) + 32 * j) * 128 + offa);
          }
        }
      }
#pragma unroll
      for (int su = 0; su < SUB; ++su)
#pragma unroll
        for (int u = 0; u < SPW / 2; ++u)
#pragma unroll
          for (int v = 0; v < 3; ++v)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
                acc[v % NACC][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[su][u][v][j], fb[su][u][v][i],
                                                                             acc[v % NACC][i][j], 0, 0, 0);
    } else {
      f16x8 fb[SUB][SPW][TM], fa[SUB][SPW][TN];
#pragma unroll
      for (int su = 0; su < SUB; ++su) {
        const char* sb = smem + slot * SB + su * SBS;
        const char* sa = sb + BM * 128;
#pragma unroll
        for (int u = 0; u < SPW; ++u) {
          const int s = kg * SPW + u;
          const int off = ((((2 * s + h) ^ key)) << 4) + l32 * 128;
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fb[su][u][i] = *reinterpret_cast<const f16x8*>(sb + (wm * (BM / 2) + 32 * i) * 128 + off);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fa[su][u][j] = *reinterpret_cast<const f16x8*>(sa + (wn * (BN / 2) + 32 * j) * 128 + off);
        }
      }
#pragma unroll
      for (int su = 0; su < SUB; ++su)
#pragma unroll
        for (int u = 0; u < SPW; ++u)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              if constexpr (Q8)
                acc[u % NACC][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
                    __builtin_bit_cast(i8x16, fa[su][u][j]), __builtin_bit_cast(i8x16, fb[su][u][i]),
                    acc[u % NACC][i][j], 0, 0, 0);
              else
                acc[u % NACC][i][j] =
                    __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[su][u][j], fb[su][u][i], acc[u % NACC][i][j], 0, 0, 0);
            }
    }
  };

  static_assert(NSTAGE >= 2 && NSTAGE <= 4, "ring depth");
#pragma unroll
  for (int s0 = 0; s0 < NSTAGE - 1; ++s0)
    if (nk > s0) issue(s0);
  YM_STAMP(1);
  for (int it = 0; it < nk; ++it) {
    // stage it is complete when at most the stages issued after it are outstanding (loads retire in order)
    if (it + NSTAGE - 2 < nk) wait_vm<(NSTAGE - 2) * NL>();
    else if (NSTAGE == 4 && it + 1 < nk) wait_vm<NL>();
    else wait_vm<0>();
    YM_STAMP(8 + 4 * (it & 63));
    raw_barrier();  // stage it is in LDS for every wave; every wave is done reading stage it-1's slot
    YM_STAMP(9 + 4 * (it & 63));
    if (it + NSTAGE - 1 < nk) issue((it + NSTAGE - 1) % NSTAGE);
    YM_STAMP(10 + 4 * (it & 63));
    compute(it % NSTAGE);
    YM_STAMP(11 + 4 * (it & 63));
  }
  YM_STAMP(2);
  if constexpr (NACC == 2) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[0][i][j] += acc[1][i][j];
  }
  // ---- wave groups 1..KG-1 hand their partial tiles to group 0 through the (now idle) stage ring
  if constexpr (KG > 1) {
    static_assert(NSTAGE * SB >= (KG - 1) * 4 * NREG * 64 * 4, "reduction area exceeds the ring");
    float* red = reinterpret_cast<float*>(smem);  // [(kg-1)][wq][NREG][64]
    __syncthreads();                              // every wave is past its last ds_read of the ring
    if (kg > 0) {
      float* d = red + ((size_t)((kg - 1) * 4 + wq) * NREG) * 64 + lane;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            // (an element copied out first: __builtin_bit_cast straight on a vector element miscompiled — round 6,
            // every KG 2 and split-K configuration of every plan returned wrong tiles until this was found)
            const auto x = acc[0][i][j][r];
            if constexpr (Q8) d[((i * TN + j) * 16 + r) * 64] = __int_as_float(x);
            else d[((i * TN + j) * 16 + r) * 64] = x;
          }
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int g = 1; g < KG; ++g) {
        const float* q = red + ((size_t)((g - 1) * 4 + wq) * NREG) * 64 + lane;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              if constexpr (Q8) acc[0][i][j][r] += __float_as_int(q[((i * TN + j) * 16 + r) * 64]);
              else acc[0][i][j][r] += q[((i * TN + j) * 16 + r) * 64];
            }
      }
    }
  }

  // ---- split-K: publish the partial tile write-through, the last arriver reduces (wave group 0 only holds the
  // tile; every thread still takes part in the workgroup barriers)
  if constexpr (SPLIT > 1) {
    const int tile = tm * a.tiles_n + tn;
    const __amdgpu_buffer_rsrc_t rsl =
        __builtin_amdgcn_make_buffer_rsrc(a.slab, 0, (int)(a.slab_cap < 0x7FFFFFF0L ? a.slab_cap : 0x7FFFFFF0L),
                                          0x00020000);
    constexpr int SC1 = 16;  // cache-policy aux bit: sc1 (write-through stores / L1-bypassing loads)
    const unsigned mine = (unsigned)(tile * SPLIT + sp) * (256u * NREG * 4u);
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int qq = (i * TN + j) * 4 + q;
            typedef typename std::conditional<Q8, i32x4, f32x4>::type V4;  // (whole-vector bit cast, see above)
            const V4 v{acc[0][i][j][4 * q], acc[0][i][j][4 * q + 1], acc[0][i][j][4 * q + 2], acc[0][i][j][4 * q + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsl,
                                                   mine + (qq * 256u + tid) * 16u, 0, SC1);
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    }
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem + NSTAGE * SB);
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == SPLIT - 1;
      if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    const bool last_arrival = *flag;
    if (!last_arrival || kg != 0) return last_arrival;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below the ticket
    // sum every slab (this workgroup's own included) in split order — bitwise-reproducible whichever split arrived
    // last; all slabs' loads are issued together (one memory latency, not SPLIT)
    f32x4 part[SPLIT][TM * TN * 4];
#pragma unroll
    for (int s2 = 0; s2 < SPLIT; ++s2) {
      const unsigned o = (unsigned)(tile * SPLIT + s2) * (256u * NREG * 4u);
#pragma unroll
      for (int qq = 0; qq < TM * TN * 4; ++qq)
        part[s2][qq] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsl, o + (qq * 256u + tid) * 16u,
                                                                                       0, SC1));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int qq = (i * TN + j) * 4 + q;
          if constexpr (Q8) {
            i32x4 v = __builtin_bit_cast(i32x4, part[0][qq]);
#pragma unroll
            for (int s2 = 1; s2 < SPLIT; ++s2) v += __builtin_bit_cast(i32x4, part[s2][qq]);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[0][i][j][4 * q + e] = v[e];
          } else {
            f32x4 v = part[0][qq];
#pragma unroll
            for (int s2 = 1; s2 < SPLIT; ++s2) v += part[s2][qq];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[0][i][j][4 * q + e] = v[e];
          }
        }
  }
  if constexpr (FUSE) {
    // ---- fused 1x1: T = the first conv's activated tile (exactly its stored split) in the ring, W2 in w2s, then
    // the second GEMM (all of its K sub-steps in wave group 0) into acc[0]
    __syncthreads();  // every wave is past its last read of the ring (and of the wave-group reduction area)
    char* T = smem;
    const int key = (l32 >> 1) & 7;
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f16x4 hv, lv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x = X3 ? ym_x3_pre(acc[0][i][j][4 * q + e], a.wsc, bias4a[j][q][e])
                                 : acc[0][i][j][4 * q + e] + bias4a[j][q][e];
              const float v = a.act ? (X3 ? ym_silu_x3(x) : ym_silu_fast(x)) : x;
              hv[e] = (f16)v;
              lv[e] = (f16)(v - (float)hv[e]);
            }
            const int row = wm * (BM / 2) + 32 * i + l32;
            const int jc = (wn * (BN / 2) + 32 * j + 8 * q) >> 3;  // tile-local logical chunk
            auto put = [&](int sc, f16x4 val) {                    // storage chunk sc of the second GEMM's K
              *reinterpret_cast<f16x4*>(T + (sc >> 3) * BM * 128 + row * 128 + (((sc & 7) ^ key) << 4) + 8 * h) = val;
            };
            if constexpr (X3) {
              put(2 * jc, hv);
              put(2 * jc + 1, lv);
            } else {
              put(jc, hv);
            }
          }
    }
#pragma unroll
    for (int u = 0; u < W2P; ++u) {
      const int p = tid + 256 * KG * u, n2 = p / (8 * KS2), cs = p % (8 * KS2);
      const bool ok = n2 < a.N2 && 8 * cs < a.Kpad2;
      u32x4 v;
      if constexpr (W2LATE)
        v = ym_gld<u32x4>(static_cast<const f16*>(a.w2) + (ok ? (size_t)n2 * a.Kpad2 + 8 * cs : 0));
      else
        v = w2r[u];
      *reinterpret_cast<u32x4*>(w2s + (cs >> 3) * BN * 128 + n2 * 128 + (((cs & 7) ^ ((n2 >> 1) & 7)) << 4)) =
          ok ? v : u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    if (kg != 0) return true;
    f32x16 acc2[NACC][TM][TN];
#pragma unroll
    for (int u = 0; u < NACC; ++u)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc2[u][i][j][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      const char* sb = T + ks * BM * 128;
      const char* sa = w2s + ks * BN * 128;
      if constexpr (X3) {
#pragma unroll
        for (int s = 0; s < 4; s += 2) {  // sub-step pairs (0, 1), (2, 3): the main loop's three split MFMAs
          const int ca[3] = {2 * s, 2 * s + 2, 2 * (s + h) + 1}, cbx[3] = {2 * s + h, 2 * s + 2 + h, 2 * (s + h)};
          f16x8 fb[3][TM], fa[3][TN];
#pragma unroll
          for (int v = 0; v < 3; ++v) {
            const int offa = ((ca[v] ^ key) << 4) + l32 * 128, offb = ((cbx[v] ^ key) << 4) + l32 * 128;
#pragma unroll
            for (int i = 0; i < TM; ++i)
              fb[v][i] = *reinterpret_cast<const f16x8*>(sb + (wm * (BM / 2) + 32 * i) * 128 + offb);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              fa[v][j] = *reinterpret_cast<const f16x8*>(sa + (wn * (BN / 2) + 32 * j) * 128 + offa);
          }
#pragma unroll
          for (int v = 0; v < 3; ++v)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
                acc2[v % NACC][i][j] =
                    __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[v][j], fb[v][i], acc2[v % NACC][i][j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int off = (((2 * s + h) ^ key) << 4) + l32 * 128;
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc2[s % NACC][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                  *reinterpret_cast<const f16x8*>(sa + (wn * (BN / 2) + 32 * j) * 128 + off),
                  *reinterpret_cast<const f16x8*>(sb + (wm * (BM / 2) + 32 * i) * 128 + off), acc2[s % NACC][i][j], 0,
                  0, 0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[0][i][j] = acc2[0][i][j];
        if constexpr (NACC == 2) acc[0][i][j] += acc2[1][i][j];
      }
  }
  if (kg != 0) return true;

  if constexpr (Q8) {
    // ---- int8 epilogue (conv_i8's): lane owns channels nb + 32j + 8q + 4h + {0..3} of pixel pbm + 32i + l32
    const QRec* Q = a.q;
    const float* post = reinterpret_cast<const float*>(smem + NSTAGE * SB + 16 + 256);
    const int mode = Q->mode;
    const i8* res = static_cast<const i8*>(a.res);
    const int zpad = Q->z_in - 128;  // the byte the quantized conv reads in a padding tap (the DMA read 0)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = tm * BM + wm * (BM / 2) + 32 * i + l32;
      if (m >= a.M) continue;
      const int b = ym_div(m, a.fd_hw), rem = m - b * (a.Ho * a.Wo);
      const int oy = ym_div(rem, a.fd_w), ox = rem - oy * a.Wo;
      const size_t obase = (size_t)(b * a.d_P + a.d_pixoff + oy * a.d_W + ox) * a.d_ctot + a.d_coff;
      const size_t rbase = res ? (size_t)(b * a.r_P + oy * a.Wo + ox) * a.r_ctot + a.r_coff : 0;
      unsigned outside = 0;  // 3x3 taps of this pixel's window outside the image
      if (a.k == 3) {
        const int iy0 = oy * a.s - 1, ix0 = ox * a.s - 1;
#pragma unroll
        for (int t = 0; t < 9; ++t)
          outside |= ((unsigned)(iy0 + t / 3) >= (unsigned)a.Hin || (unsigned)(ix0 + t % 3) >= (unsigned)a.Win) ? (1u << t)
                                                                                                              : 0u;
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = tn * BN + wn * (BN / 2) + 32 * j + 8 * q + 4 * h;
          if (n >= a.N) continue;
          i32x4 bi = *reinterpret_cast<const i32x4*>(a.biasi + n);
          if (outside) {
            for (int t = 0; t < 9; ++t)
              if ((outside >> t) & 1u) bi += zpad * *reinterpret_cast<const i32x4*>(a.wtap + t * a.N + n);
          }
          const f32x4 sa = *reinterpret_cast<const f32x4*>(a.sasw + n);
          const f32x4 bf = *reinterpret_cast<const f32x4*>(a.bias + n);
          const int r4 = res ? *reinterpret_cast<const int*>(res + rbase + n) : 0;
          int ov[4];
          float fv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int qc = Q8S::code(acc[0][i][j][4 * q + e], bi[e], sa[e], bf[e], Q);
            if (mode == 1) {
              ov[e] = Q8S::raw_byte(qc);
              continue;
            }
            float v = post[qc];
            if (res) v = __fadd_rn(v, Q8S::dec(r4 >> (8 * e), Q->z_r, Q->s_r));
            fv[e] = v;
            ov[e] = Q8S::store(v, Q);
          }
          if (mode == 2) *reinterpret_cast<f32x4*>(static_cast<float*>(a.dst) + obase + n) = f32x4{fv[0], fv[1], fv[2], fv[3]};
          else *reinterpret_cast<int*>(static_cast<i8*>(a.dst) + obase + n) = pack4(ov);
        }
    }
    return true;
  } else {
  // ---- epilogue: lane owns channels nb + 32j + 8q + 4h + {0..3} of pixel pbm + 32i + l32
  OutT* dst = static_cast<OutT*>(a.dst);
  // x3 pair-layout outputs: lanes l and l ^ 32 (h = 0 / 1: channels +0..3 / +4..7 of one chunk of one pixel) write
  // the chunk as one 32-byte run (ym_p2_store4_pair) where the slice, the channel count and the pixel-shuffle
  // sub-pixel width keep every chunk whole (uniform)
  constexpr bool PAIRST = X3 && std::is_same<OutT, P2>::value;
  const bool pairst = PAIRST && (a.pst & 1) && ((NOUT | a.d_coff | a.d_ctot) & 7) == 0 && (!a.shuffle || (a.npr & 7) == 0);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if (ep_m[i] >= a.M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = tn * BN + wn * (BN / 2) + 32 * j + 8 * q + 4 * h;
        if constexpr (PAIRST) {
          if (pairst) {  // both lanes of a pair take this branch together (same pixel, n < N alike)
            const bool okn = n < NOUT;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x = ym_x3_pre(acc[0][i][j][4 * q + e], FUSE ? a.wsc2 : a.wsc, bias4[j][q][e]);
              v[e] = ((FUSE ? a.act2 : a.act) ? ym_silu_x3(x) : x) + (float)res4[i][j][q][e];
            }
            size_t o = ep_obase[i] + n;
            if (a.shuffle) {
              const int sub = n / a.npr;
              const int ch = n - sub * a.npr;
              o = ep_obase[i] + (size_t)((sub >> 1) * a.d_W + (sub & 1)) * a.d_ctot + ch;
            }
            if constexpr (SC1OUT)
              ym_p2_store4_pair<32, true>(dst + (okn ? o : 0), v, h, okn, a.pst & 16, a.dst);
            else
              ym_p2_store4_pair<32>(dst + (okn ? o : 0), v, h, okn, a.pst & 16);
            continue;
          }
        }
        if (n >= NOUT) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = X3 ? ym_x3_pre(acc[0][i][j][4 * q + e], FUSE ? a.wsc2 : a.wsc, bias4[j][q][e])
                             : acc[0][i][j][4 * q + e] + bias4[j][q][e];
          v[e] = ((FUSE ? a.act2 : a.act) ? (X3 ? ym_silu_x3(x) : ym_silu_fast(x)) : x) + (float)res4[i][j][q][e];
        }
        if constexpr (SC1OUT) {  // (the chain kernel takes no pixel-shuffle ops)
          static_assert(std::is_same<OutT, P2>::value, "write-through epilogue: pair-layout outputs");
          ym_p2_store4<true>(dst + ep_obase[i] + n, v);
        } else if (a.shuffle) {
          const int sub = n / a.npr;
          const int ch = n - sub * a.npr;
          Store4<OutT>::st(dst + ep_obase[i] + (size_t)((sub >> 1) * a.d_W + (sub & 1)) * a.d_ctot + ch, v);
        } else {
          Store4<OutT>::st(dst + ep_obase[i] + n, v);
        }
      }
  }
  YM_STAMP(3);
  return true;
  }
}

template <typename OutT, int BM, int BN, int KIND, int SPLIT, int KG, int NSTAGE, int SUB, bool X3 = false,
          bool FUSE = false, bool Q8 = false>
__global__ __launch_bounds__(256 * KG) void conv_dma(const ConvArgs a) {
  constexpr int KS2 = FUSE ? (X3 ? 2 : 1) * BN / 64 : 0;
  typedef DmaSmem<NSTAGE, SUB * (BM + BN) * 128, BN, KS2, Q8> SM;
  __shared__ __attribute__((aligned(16))) char smem[SM::ring];
  __shared__ __attribute__((aligned(16))) char w2s[SM::w2];
#ifndef YM_NO_WARM
  ym_warm_kernargs<sizeof(ConvArgs)>();
#endif
  conv_dma_body<OutT, BM, BN, KIND, SPLIT, KG, NSTAGE, SUB, X3, FUSE, false, Q8>(a, blockIdx.x, smem, w2s);
}

struct DmaCfg {
  int bm, bn, split, kg, ns, sub;
};
// (ids 17 + i in the conv config space of csrc/ym_conv.hip; the configurations no tuned table chose or came within 3 %
// of were dropped in round 2).  (bm, bn, split, kg, ns, sub): tile, in-launch K split, wave groups, ring depth, K
// sub-stages per stage.  The double-buffered (ns 2) 4-wave configs fit two or three workgroups per CU, whose
// barrier-separated phases (DMA issue, LDS fragment reads, MFMAs) then overlap across workgroups: yolo11s B=8
// model.3 34.5 -> 28.5 us, model.16.cv1 21.1 -> 18.4, model.23.cv2.0.0 19.0 -> 17.1
#define YM_DMA_CFGS(X) \
  X(0, 64, 64, 1, 1, 4, 1) X(1, 64, 64, 8, 1, 4, 1) X(2, 128, 128, 1, 1, 4, 1) X(3, 64, 64, 1, 2, 4, 1)        \
  X(4, 64, 64, 4, 2, 4, 1) X(5, 128, 64, 1, 2, 4, 1) X(6, 64, 128, 1, 2, 4, 1) X(7, 64, 64, 1, 2, 4, 2)        \
  X(8, 64, 64, 2, 2, 4, 2) X(9, 64, 128, 1, 2, 3, 2) X(10, 64, 64, 1, 2, 3, 2) X(11, 64, 64, 1, 2, 3, 3)       \
  X(12, 64, 64, 1, 2, 2, 4) X(13, 64, 64, 2, 2, 3, 3) X(14, 64, 128, 1, 2, 2, 3) X(15, 128, 128, 1, 2, 2, 2)   \
  X(16, 128, 64, 1, 2, 2, 3) X(17, 128, 128, 1, 1, 2, 1) X(18, 128, 64, 1, 1, 2, 1) X(19, 64, 128, 1, 1, 2, 1) \
  X(20, 128, 128, 1, 1, 2, 2) X(21, 64, 64, 1, 1, 2, 2) X(22, 256, 64, 1, 1, 2, 1) X(23, 128, 128, 2, 1, 2, 1) \
  X(24, 64, 64, 1, 1, 2, 1) X(25, 128, 64, 1, 1, 3, 1) X(26, 64, 64, 1, 2, 2, 2) X(27, 64, 64, 2, 1, 2, 1)     \
  X(28, 64, 128, 2, 1, 2, 1) X(29, 128, 64, 2, 1, 2, 1)
constexpr DmaCfg kDma[] = {
#define YM_X(id, bm, bn, sp, kg, ns, sub) {bm, bn, sp, kg, ns, sub},
    YM_DMA_CFGS(YM_X)
#undef YM_X
};
constexpr int kNumDma = sizeof(kDma) / sizeof(kDma[0]);

template <typename OutT, int BM, int BN, int SPLIT, int KG, int NS, int SUB, bool X3 = false, bool Q8 = false>
hipError_t launch_dma(ConvArgs a, int kind, hipStream_t st) {
  if (X3 && (4 / KG) % 2) return hipErrorInvalidValue;
  const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
  a.tiles_n = (a.N + BN - 1) / BN;
  a.fd_tn = ym_fdiv(a.tiles_n);
  a.fd_cin8 = ym_fdiv(a.Cin8 > 0 ? a.Cin8 : 1);
  a.tm_per_xcd = tiles_m8 / 8;
  if (SPLIT > 1) {
    const long tiles = (long)tiles_m8 * a.tiles_n;
    if (tiles > a.cnt_cap || tiles * SPLIT * BM * BN * 4 > a.slab_cap) return hipErrorInvalidValue;
    if (a.Kpad / DK < SPLIT) return hipErrorInvalidValue;
  }
  if (SUB > 1 && (a.Kpad / DK) % (SPLIT * SUB)) return hipErrorInvalidValue;  // whole stages in every split
  const dim3 grid(tiles_m8 * a.tiles_n * SPLIT), block(256 * KG);
  if (kind == 1) {
    hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 1, SPLIT, KG, NS, SUB, X3, false, Q8>), grid, block, 0, st, a);
  } else if constexpr (!std::is_same<OutT, float>::value) {  // fp32 outputs: only the Detect head's 1x1 convs
    if (kind == 4)
      hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 4, SPLIT, KG, NS, SUB, X3, false, Q8>), grid, block, 0, st, a);
    else
      hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 3, SPLIT, KG, NS, SUB, X3, false, Q8>), grid, block, 0, st, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// x3-only configurations (op cfg ids appended after the whole f16 catalogue, so the f16 tables keep their ids): the
// pair layout doubles a conv's storage K, and with it the chain of K stages of the latency-bound 20² / 40² layers —
// split K 3-8 ways over workgroups with 128-192-deep stages to shorten it.  (Round 5 tried the same splits on 128-wide
// tiles, whose waves own 64 x 64 blocks and so read each LDS fragment for 2 MFMAs instead of 1: slower on every 20² /
// 40² op, e.g. 16.3 vs 12.3 us for a 20² 3x3 128 -> 128 — fewer workgroups and one wave per SIMD;
// profiles/r05l_x3_wide_tiles.txt.)
#define YM_DMA_X3_CFGS(X)                                                                                      \
  X(0, 64, 64, 4, 2, 2, 3) X(1, 64, 64, 4, 2, 2, 2) X(2, 64, 64, 3, 2, 2, 2) X(3, 64, 64, 6, 2, 2, 2)          \
  X(4, 64, 64, 8, 2, 2, 2) X(5, 64, 64, 4, 1, 2, 2) X(6, 64, 128, 4, 2, 2, 2) X(7, 64, 64, 2, 2, 2, 4)         \
  X(8, 64, 64, 4, 2, 3, 2)
constexpr int kNumDmaX3 = 9;

template <typename OutT>
hipError_t dispatch_x3only(const ConvArgs& a, int kind, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, bm, bn, sp, kg, ns, sub) \
  case id: return launch_dma<OutT, bm, bn, sp, kg, ns, sub, true>(a, kind, st);
    YM_DMA_X3_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

template <typename OutT, bool X3 = false>
hipError_t dispatch(const ConvArgs& a, int kind, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, bm, bn, sp, kg, ns, sub) \
  case id: return launch_dma<OutT, bm, bn, sp, kg, ns, sub, X3>(a, kind, st);
    YM_DMA_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

// Fused conv -> 1x1 pairs (FUSE, x3): the DMA configurations (ids as in YM_DMA_CFGS) instantiated with the second GEMM
// — whole-K tiles (no split) of BN 64 / 128 holding the first conv's N: s model.1+cv1 (3x3 s2 32 -> 64, 1x1 64 -> 64),
// model.3+cv1 (3x3 s2 64 -> 128, 1x1 128 -> 128), the Detect cv2.l.1 -> cv2.l.2 chains (3x3 64 -> 64, 1x1 64 -> 64 fp32
// rows), s-seg cv4.l.1 -> cv4.l.2
// (the 144-KB rings of ids 11 / 16 leave no room for W2)
#define YM_DMA_FUSE_CFGS(X) \
  X(7, 64, 64, 1, 2, 4, 2) X(18, 128, 64, 1, 1, 2, 1) X(21, 64, 64, 1, 1, 2, 2) X(24, 64, 64, 1, 1, 2, 1) \
  X(26, 64, 64, 1, 2, 2, 2) X(17, 128, 128, 1, 1, 2, 1) X(19, 64, 128, 1, 1, 2, 1) X(3, 64, 64, 1, 2, 4, 1)     \
  X(5, 128, 64, 1, 2, 4, 1) X(25, 128, 64, 1, 1, 3, 1)

template <typename OutT, int BM, int BN, int KG, int NS, int SUB>
hipError_t launch_fuse(ConvArgs a, int kind, hipStream_t st) {
  if ((4 / KG) % 2) return hipErrorInvalidValue;
  if (a.N > BN || a.N2 > BN) return hipErrorInvalidValue;
  if (SUB > 1 && (a.Kpad / DK) % SUB) return hipErrorInvalidValue;  // whole stages
  const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
  a.tiles_n = 1;
  a.fd_tn = ym_fdiv(1);
  a.fd_cin8 = ym_fdiv(a.Cin8 > 0 ? a.Cin8 : 1);
  a.tm_per_xcd = tiles_m8 / 8;
  const dim3 grid(tiles_m8), block(256 * KG);
  if (kind == 4)
    hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 4, 1, KG, NS, SUB, true, true>), grid, block, 0, st, a);
  else if (kind == 3)
    hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 3, 1, KG, NS, SUB, true, true>), grid, block, 0, st, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <typename OutT>
hipError_t dispatch_fuse(const ConvArgs& a, int kind, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, bm, bn, sp, kg, ns, sub) \
  case id: return launch_fuse<OutT, bm, bn, kg, ns, sub>(a, kind, st);
    YM_DMA_FUSE_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------------------------
// Persistent chain of two dependent x3 convs in ONE launch (verdict r5 item 1: the 20² dependent chain, built and
// measured instead of priced).  Workgroup w runs work item w of op 0 (the conv_dma_body tile map,
// split-K included), publishes it, then runs item w of op 1, whose pixel tile first waits for the op-0 pixel tiles
// its 3x3 window reads (per-tile ready counters, no grid barrier).  Hand-off (cdna_hip_programming.md §6 Guideline
// 16): op 0's epilogue stores write through (sc1) → every storing wave's vmcnt(0) → workgroup barrier → one lane's
// agent-scope counter add; the consumer's one lane polls the counters relaxed (sc1 loads + s_sleep, bounded: a give-up
// sets `tmo`), then one agent-scope acquire (L1 invalidate) → vmcnt(0) → workgroup barrier → the ring's LDS-DMA loads.
// The grid is at most one workgroup per CU (the 147 KB rings of these configurations admit one), so every workgroup
// is resident once earlier kernels drain; only one chain kernel runs at a time (the runtime places chains on the main
// stream only).  The last workgroup to finish zeroes the counters for the next launch.
struct ChainArgs {
  ConvArgs op[2];
  int* ready;        // per op-0 pixel tile: (tn) tiles stored; zero at launch
  int* done;         // workgroups finished
  int* tmo;          // 1 when a wait gave up
  int halo;          // op-0 output pixels an op-1 tile reads beyond its own range (Wo + 1 for a 3x3, 0 for a 1x1)
  int tiles_m0;      // real op-0 pixel tiles
  int ready_target;  // op 0's N tiles
  int items0, items1;
};

template <int SPLIT>
__device__ __forceinline__ int chain_tm(const ConvArgs& a, int bid) {  // conv_dma_body's pixel tile of item bid
  const int rest = (bid >> 3) / SPLIT;
  return (bid & 7) * a.tm_per_xcd + ym_div(rest, a.fd_tn);
}

template <int BM, int BN, int KA, int KB, int SPLIT, int KG, int NS, int SUB>
__global__ __launch_bounds__(256 * KG) void conv_dma_chain(const ChainArgs c) {
  typedef DmaSmem<NS, SUB * (BM + BN) * 128, BN, 0> SM;
  __shared__ __attribute__((aligned(16))) char smem[SM::ring];
  __shared__ __attribute__((aligned(16))) char w2s[SM::w2];
#ifndef YM_NO_WARM
  ym_warm_kernargs<sizeof(ChainArgs)>();
#endif
  const int G = gridDim.x, tid = threadIdx.x;
  for (int it = blockIdx.x; it < c.items0; it += G) {
    const bool fin = conv_dma_body<P2, BM, BN, KA, SPLIT, KG, NS, SUB, true, false, true>(c.op[0], it, smem, w2s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
    __syncthreads();
    if (tid == 0 && fin)
      __hip_atomic_fetch_add(c.ready + chain_tm<SPLIT>(c.op[0], it), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int it = blockIdx.x; it < c.items1; it += G) {
    const ConvArgs& b = c.op[1];
    const int tm = chain_tm<SPLIT>(b, it);
    if (tm * BM < b.M) {
      if (tid == 0) {
        const int lo = tm * BM - c.halo <= 0 ? 0 : (tm * BM - c.halo) / BM;
        const int hi = min(c.tiles_m0 - 1, (tm * BM + BM - 1 + c.halo) / BM);
        bool gave_up = __hip_atomic_load(c.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        for (int t = lo; t <= hi && !gave_up; ++t) {
          unsigned spins = 0;
          while (__hip_atomic_load(c.ready + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < c.ready_target) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 20)) {  // bounded: a missing producer ends the launch (with wrong tiles), never hangs
              __hip_atomic_store(c.tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              gave_up = true;
              break;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // ONE L1 invalidate after the match
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
    conv_dma_body<P2, BM, BN, KB, SPLIT, KG, NS, SUB, true, false, false>(b, it, smem, w2s);
  }
  __syncthreads();
  if (tid == 0) {  // the last workgroup: every wait of this launch is over, zero the counters for the next one
    const int d = __hip_atomic_fetch_add(c.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == G - 1) {
      for (int t = 0; t < c.tiles_m0; ++t) __hip_atomic_store(c.ready + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// kind of one chain op: 1 (1x1, one source), 4 (3x3, Cin % 64 == 0 in storage chunks), 3 (other 3x3); -1: none
inline int chain_kind(const ConvArgs& a) {
  if (a.src1 || a.up0 || a.w2 || a.dw_w || a.shuffle || a.nchw || !a.src0) return -1;
  if (a.k == 1 && a.s == 1) return 1;
  if (a.k == 3) return a.Cin8 % 8 == 0 ? 4 : 3;
  return -1;
}

template <int BM, int BN, int SPLIT, int KG, int NS, int SUB>
hipError_t launch_chain(ConvArgs a0, ConvArgs a1, int* ctl, int cap, hipStream_t st) {
  if ((4 / KG) % 2) return hipErrorInvalidValue;
  ConvArgs* ops[2] = {&a0, &a1};
  int items[2];
  for (int i = 0; i < 2; ++i) {
    ConvArgs& a = *ops[i];
    const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
    a.tiles_n = (a.N + BN - 1) / BN;
    a.fd_tn = ym_fdiv(a.tiles_n);
    a.fd_cin8 = ym_fdiv(a.Cin8 > 0 ? a.Cin8 : 1);
    a.tm_per_xcd = tiles_m8 / 8;
    if (SPLIT > 1) {
      const long tiles = (long)tiles_m8 * a.tiles_n;
      if (tiles > a.cnt_cap || tiles * SPLIT * BM * BN * 4 > a.slab_cap || a.Kpad / DK < SPLIT) return hipErrorInvalidValue;
    }
    if (SUB > 1 && (a.Kpad / DK) % (SPLIT * SUB)) return hipErrorInvalidValue;
    items[i] = tiles_m8 * a.tiles_n * SPLIT;
  }
  const int ka = chain_kind(a0), kb = chain_kind(a1);
  if (ka != 4 || kb != 4) return hipErrorInvalidValue;  // (the prototype: 3x3 -> 3x3)
  if (a1.src0 != a0.dst || a1.s0_coff != a0.d_coff || a1.s0_ctot != a0.d_ctot || a0.M != a1.M || a1.s != 1 ||
      a0.N != a1.Cin8 * 8 / 2)
    return hipErrorInvalidValue;
  const int G = items[0] > items[1] ? items[0] : items[1];
  const int tiles_m0 = (a0.M + BM - 1) / BM;
  if (G > 256 || tiles_m0 + 2 > cap) return hipErrorInvalidValue;  // one workgroup per CU, all resident
  ChainArgs c{};
  c.op[0] = a0;
  c.op[1] = a1;
  c.ready = ctl;
  c.done = ctl + cap - 2;
  c.tmo = ctl + cap - 1;
  c.halo = a1.k == 3 ? a1.Wo + 1 : 0;
  c.tiles_m0 = tiles_m0;
  c.ready_target = a0.tiles_n;
  c.items0 = items[0];
  c.items1 = items[1];
  hipLaunchKernelGGL((conv_dma_chain<BM, BN, 4, 4, SPLIT, KG, NS, SUB>), dim3(G), dim3(256 * KG), 0, st, c);
  return hipGetLastError();
}

hipError_t dispatch_i8(const ConvArgs& a, int kind, int i, hipStream_t st) {
  switch (i) {
#define YM_X(id, bm, bn, sp, kg, ns, sub) \
  case id: return launch_dma<i8, bm, bn, sp, kg, ns, sub, false, true>(a, kind, st);
    YM_DMA_CFGS(YM_X)
#undef YM_X
  }
  return hipErrorInvalidValue;
}

}  // namespace

// The int8 PTQ plan on LDS-DMA configuration i (ids as in YM_DMA_CFGS): the int8 tensors and weight rows are described
// to the kernel as fp16 tensors of half the channels (ctot, coff, Kpad, element counts halved; Cin8 already counts
// 16-channel chunks), the epilogue keeps int8 units (d_*, r_*).  1x1 stride-1 single-source and 3x3 convs, whole
// 128-byte K stages (Kpad % 128 == 0); fp8 plans stay on conv_i8 (their fp8 MFMA chain is restated per kernel).
hipError_t ym_launch_conv_dma_i8(const ConvArgs& a0, int i, hipStream_t st) {
  if (i < 0 || i >= kNumDma || !a0.q || !a0.sasw || !a0.biasi || a0.nchw || a0.src1 || a0.up0 || a0.shuffle || a0.w2 ||
      a0.dw_w || !a0.src0)
    return hipErrorInvalidValue;
  int kind;
  if (a0.k == 1 && a0.s == 1) kind = 1;
  else if (a0.k == 3 && a0.wtap) kind = a0.Cin8 % 8 == 0 ? 4 : 3;
  else return hipErrorInvalidValue;
  if (a0.Kpad % 128 || (a0.s0_ctot | a0.s0_coff) & 15 || (a0.N & 3) || (a0.d_ctot & 3) || (a0.d_coff & 3))
    return hipErrorInvalidValue;
  ConvArgs a = a0;
  a.s0_ctot /= 2;
  a.s0_coff /= 2;
  a.Kpad /= 2;
  a.s0_elems /= 2;
  const long lim = 0x7FFFFFF0L / 2;  // fp16 elements
  if ((long)a.N * a.Kpad > lim || a.s0_elems > lim) return hipErrorInvalidValue;
  return dispatch_i8(a, kind, i, st);
}

// Two dependent x3 convs (op 1 reads op 0's output) as one persistent launch on LDS-DMA configuration i (ids as in
// YM_DMA_CFGS; instantiated: 8, 13, 26).  ctl: `cap` zeroed ints (ready counters, done, give-up word), left zeroed.
hipError_t ym_launch_conv_dma_chain(const ConvArgs& a0, const ConvArgs& a1, int i, int* ctl, int cap, hipStream_t st) {
  if (!a0.x3 || !a1.x3 || a0.Kpad % DK || a1.Kpad % DK) return hipErrorInvalidValue;
  if ((a0.N & 7) || (a1.N & 7) || (a0.d_ctot & 7) || (a0.d_coff & 7) || (a1.d_ctot & 3) || (a1.d_coff & 3))
    return hipErrorInvalidValue;
  const long lim = 0x7FFFFFF0L / 2;
  if ((long)a0.N * a0.Kpad > lim || (long)a1.N * a1.Kpad > lim || a0.s0_elems > lim || a1.s0_elems > lim)
    return hipErrorInvalidValue;
  switch (i) {
    case 8: return launch_chain<64, 64, 2, 2, 4, 2>(a0, a1, ctl, cap, st);
    case 13: return launch_chain<64, 64, 2, 2, 3, 3>(a0, a1, ctl, cap, st);
    case 26: return launch_chain<64, 64, 1, 2, 2, 2>(a0, a1, ctl, cap, st);
  }
  return hipErrorInvalidValue;
}

// A fused conv -> 1x1 pair (ConvArgs::w2, k2 == 1) on the LDS-DMA kernel with the second GEMM in its epilogue (x3
// plans; i: a DMA configuration id, only YM_DMA_FUSE_CFGS are instantiated)
hipError_t ym_launch_conv_dma_fuse(int out_f32, const ConvArgs& a, int i, hipStream_t st) {
  if (!a.x3 || !a.w2 || a.k2 != 1 || a.k != 3 || a.res || a.shuffle || a.src1 || a.up0 || !a.src0 || a.nchw)
    return hipErrorInvalidValue;
  if (a.Kpad % DK || (a.N & 7) || (a.N2 & 7) || a.Kpad2 < 2 * a.N || (a.d_ctot & 3) || (a.d_coff & 3))
    return hipErrorInvalidValue;
  const long lim = 0x7FFFFFF0L / 2;  // elements
  if ((long)a.N * a.Kpad > lim || a.s0_elems > lim) return hipErrorInvalidValue;
  const int kind = a.Cin8 % 8 == 0 ? 4 : 3;
  return out_f32 ? dispatch_fuse<float>(a, kind, i, st) : dispatch_fuse<P2>(a, kind, i, st);
}

int ym_conv_dma_num_cfgs() { return kNumDma; }
int ym_conv_dma_x3_num_cfgs() { return kNumDmaX3; }

// Host-side applicability: f16 plans, 1x1 stride-1 or 3x3 convs, byte offsets < 2^31 for every operand, and a
// 64-aligned concat split (a stage never straddles the two sources).  i >= kNumDma: the x3-only configurations.
hipError_t ym_launch_conv_dma(int out_f32, const ConvArgs& a, int i, hipStream_t st) {
  if (i < 0 || i >= kNumDma + (a.x3 ? kNumDmaX3 : 0)) return hipErrorInvalidValue;
  int kind;
  if (a.k == 1 && a.s == 1) kind = 1;
  else if (a.k == 3) kind = a.Cin8 % 8 == 0 ? 4 : 3;
  else return hipErrorInvalidValue;
  if (a.Kpad % DK || !a.src0 || a.nchw) return hipErrorInvalidValue;
  if (kind == 1 && a.src1 && (a.x3 ? 2 : 1) * a.C0 % DK) return hipErrorInvalidValue;
  const long lim = 0x7FFFFFF0L / 2;  // elements
  if ((long)a.N * a.Kpad > lim || a.s0_elems > lim || a.s1_elems > lim) return hipErrorInvalidValue;
  if ((a.N & 3) || (a.d_ctot & 3) || (a.d_coff & 3)) return hipErrorInvalidValue;
  if (a.x3 && i >= kNumDma)
    return out_f32 ? dispatch_x3only<float>(a, kind, i - kNumDma, st) : dispatch_x3only<P2>(a, kind, i - kNumDma, st);
  if (a.x3) return out_f32 ? dispatch<float, true>(a, kind, i, st) : dispatch<P2, true>(a, kind, i, st);
  return out_f32 ? dispatch<float>(a, kind, i, st) : dispatch<f16>(a, kind, i, st);
}
