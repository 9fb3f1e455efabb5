// LDS-DMA implicit-GEMM convolution for gfx950 with in-launch split-K — the fp16 conv hot path, second generation.
//
// Same GEMM as csrc/ym_conv.hip (D[n][m] = Σ_k W[n][k]·X[k][m], n = output channel on the MFMA rows, m = output pixel on
// the columns, k = (ky, kx, c) so an 8-element K chunk is 8 channels of one input pixel), built for the two regimes
// that cost the first-generation kernels most on YOLO11 shapes:
//  * operands stream global → LDS with `buffer_load_dwordx4 … lds` (LDS-DMA: no VGPR staging, no ds_write pass)
//    into a 3-deep ring of 64-deep K stages, one raw barrier per stage and a counted `s_waitcnt vmcnt`, so two
//    stages of loads are always in flight behind the MFMAs.  The implicit-im2col gather is per lane (each lane
//    computes its own pixel/tap byte offset); 3x3 zero padding, K tails and M/N tails are out-of-range buffer offsets,
//    which the DMA turns into zeros in LDS — no branches in the load path;
//  * LDS image: row = one pixel (or one weight row) × 64 K = 128 B; chunk c of row r sits at slot c ^ ((r >> 1) & 7),
//    which makes the 16-lane groups of every ds_read_b128 fragment read hit 16 distinct 16-byte bank groups;
//    the swizzle is applied on the SOURCE side (the DMA destination is lane-linear);
//  * small-M deep layers (20x20 / 40x40 maps: a few hundred pixels per image, K up to 4608) are bound by the serial
//    chain of K stages, not by MFMA or HBM: SPLIT workgroups share one output tile, each takes a contiguous K range,
//    writes its fp32 partial tile (a "slab"), and the last to arrive at the tile's counter (agent-scope release /
//    acquire, cdna_hip_programming.md §5 "In-launch split-K reduction") sums the slabs and runs the epilogue.
// Epilogue as in ym_conv.hip: + folded-BN bias, SiLU, + residual, channel-slice store (zero-copy concat), fp32
// anchor-major Detect rows, 2x2 pixel shuffle (Proto ConvTranspose2d).
#include "ym_common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;

namespace {

constexpr int DK = 64;                    // K per stage
constexpr int NSTAGE = 3;                 // LDS ring depth
constexpr unsigned OOB = 0x80000000u;     // byte offset past num_records: the DMA deposits zeros

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
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

// 256 threads = 2x2 waves; a wave owns (BM/2) pixels x (BN/2) channels = TM x TN blocks of 32x32.
template <typename OutT, int BM, int BN, int KIND, int SPLIT>
__global__ __launch_bounds__(256) void conv_dma(const ConvArgs a) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int GB = BM / 32, GA = BN / 32;  // DMA wave-instructions per stage per wave (8 rows of 128 B each)
  constexpr int NL = GA + GB;
  constexpr int SB = (BM + BN) * 128;        // bytes per stage
  constexpr int NREG = TM * TN * 16;
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * SB + 16];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid & 1, wn = wid >> 1;
  const int l32 = lane & 31, h = lane >> 5;
  // tile map: every N tile and every K split of pixel tile tm share bid % 8 = one XCD (its L2 holds the pixels and
  // the split's slabs); padding workgroups (tm beyond M) exit before touching a counter
  const int bid = blockIdx.x;
  int rest = bid >> 3;
  const int sp = rest % SPLIT;
  rest /= SPLIT;
  const int tn = rest % a.tiles_n;
  const int tm = (rest / a.tiles_n) * 8 + (bid & 7);
  if (tm * BM >= a.M) return;
  const int HWo = a.Ho * a.Wo;

  // ---- DMA lanes: instruction-row rr = lane >> 3, LDS slot lane & 7, so this lane fetches chunk c of its row with
  // c = slot ^ ((row >> 1) & 7); rows of wave wid's groups are (wid + 4 gi) * 8 + rr, hence (row >> 1) & 7 =
  // ((wid & 1) << 2) | (rr >> 1) for every group of this wave: one chunk index per lane.
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
#pragma unroll
  for (int gi = 0; gi < GB; ++gi) {
    const int m = tm * BM + (wid + 4 * gi) * 8 + rr;
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    const int b = mm / HWo, rem = mm - (mm / HWo) * HWo;
    const int oy = rem / a.Wo, ox = rem - (rem / a.Wo) * a.Wo;
    if constexpr (KIND == 1) {
      const int sy = a.up0 ? (oy >> 1) : oy, sx = a.up0 ? (ox >> 1) : ox;
      pbase0[gi] = ok ? (b * a.s0_P + sy * a.s0_W + sx) * a.s0_ctot + a.s0_coff : -1;
      // (row bases stay >= 0 for valid rows: -1 marks an M-tail row, so the -C0 of the second source's channel
      // index is applied per stage, not folded in here)
      pbase1[gi] = ok && a.src1 ? (b * a.s1_P + oy * a.Win + ox) * a.s1_ctot + a.s1_coff : -1;
      piy[gi] = pix[gi] = 0;
    } else {
      pbase0[gi] = ok ? b * a.s0_P : -1;  // image pixel base
      pbase1[gi] = 0;
      piy[gi] = oy * a.s - 1;
      pix[gi] = ox * a.s - 1;
    }
  }
  int wbase[GA];
#pragma unroll
  for (int gi = 0; gi < GA; ++gi) {
    const int n = tn * BN + (wid + 4 * gi) * 8 + rr;
    wbase[gi] = n < a.N ? n * a.Kpad + c * 8 : -1;
  }

  const int nst = a.Kpad / DK;
  const int k_lo = (nst * sp) / SPLIT, k_hi = (nst * (sp + 1)) / SPLIT;
  const int nk = k_hi - k_lo;
  // KIND 3: tap / channel block of this lane's chunk at stage k_lo (chunk index k*8 + c)
  int tap = 0, cb = 0;
  if constexpr (KIND == 3) {
    const int idx = k_lo * 8 + c;
    tap = idx / a.Cin8;
    cb = idx - tap * a.Cin8;
  }
  int kcur = k_lo;  // stage whose loads are issued next

  auto issue = [&](int slot) {
    char* sbase = smem + slot * SB;
    const int chunk = kcur * 8 + c;
    // B: pixels
    if constexpr (KIND == 1) {
      const bool second = a.src1 && kcur * DK >= a.C0;  // wave-uniform (C0 % 64 == 0 when src1 is used)
#pragma unroll
      for (int gi = 0; gi < GB; ++gi) {
        const int pb = second ? pbase1[gi] : pbase0[gi];
        const unsigned off = pb >= 0 ? (unsigned)(pb + chunk * 8 - (second ? a.C0 : 0)) * 2u : OOB;
        dma16(second ? rs1 : rs0, sbase + (wid + 4 * gi) * 1024, off);
      }
    } else {
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
      for (int gi = 0; gi < GB; ++gi) {
        const int iy = piy[gi] + ky, ix = pix[gi] + kx;
        const bool ok = pbase0[gi] >= 0 && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        const unsigned off =
            ok ? (unsigned)((pbase0[gi] + iy * a.Win + ix) * a.s0_ctot + a.s0_coff + cb * 8) * 2u : OOB;
        dma16(rs0, sbase + (wid + 4 * gi) * 1024, off);
      }
      cb += 8;
      while (cb >= a.Cin8) { cb -= a.Cin8; ++tap; }
    }
    // A: weights
#pragma unroll
    for (int gi = 0; gi < GA; ++gi) {
      const unsigned off = wbase[gi] >= 0 ? (unsigned)(wbase[gi] + kcur * DK) * 2u : OOB;
      dma16(rw, sbase + BM * 128 + (wid + 4 * gi) * 1024, off);
    }
    ++kcur;
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int key = (l32 >> 1) & 7;
  auto compute = [&](int slot) {
    const char* sb = smem + slot * SB;
    const char* sa = sb + BM * 128;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int off = ((((2 * s + h) ^ key)) << 4) + l32 * 128;
      f16x8 fb[TM], fa[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fb[i] = *reinterpret_cast<const f16x8*>(sb + (wm * (BM / 2) + 32 * i) * 128 + off);
#pragma unroll
      for (int j = 0; j < TN; ++j) fa[j] = *reinterpret_cast<const f16x8*>(sa + (wn * (BN / 2) + 32 * j) * 128 + off);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[j], fb[i], acc[i][j], 0, 0, 0);
    }
  };

  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int it = 0; it < nk; ++it) {
    if (it + 1 < nk) wait_vm<NL>(); else wait_vm<0>();
    raw_barrier();  // stage it is in LDS for every wave; every wave is done reading stage it-1's slot
    if (it + 2 < nk) issue((it + 2) % NSTAGE);
    compute(it % NSTAGE);
  }

  // ---- split-K: publish the partial tile, the last arriver reduces
  if constexpr (SPLIT > 1) {
    const int tile = tm * a.tiles_n + tn;
    float* slab = a.slab + (size_t)(tile * SPLIT + sp) * (256 * NREG);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int qq = (i * TN + j) * 4 + q;
          *reinterpret_cast<f32x4*>(slab + ((size_t)qq * 256 + tid) * 4) =
              f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem + NSTAGE * SB);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == SPLIT - 1;
      if (last) {
        __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // sum every slab (this workgroup's own included) in split order, so the result does not depend on which split
    // arrived last: bitwise-reproducible launches
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll 1
    for (int s2 = 0; s2 < SPLIT; ++s2) {
      const float* o = a.slab + (size_t)(tile * SPLIT + s2) * (256 * NREG);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int qq = (i * TN + j) * 4 + q;
            const f32x4 v = *reinterpret_cast<const f32x4*>(o + ((size_t)qq * 256 + tid) * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] += v[e];
          }
    }
  }

  // ---- epilogue: lane owns channels nb + 32j + 8q + 4h + {0..3} of pixel pbm + 32i + l32
  OutT* dst = static_cast<OutT*>(a.dst);
  const f16* res = static_cast<const f16*>(a.res);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = tm * BM + wm * (BM / 2) + 32 * i + l32;
    if (m >= a.M) continue;
    const int b = m / HWo, rem = m - (m / HWo) * HWo;
    const int oy = rem / a.Wo, ox = rem - (rem / a.Wo) * a.Wo;
    const int pix = a.shuffle ? (2 * oy) * a.d_W + 2 * ox : oy * a.d_W + ox;
    const size_t obase = (size_t)(b * a.d_P + a.d_pixoff + pix) * a.d_ctot + a.d_coff;
    const size_t rbase = res ? (size_t)(b * a.r_P + oy * a.Wo + ox) * a.r_ctot + a.r_coff : 0;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = tn * BN + wn * (BN / 2) + 32 * j + 8 * q + 4 * h;
        if (n >= a.N) continue;
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bias + n);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = acc[i][j][4 * q + e] + b4[e];
          v[e] = a.act ? ym_silu(x) : x;
        }
        if (res) {
          const f16x4 r4 = *reinterpret_cast<const f16x4*>(res + rbase + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
        }
        if (a.shuffle) {
          const int sub = n / a.npr;
          const int ch = n - sub * a.npr;
          Store4<OutT>::st(dst + obase + (size_t)((sub >> 1) * a.d_W + (sub & 1)) * a.d_ctot + ch, v);
        } else {
          Store4<OutT>::st(dst + obase + n, v);
        }
      }
  }
}

struct DmaCfg {
  int bm, bn, split;
};
constexpr DmaCfg kDma[] = {{64, 64, 1}, {64, 64, 2}, {64, 64, 4}, {64, 64, 8}, {128, 64, 1}, {128, 64, 2},
                           {128, 64, 4}, {64, 128, 1}, {64, 128, 2}, {64, 128, 4}, {128, 128, 1}, {128, 128, 2}};
constexpr int kNumDma = sizeof(kDma) / sizeof(kDma[0]);

template <typename OutT, int BM, int BN, int SPLIT>
hipError_t launch_dma(ConvArgs a, int kind, hipStream_t st) {
  const int tiles_m8 = ((a.M + BM - 1) / BM + 7) / 8 * 8;
  a.tiles_n = (a.N + BN - 1) / BN;
  if (SPLIT > 1) {
    const long tiles = (long)tiles_m8 * a.tiles_n;
    if (tiles > a.cnt_cap || tiles * SPLIT * BM * BN * 4 > a.slab_cap) return hipErrorInvalidValue;
    if (a.Kpad / DK < SPLIT) return hipErrorInvalidValue;
  }
  const dim3 grid(tiles_m8 * a.tiles_n * SPLIT);
  if (kind == 1)
    hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 1, SPLIT>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_dma<OutT, BM, BN, 3, SPLIT>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

template <typename OutT>
hipError_t dispatch(const ConvArgs& a, int kind, int i, hipStream_t st) {
  switch (i) {
    case 0: return launch_dma<OutT, 64, 64, 1>(a, kind, st);
    case 1: return launch_dma<OutT, 64, 64, 2>(a, kind, st);
    case 2: return launch_dma<OutT, 64, 64, 4>(a, kind, st);
    case 3: return launch_dma<OutT, 64, 64, 8>(a, kind, st);
    case 4: return launch_dma<OutT, 128, 64, 1>(a, kind, st);
    case 5: return launch_dma<OutT, 128, 64, 2>(a, kind, st);
    case 6: return launch_dma<OutT, 128, 64, 4>(a, kind, st);
    case 7: return launch_dma<OutT, 64, 128, 1>(a, kind, st);
    case 8: return launch_dma<OutT, 64, 128, 2>(a, kind, st);
    case 9: return launch_dma<OutT, 64, 128, 4>(a, kind, st);
    case 10: return launch_dma<OutT, 128, 128, 1>(a, kind, st);
    case 11: return launch_dma<OutT, 128, 128, 2>(a, kind, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace

int ym_conv_dma_num_cfgs() { return kNumDma; }

// Host-side applicability: f16 plans, 1x1 stride-1 or 3x3 convs, byte offsets < 2^31 for every operand, and a
// 64-aligned concat split (a stage never straddles the two sources).
hipError_t ym_launch_conv_dma(int out_f32, const ConvArgs& a, int i, hipStream_t st) {
  if (i < 0 || i >= kNumDma) return hipErrorInvalidValue;
  int kind;
  if (a.k == 1 && a.s == 1) kind = 1;
  else if (a.k == 3) kind = 3;
  else return hipErrorInvalidValue;
  if (a.Kpad % DK || !a.src0 || a.nchw) return hipErrorInvalidValue;
  if (kind == 1 && a.src1 && a.C0 % DK) return hipErrorInvalidValue;
  const long lim = 0x7FFFFFF0L / 2;  // elements
  if ((long)a.N * a.Kpad > lim || a.s0_elems > lim || a.s1_elems > lim) return hipErrorInvalidValue;
  if ((a.N & 3) || (a.d_ctot & 3) || (a.d_coff & 3)) return hipErrorInvalidValue;
  return out_f32 ? dispatch<float>(a, kind, i, st) : dispatch<f16>(a, kind, i, st);
}
