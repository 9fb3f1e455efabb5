// Shared device/host definitions for the yolomi HIP runtime (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define YM_WAVE 64

// Activation storage precision of a plan: f16 (MFMA 32x32x16 f16), f32 (exact-f32 MFMA 32x32x2, parity mode),
// i8 (PTQ int8: activations stored as q - 128 in int8, weights int8, MFMA 32x32x32 i8 with int32 accumulation), or
// x3 (fp32 storage, every conv GEMM as three f16 MFMAs on split operands: x = hi + lo with hi = fp16(x),
// lo = fp16(x - hi); x·w ≈ hi·w_hi + lo·w_hi + hi·w_lo, fp32 accumulation — ~2^-21 relative, the f16 MFMA rate / 3).
enum { YM_DT_F16 = 0, YM_DT_F32 = 1, YM_DT_I8 = 2, YM_DT_F8 = 3, YM_DT_X3 = 4 };
// plans whose activations are stored fp32 (the exact-f32 parity plan and the split-f16 plan share every non-GEMM kernel)
inline bool ym_dt_f32s(int dt) { return dt == YM_DT_F32 || dt == YM_DT_X3; }
// one-byte quantized plans (int8 affine / fp8 e4m3): same graph, storage and kernels (csrc/ym_quant.h Q8)
inline bool ym_dt_q8(int dt) { return dt == YM_DT_I8 || dt == YM_DT_F8; }

typedef signed char i8;

// x3 plans: an fp32 operand fragment as its fp16 high part and the fp16 rounding of the remainder.  The remainder is
// exact in fp32 and below 2^-11 |x|, so its fp16 rounding may be subnormal: v_mfma_f32_*_f16 keeps fp16 subnormal
// operands (measured on gfx950, tools/x3_probe.hip), so no rescaling of the low part is needed.
struct HL {
  f16x8 hi, lo;
};
__device__ __forceinline__ HL ym_split8(const f32x8& v) {
  HL r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const f16 h = (f16)v[e];
    r.hi[e] = h;
    r.lo[e] = (f16)(v[e] - (float)h);
  }
  return r;
}

// 8 consecutive channels of one pixel: the unit of every NHWC load in this runtime (16 B in f16, 32 B in f32).
template <typename T> struct Vec8;
template <> struct Vec8<f16> {
  typedef f16x8 type;
  typedef f16 elem;  // element type of `type`
  static __device__ __forceinline__ type load(const f16* p) { return *reinterpret_cast<const f16x8*>(p); }
  static __device__ __forceinline__ void store(f16* p, type v) { *reinterpret_cast<f16x8*>(p) = v; }
  static __device__ __forceinline__ type zero() { return type{0, 0, 0, 0, 0, 0, 0, 0}; }
};
template <> struct Vec8<float> {
  typedef f32x8 type;
  typedef float elem;
  static __device__ __forceinline__ type load(const float* p) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    return type{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  }
  static __device__ __forceinline__ void store(float* p, type v) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
  static __device__ __forceinline__ type zero() { return type{0, 0, 0, 0, 0, 0, 0, 0}; }
};

template <> struct Vec8<i8> {  // int8 plans (8 bytes)
  typedef i8 type __attribute__((ext_vector_type(8)));
  typedef i8 elem;
  static __device__ __forceinline__ type load(const i8* p) { return *reinterpret_cast<const type*>(p); }
  static __device__ __forceinline__ void store(i8* p, type v) { *reinterpret_cast<type*>(p) = v; }
  static __device__ __forceinline__ type zero() { return type{0, 0, 0, 0, 0, 0, 0, 0}; }
};

// x3 activation storage ("pair" layout): every chunk of 8 logical channels is 32 bytes, [fp16 hi x8 | fp16 lo x8], the
// split made once by the producer's epilogue.  A P2 is one logical element (4 bytes), so NHWC pointer arithmetic in
// P2 units (pixel * ctot + coff + c) lands on chunk starts for c % 8 == 0 exactly as with f16 / fp32 storage; every
// buffer is 256-byte aligned and its channel counts are multiples of 8, so chunks are 32-byte aligned.  Seen as fp16,
// a pair buffer is an NHWC tensor of 2C channels whose chunk 2j is the hi part of logical chunk j and 2j + 1 its lo
// part: the LDS-DMA / streaming GEMM loaders fetch it unchanged, with doubled channel counts.
struct P2 {
  unsigned bits;
};
template <> struct Vec8<P2> {
  typedef f32x8 type;  // hi + lo (one fp32 rounding: exact for every split value pair the epilogues store)
  typedef float elem;
  static __device__ __forceinline__ type load(const P2* p) {
    const f16x8 h = *reinterpret_cast<const f16x8*>(p), lo = *(reinterpret_cast<const f16x8*>(p) + 1);
    type v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)h[e] + (float)lo[e];
    return v;
  }
  static __device__ __forceinline__ void store(P2* p, type v) {
    const HL x = ym_split8(v);
    *reinterpret_cast<f16x8*>(p) = x.hi;
    *(reinterpret_cast<f16x8*>(p) + 1) = x.lo;
  }
  static __device__ __forceinline__ type zero() { return type{0, 0, 0, 0, 0, 0, 0, 0}; }
};
__device__ __forceinline__ HL ym_load_hl(const P2* p) {
  return HL{*reinterpret_cast<const f16x8*>(p), *(reinterpret_cast<const f16x8*>(p) + 1)};
}
// 4 consecutive logical channels (c % 4 == 0) at P2 address p: their hi halves sit at byte 2 (c % 8) of the chunk,
// the lo halves 16 bytes further
__device__ __forceinline__ f16* ym_p2_hi4(P2* p) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  return reinterpret_cast<f16*>((u & ~(uintptr_t)31) + ((u & 31) >> 1));
}
__device__ __forceinline__ const f16* ym_p2_hi4(const P2* p) { return ym_p2_hi4(const_cast<P2*>(p)); }
// SC1: write-through stores (sc1: the line leaves this XCD's L2 at once), for a consumer workgroup of the same
// launch on any XCD (the persistent chain kernel, csrc/ym_conv_dma.hip; cdna_hip_programming.md §6 Guideline 16)
template <bool SC1 = false>
__device__ __forceinline__ void ym_p2_store4(P2* p, const float* v) {
  f16x4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (f16)v[e];
    l[e] = (f16)(v[e] - (float)h[e]);
  }
  f16* q = ym_p2_hi4(p);
  if constexpr (SC1) {
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    __hip_atomic_store((gu64*)q, __builtin_bit_cast(unsigned long long, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu64*)(q + 8), __builtin_bit_cast(unsigned long long, l), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *reinterpret_cast<f16x4*>(q) = h;
    *reinterpret_cast<f16x4*>(q + 8) = l;
  }
}
// v of lane ^ XOR (XOR 16 or 32): ds_bpermute (LDS crossbar), or with `vp` the VALU row swap v_permlane16_swap /
// v_permlane32_swap with one register as both operands — the odd 16-lane rows (32: the upper half) find the partner's
// value in the first result, the others in the second (tools/permlane_probe.hip)
template <int XOR>
__device__ __forceinline__ unsigned ym_lane_xor(unsigned v, bool vp) {
  static_assert(XOR == 16 || XOR == 32, "row swaps: lane ^ 16 or lane ^ 32");
  if (vp) {
    const bool upper = (threadIdx.x & XOR) != 0;
    if constexpr (XOR == 16) {
      const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
      return upper ? r[0] : r[1];
    } else {
      const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      return upper ? r[0] : r[1];
    }
  }
  return (unsigned)__shfl_xor((int)v, XOR);
}
// The same 4 channels stored by a LANE PAIR: the lane holding channels c .. c+3 of a chunk (c % 8 == 0, `odd` false)
// and its partner lane (lane ^ XOR, same pixel) holding c+4 .. c+7 swap halves, so the even lane writes the chunk's
// hi x8 (16 B) and the odd lane its lo x8 (16 B) — the chunk is one 32-byte run, not four 8-byte pieces
// (tools/store_probe.hip: the 8-byte pattern of ym_p2_store4 writes HBM at 4.8-5.4 TB/s, 32-byte runs at 6.5-6.9).
// Same stored bits as ym_p2_store4.  Both lanes of a pair must execute it (the exchange is a cross-lane read);
// `ok` predicates only the store, and p may be any address when !ok.
// SC1: write-through (see ym_p2_store4), as a buffer store off the wave-uniform `base` (offsets < 2^31 bytes)
template <int XOR, bool SC1 = false>
__device__ __forceinline__ void ym_p2_store4_pair(P2* p, const float* v, bool odd, bool ok, bool vp = false,
                                                  const void* base = nullptr) {
  f16x4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (f16)v[e];
    l[e] = (f16)(v[e] - (float)h[e]);
  }
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  const u32x2_t s = __builtin_bit_cast(u32x2_t, odd ? h : l);  // the half the partner stores
  u32x2_t r;
  r[0] = ym_lane_xor<XOR>(s[0], vp);
  r[1] = ym_lane_xor<XOR>(s[1], vp);
  const f16x4 q = __builtin_bit_cast(f16x4, r);
  const f16x8 o = odd ? f16x8{q[0], q[1], q[2], q[3], l[0], l[1], l[2], l[3]}
                      : f16x8{h[0], h[1], h[2], h[3], q[0], q[1], q[2], q[3]};
  if (ok) {
    const uintptr_t u = reinterpret_cast<uintptr_t>(p);
    if constexpr (SC1) {  // one 16-byte write-through store: a buffer store with the sc1 bit (aux 16)
      const uintptr_t t = (u & ~(uintptr_t)31) + (odd ? 16 : 0);
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFF0,
                                                                         0x00020000);
      typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), r,
                                             (unsigned)(t - reinterpret_cast<uintptr_t>(base)), 0, 16);
    } else {
      *reinterpret_cast<f16x8*>((u & ~(uintptr_t)31) + (odd ? 16 : 0)) = o;
    }
  }
}
__device__ __forceinline__ void ym_p2_load4(const P2* p, float* v) {  // v[e] = hi + lo
  const f16* q = ym_p2_hi4(p);
  const f16x4 h = *reinterpret_cast<const f16x4*>(q), l = *reinterpret_cast<const f16x4*>(q + 8);
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (float)h[e] + (float)l[e];
}
// one logical element (scalar paths)
__device__ __forceinline__ float ym_p2_get(const P2* p) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  const f16* q = reinterpret_cast<const f16*>((u & ~(uintptr_t)31) + ((u & 31) >> 1));
  return (float)q[0] + (float)q[8];
}
__device__ __forceinline__ void ym_p2_set(P2* p, float v) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  f16* q = reinterpret_cast<f16*>((u & ~(uintptr_t)31) + ((u & 31) >> 1));
  const f16 h = (f16)v;
  q[0] = h;
  q[8] = (f16)(v - (float)h);
}

// order-preserving float <-> int map (atomicMax on floats of either sign)
__device__ __forceinline__ int f2ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

// The input statistics word of a forward (LoadTensor's batch max) is spread over YM_CTL_SLOTS atomicMax targets 64 B
// apart (same-address atomics serialise at ~90 per µs); readers take the max of the slots.
constexpr int YM_CTL_SLOTS = 16, YM_CTL_STRIDE = 16;  // ints
// the ctl region: the slots, a ticket on its own 256-byte line, input_stats' per-block partial maxima, then its
// YM_STATS_GROUPS group tickets 128 B apart
constexpr int YM_STATS_GROUPS = 16;
constexpr int YM_CTL_BYTES = (YM_CTL_SLOTS * YM_CTL_STRIDE + 64 + 1024 + 32 * YM_STATS_GROUPS) * 4;
static_assert(YM_CTL_BYTES <= 8192, "ym_input_max's region of the context scratch (ym_runtime.cpp d_misc)");
__device__ __forceinline__ float ym_input_max(const float* ctl) {
  const int* c = reinterpret_cast<const int*>(ctl);
  int m = c[0];
#pragma unroll
  for (int s = 1; s < YM_CTL_SLOTS; ++s) m = max(m, c[s * YM_CTL_STRIDE]);
  return ord2f(m);
}

// A value the compiler cannot see through: keeps `a * b` and a following `+ c` as two roundings.  hipcc compiles
// with -ffp-contract=fast, which fuses across statements, ignores `#pragma clang fp contract`, and sees straight through
// HIP's __fmul_rn / __fadd_rn (plain operators); parity with torch's separate fp32 ops needs the two roundings.
__device__ __forceinline__ float ym_opaque(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ float ym_silu(float x) { return x / (1.0f + expf(-x)); }
// x3 plans: SiLU from the hardware exp2 and reciprocal, the reciprocal refined by one Newton step (denominator
// clamped below inf so the step stays finite): ~2 ulp plus the exp2 argument's rounding (|x|·2^-24·ln 2 relative) —
// far below the x3 GEMMs' ~2^-21 operand precision, in ~7 VALU instructions instead of expf + IEEE division's ~25
// (the x3 epilogues were VALU-bound on them: every conv output element pays one SiLU)
__device__ __forceinline__ float ym_silu_x3(float x) {
  const float d = fminf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x), 1e30f);
  float r = __builtin_amdgcn_rcpf(d);
  r = fmaf(r, fmaf(-d, r, 1.0f), r);
  return x * r;
}
// SiLU from the hardware exp2 / reciprocal (each ~1 ulp): for epilogues whose outputs are rounded to fp16 anyway
__device__ __forceinline__ float ym_silu_fast(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// Division by a runtime constant d >= 1 for 0 <= n < 2^31: n / d == (n * m) >> p with p = 31 + ceil(log2 d),
// m = ceil(2^p / d) < 2^32 (the rounding error m*d - 2^p < d <= 2^(p-31) keeps the floor exact).
struct FDiv {
  unsigned m;
  int p;
};
inline FDiv ym_fdiv(int d) {
  int s = 0;
  while ((1LL << s) < d) ++s;
  const int p = 31 + s;
  return FDiv{(unsigned)(((1ULL << p) + (unsigned long long)d - 1) / (unsigned long long)d), p};
}
__device__ __forceinline__ int ym_div(int n, FDiv f) { return (int)(((unsigned long long)(unsigned)n * f.m) >> f.p); }
__device__ __forceinline__ float ym_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }

// ------------------------------------------------------------------------------------------------------------
// int8 (PTQ) quantisation record of one op, stored in the weight blob (yolomi/plan.py `_qrec`; semantics:
// oracle/quant.py).  A quantized conv: acc = Σ (q_x - z_x)·q_w (int32, exact; the int8 storage holds q - 128, the
// difference is folded into a per-channel int32 bias), y = float(acc)·sasw[n] + bias[n] (two fp32 roundings),
// q_c = clamp(rint(y·inv_sc) + zc, qlo, qhi); then by mode
//   0: v = post[q_c] (+ residual (q_r - z_r)·s_r), stored as clamp(rint(v·inv_so) + zo, qlo, qhi) - 128,
//   1: stored as q_c - 128 (the tensor keeps the conv's own output quantisation: Attention.qkv, Proto.upsample),
//   2: v written as fp32 (terminal head outputs).
struct QRec {
  float inv_sc; int zc;  // conv output requantisation (1 / s_out, zero point)
  int qlo, qhi;          // [0, 255], or [0, 127] with reduce_range
  int mode;
  float inv_so; int zo;  // stored tensor (mode 0)
  float s_r; int z_r;    // residual tensor
  float s_in; int z_in;  // input tensor (dequantisation; 3x3 padding reads z_in)
  float inv_s_in;        // stem: quantisation of the image
  int pad[4];
  float post[256];       // post[q] = act((q - zc)·s_out) (SiLU in float64, rounded to fp32) or the plain dequant
};

// ------------------------------------------------------------------------------------------------------------
// Kernel argument blocks (plain structs passed by value).

// XCD-contiguous block order: the dispatcher deals workgroups round-robin over the 8 XCDs (bid % 8), each with its
// own L2.  Renumber so XCD x runs one contiguous range of logical blocks: neighbouring output tiles (whose 3x3
// windows share input rows) then read those rows through the same L2 instead of fetching them from HBM once per
// XCD.  A bijection for any grid size; placement only affects speed, never results.  Used by the stem (yolo11n
// B=8: 22.7 -> 19.8 us), the depthwise / SPPF / attention kernels, conv_small, conv_halo, conv_bneck and the int8
// convs; conv_igemm / conv_lds / conv_dma (xcd_tile) and conv_stream (per-XCD group ranges) map their tiles
// XCD-contiguously in their own tile maps — conv HBM traffic of yolo11s B=8 1.46x -> 1.21x the algorithmic bytes.
__device__ __forceinline__ int ym_xcd_block(int bid, int n) {
  const int q = n >> 3, r = n & 7, x = bid & 7;
  return x * q + (x < r ? x : r) + (bid >> 3);
}

struct ConvArgs {
  const void* src0; int s0_ctot, s0_coff, C0, s0_W, s0_P, up0;  // first A source; up0: read at (y>>1, x>>1)
  const void* src1; int s1_ctot, s1_coff, C1, s1_P;             // optional second A source (concat tail)
  const void* w; const float* bias;                             // W packed [N][Kpad] (act dtype), bias f32 [N]
  void* dst; int d_ctot, d_coff, d_P, d_pixoff, d_W;            // output view (d_W: dst row width in pixels)
  const void* res; int r_ctot, r_coff, r_P;                     // optional residual view (same geometry as dst)
  int Hin, Win, Ho, Wo, k, s, pad, Cin8, Kc, N, Kpad, act, shuffle, npr, M, tiles_n;
  // stem only: read the caller's NCHW fp32 input directly, applying LoadTensor's /255 rule on load
  const float* nchw; const float* ctl; float eps;
  const float* wstem;          // stem weights, fp32 [27][N] (tap (ky, kx, c)-major), re-laid out at load
  // LDS-DMA kernels (csrc/ym_conv_dma.hip): operand extents (elements) and the split-K slab/counter workspace
  long s0_elems, s1_elems;
  FDiv fd_hw, fd_w;            // division by Ho*Wo and by Wo
  float* slab; long slab_cap;  // bytes
  int* cnt; int cnt_cap;       // per-tile arrival counters, zero between launches
  // int8 plans: quantisation record, per-channel s_in·s_w and the int32 zero-point correction Σ_k (128 - z_in)·w
  const QRec* q; const float* sasw; const int* biasi;
  float* raw;                  // f32 calibration runs: pre-activation conv output, (M, N) row-major, or null
  // fused pair (f16 streaming kernels): a following 1x1 conv consumes this conv's activated output straight from
  // registers — out = act2(W2 · h + bias2) (+ res) with h = fp16(act(W · x + bias)); dst/res then describe the
  // second conv's output.  w2 [N2][Kpad2] (K = this conv's N output channels), null for a single conv.
  const void* w2; const float* bias2; int N2, Kpad2, act2;
  // successor kernel size: 1 = the 1x1 above (streaming FUSE); 3 = a YOLO11 Bottleneck's second 3x3 conv, dst/res the
  // Bottleneck output / shortcut (csrc/ym_conv_bneck.hip); w2 then [N2][Kpad2] with K = (ky, kx, mid channel)
  int k2;
  // x3 plans: activations in the pair layout (P2), weights [N][Kpad] fp16 with every 8-channel K chunk as [hi x8 |
  // lo x8]; Cin8 / Kc / Kpad then count fp16 storage chunks (twice the logical ones), ctot / coff / C0 / C1 / d_* / r_*
  // stay logical channels, s0_elems / s1_elems count fp16 elements
  int x3;
  // x3 pair-layout outputs: lane-pair whole-chunk epilogue stores (ym_p2_store4_pair) where the output slice allows
  // them; a bit mask per kernel family (1 LDS-DMA, 2 streaming, 4 stem, 8 fused Bottleneck; 16: the lane exchange
  // by v_permlane*_swap instead of ds_bpermute; YM_PAIRST for A/B); a clear family bit keeps the per-lane
  // ym_p2_store4.  Same stored bits either way.  Default 21 = LDS-DMA + stem with permlane: the families whose ops
  // got faster in two same-box A/Bs (model.1+cv1 83 -> 79 us, stem 40 -> 38, the 80x80 head 1x1s -1.2 us each);
  // the streaming kernel lost (model.2.cv2 55 -> 61 us) and the Bottleneck kernel ~1 us (profiles/r03i_pairst_ab.txt).
  int pst;
  // x3 plans: every conv weight matrix (W, and W2 of a fused pair) is packed scaled by a power of two 2^s, its max |w|
  // then in (2^13, 2^14] (yolomi/plan.py), so that the fp16 lo parts of the split stay normal: unscaled, a weight of
  // 0.03 kept only ~1e-6 relative precision in a subnormal lo (tools/x3_emulate.py: the x3 plan's max |Δxy| 1.3e-3 ->
  // 7.6e-4 px, the fp32 oracle's own distance from float64 being 8.2e-4).  wsc / wsc2 = 2^-s undo it exactly in the
  // epilogue: fmaf(acc, wsc, bias) rounds once, as acc + bias did (ym_x3_pre).  1 for every other plan.
  float wsc, wsc2;
  // LDS-DMA kernels (csrc/ym_conv_dma.hip): request every line of the workgroup's K range into L2 before the ring
  // starts (latency-bound small-M layers; YM_DMA_PF = the largest M it is used for, 0 = never)
  int pf;
  // fused depthwise (yolomi/arch.py GraphBuilder.fuse_dw; csrc/ym_conv_dwpw.hip): src0 is the DEPTHWISE input and this
  // 1x1 conv consumes act(dw3x3(src0) + dw_b) computed in registers.  dw_w [9][C0] fp32, dw_b [C0]; null: no depthwise
  const float* dw_w; const float* dw_b; int dw_act;
  // LDS-DMA kernels (csrc/ym_conv_dma.hip launch_dma): the tile map's divisions, set on the host — tiles_n and Cin8 as
  // multiply-shift divisors, the pixel tiles per XCD — instead of runtime integer divisions in every workgroup's prologue
  FDiv fd_tn, fd_cin8;
  int tm_per_xcd;
  // int8 plans on the LDS-DMA kernels (round 6): per 3x3 tap the column sums of W, [9][N] int32 — the DMA fills
  // out-of-image taps with 0 (the stored q - 128 of q = 128), the quantized conv reads z_in there, so a border pixel's
  // accumulator gets (z_in - 128)·Σ over its outside taps of wtap[t][n] (ym_runtime.cpp computes the table at load)
  const int* wtap;
};

// Warm the scalar cache with every 64-byte line of a kernel's argument block in ONE round trip: the compiler loads
// kernel arguments lazily at first use, each batch of s_loads ending in an lgkmcnt(0) wait for a line that is not in
// the scalar cache yet (a graph replay's argument block is cold): ~6 dependent round trips for a ConvArgs block
// before the first DMA issue (tools/dma_probe.hip prologue stamps: "index setup" 3.2k cycles).  After this the lazy
// loads hit the cache.
template <int BYTES>
__device__ __forceinline__ void ym_warm_kernargs() {
  const __attribute__((address_space(4))) char* kp =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  static_assert(BYTES <= 16 * 64, "argument block too large");
  int v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i * 64 < BYTES) v[i] = *(const __attribute__((address_space(4))) int*)(kp + i * 64);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i * 64 < BYTES) asm volatile("" ::"s"(v[i]));
}

// A load through the global address space (global_load, vmcnt only; a generic pointer makes the compiler emit a
// flat load, which also counts in lgkmcnt and so is waited for together with the scalar/LDS traffic).
template <typename T>
__device__ __forceinline__ T ym_gld(const void* p) {
  return *(const __attribute__((address_space(1))) T*)(p);
}

// x3 epilogue pre-activation: the weight scale (exact: a power of two) and the bias in one rounding
__device__ __forceinline__ float ym_x3_pre(float acc, float wsc, float bias) { return fmaf(acc, wsc, bias); }

struct DwArgs {
  const void* src; int s_ctot, s_coff, s_P;
  void* dst; int d_ctot, d_coff, d_P;
  const float* w; const float* bias;  // w: [9][C] f32
  int C, H, W, act, B;
  const i8* wq; const QRec* q; const float* sasw;  // int8 plans: w [9][C] int8
  float* raw;                                      // f32 calibration runs: pre-activation output (B·H·W, C)
};

struct PoolArgs {
  void* buf; int ctot, coff, P;  // y0 at coff, writes y1,y2,y3 at coff+C, +2C, +3C
  int C, H, W, B;
  int sep;                       // separable (row-max images in LDS) vs direct 2-D windows
};

struct AttnArgs {
  const void* qkv; int q_ctot, q_coff, q_P;
  void* dst; int d_ctot, d_coff, d_P;
  const float* pe_w; const float* pe_b;  // [9][C], [C]
  int C, nh, kd, hd, H, W, N, B;
  float scale;
  const i8* pe_wq; const QRec* q; const float* pe_sasw;  // int8 plans (q: pe output, qkv input, attn.x store)
  float* raw;                                            // f32 calibration runs: pe(v) before the add, (B·N, C)
};

struct ReqArgs {  // int8 plans: dst slice = requantised (optionally 2x nearest up-sampled) src slice
  const i8* src; int s_ctot, s_coff, s_P, s_W, up;
  i8* dst; int d_ctot, d_coff, d_P, d_W;
  int C, H, W, B;  // dst geometry
  const QRec* q;   // s_in / z_in: source, inv_so / zo: destination
};

struct DecodeArgs {
  const float* anchors; int no_tot;      // (B, A, no_tot) fp32
  float4* boxes; float* scores; int* cls;  // (B, A)
  unsigned long long* keys; int* counts;   // (B, A) candidate keys, (B) counts
  int A, kstride, nc, reg_max, B;
  int lvl_W[4], lvl_off[4], nl; float lvl_stride[4];
  float conf; int has_classes; unsigned int classes[4];
};

struct NmsArgs {
  const float* anchors; int no_tot, mask_off;  // mask coefficients live at [mask_off, mask_off+nm) of each anchor row
  const float4* boxes; const float* scores; const int* cls;
  unsigned long long* keys; const int* counts;
  float4* sboxes; float* sareas; unsigned char* sup;  // per image scratch (A each)
  float* dets; int* out_counts;                       // (B, max_det, 6 + nm), (B)
  int* counts2;  // non-null (ym_infer_args.counts_after_dets): the counts again, in the words after the batch's rows
  int A, kstride, nm, max_det, max_nms, agnostic, B;
  int nc;  // classes (the blocked path's class filter takes nc <= NMS_NC)
  float max_wh, img_h, img_w;
  double iou;
  int dbg;  // YM_NMS_DBG: 1-7 phase ablations of the bit-matrix path, 10 the blocked path's sort alone (timing only);
            // 9 disables the blocked path
  // multi-workgroup presort (low conf: ym_launch_nms_presort before nms_image): chunk-sorted keys, and 1 when the
  // keys arrive sorted for the blocked path
  unsigned long long* keys2; int presorted;
};

struct LetterboxArgs {
  const unsigned char* src; int h, w, row_bytes, bgr;  // HWC uint8 image (3 channels), BGR or RGB order
  int uh, uw, top, left;                               // resized (unpadded) size and its offset in the canvas
  double scale_x, scale_y;                             // 1 / ((double)uw / w), 1 / ((double)uh / h)
  float* dst; int Hn, Wn;                              // one image of the fp32 NCHW batch (3 planes of Hn x Wn)
};

struct PrepArgs {
  const float* in; void* out;  // NCHW fp32 → NHWC act dtype, 8 channels (3 real + 5 zero)
  float* ctl;                  // ctl[0] = running max (ordered-int encoded) of the input
  int* cnt; int cnt_len;       // split-K arrival counters, zeroed at the start of every forward
  int B, C, H, W;
  float eps;                   // LoadTensor rule: /255 when max > 1 + eps
  const float* batch_max;      // non-null: the (global) batch max is given, skip the reduction
};

struct MaskArgs {
  const float* proto; int MH, MW, nm;   // (B, MH, MW, nm) fp32 NHWC prototypes of the last forward
  const float* dets; int max_det, no;   // (B, max_det, no) rows [x1 y1 x2 y2 conf cls coef_0..coef_nm-1]
  const int* offsets; int B, total;     // offsets[b] = first mask row of image b (prefix of kept counts)
  float* lowres;                        // (total, MH, MW) cropped prototype-space masks
  unsigned char* masks; int H, W;       // (total, H, W) 0/1 masks at input resolution
  int* nonempty;                        // (total) 1 when any pixel of the mask is set
  const int* counts; int cap;           // slot mode (counts != null): mask d = slot (d / cap, d % cap), used while
                                        // d % cap < counts[d / cap]; total = B * cap; nonempty[B*cap + b] = counts[b]
};

// ------------------------------------------------------------------------------------------------------------
// Host-side launchers (defined in the .hip translation units).
// cfg < 0: heuristic; strict: an inapplicable cfg is an error (else the heuristic runs)
hipError_t ym_launch_conv(int dtype, int out_f32, const ConvArgs& a, int cfg, hipStream_t st, bool strict = false);
int ym_conv_num_cfgs();
hipError_t ym_launch_dwconv(int dtype, const DwArgs& a, hipStream_t st);
hipError_t ym_launch_sppf(int dtype, const PoolArgs& a, hipStream_t st);
hipError_t ym_launch_attn(int dtype, const AttnArgs& a, hipStream_t st);
hipError_t ym_launch_prep(int dtype, const PrepArgs& a, int* counts, int B, hipStream_t st);
hipError_t ym_launch_input_max(const float* x, long n, float* ctl, float* out, hipStream_t st);
hipError_t ym_launch_decode(const DecodeArgs& a, hipStream_t st);
hipError_t ym_launch_nms(const NmsArgs& a, hipStream_t st);
hipError_t ym_launch_nms_presort(const NmsArgs& a, hipStream_t st);  // ym_misc.hip: keys sorted by 8 WGs per image
hipError_t ym_launch_conv_dma_i8(const ConvArgs& a, int dma_cfg, hipStream_t st);  // ym_conv_dma.hip
hipError_t ym_launch_conv_dma_chain(const ConvArgs& a0, const ConvArgs& a1, int dma_cfg, int* ctl, int cap,
                                    hipStream_t st);  // csrc/ym_conv_dma.hip: two dependent x3 convs, one launch
hipError_t ym_launch_stem_down_x3(const ConvArgs& s, const ConvArgs& p, hipStream_t st);  // ym_stem_fused.hip
int ym_debug_get(int key);  // ym_set_debug switches (ym_misc.hip)
int ym_debug_set(int key, int value);
void ym_debug_add(int key, int d);
const void* ym_nms_kernel();  // the NMS kernel's function (graph replays re-point its output rows: ym_infer)
hipError_t ym_launch_stem(int dtype, const ConvArgs& a, hipStream_t st);
hipError_t ym_launch_letterbox(const LetterboxArgs& a, hipStream_t st);
hipError_t ym_launch_spin(int usec, hipStream_t st);  // profiling: park the stream for usec (wall clock)
hipError_t ym_launch_conv_dma(int out_f32, const ConvArgs& a, int i, hipStream_t st);  // f16 plans only
int ym_conv_dma_num_cfgs();
hipError_t ym_launch_conv_dma_fuse(int out_f32, const ConvArgs& a, int i, hipStream_t st);  // x3 conv -> 1x1 pairs
int ym_conv_dma_x3_num_cfgs();  // x3-only LDS-DMA configurations (op cfg ids from ym_conv_num_cfgs() on)
int ym_conv_num_cfgs_dt(int dtype);  // conv-config catalogue size of a plan dtype (YM_DT_*)
hipError_t ym_launch_conv_bneck(int out_f32, const ConvArgs& a, int i, hipStream_t st);  // fused Bottleneck
int ym_conv_bneck_num_cfgs();
int ym_conv_bneck_x3_num_cfgs();  // x3-only Bottleneck variants (launch indices from ym_conv_bneck_num_cfgs() on)
hipError_t ym_launch_conv_stream(int out_f32, const ConvArgs& a, int i, hipStream_t st);  // f16 1x1 only
int ym_conv_stream_num_cfgs();
hipError_t ym_launch_conv_halo(int out_f32, const ConvArgs& a, int i, hipStream_t st);  // f16 3x3 halo tiles
hipError_t ym_launch_conv_dwpw(int dtype, int out_f32, const ConvArgs& a, int cfg, hipStream_t st, bool strict);
int ym_conv_dwpw_num_cfgs();  // fused depthwise → 1x1 (ConvArgs::dw_w): its own cfg id space 0 .. n-1
int ym_conv_halo_num_cfgs();
hipError_t ym_launch_masks(const MaskArgs& a, hipStream_t st);
bool ym_masks_fused(const MaskArgs& a);  // the one-launch path (no (total, MH, MW) scratch)  // Segment: process_mask(upsample=True)
// int8 (PTQ) plans: csrc/ym_conv_i8.hip
// (f8: the fp8 e4m3 PTQ plan on the same kernels, csrc/ym_quant.h Q8<true>)
hipError_t ym_launch_conv_i8(const ConvArgs& a, int cfg, hipStream_t st, bool strict, bool f8);
int ym_conv_i8_num_cfgs();
hipError_t ym_launch_conv_i8_stream(const ConvArgs& a, int i, hipStream_t st, bool f8);
int ym_conv_i8_stream_num_cfgs();
hipError_t ym_launch_dwconv_i8(const DwArgs& a, hipStream_t st, bool f8);
hipError_t ym_launch_attn_i8(const AttnArgs& a, hipStream_t st, bool f8);
hipError_t ym_launch_requant(const ReqArgs& a, hipStream_t st, bool f8);
