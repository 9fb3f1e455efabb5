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

// Activation storage precision of a plan: f16 (MFMA 16x16x32 f16) or f32 (exact-f32 MFMA 16x16x4, parity mode).
enum { YM_DT_F16 = 0, YM_DT_F32 = 1 };

// 8 consecutive channels of one pixel: the unit of every NHWC load in this runtime (16 B in f16, 32 B in f32).
template <typename T> struct Vec8;
template <> struct Vec8<f16> {
  typedef f16x8 type;
  static __device__ __forceinline__ type load(const f16* p) { return *reinterpret_cast<const f16x8*>(p); }
  static __device__ __forceinline__ void store(f16* p, type v) { *reinterpret_cast<f16x8*>(p) = v; }
  static __device__ __forceinline__ type zero() { return type{0, 0, 0, 0, 0, 0, 0, 0}; }
};
template <> struct Vec8<float> {
  typedef f32x8 type;
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

// order-preserving float <-> int map (atomicMax on floats of either sign)
__device__ __forceinline__ int f2ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

__device__ __forceinline__ float ym_silu(float x) { return x / (1.0f + expf(-x)); }
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
// Kernel argument blocks (plain structs passed by value).

struct ConvArgs {
  const void* src0; int s0_ctot, s0_coff, C0, s0_W, s0_P, up0;  // first A source; up0: read at (y>>1, x>>1)
  const void* src1; int s1_ctot, s1_coff, C1, s1_P;             // optional second A source (concat tail)
  const void* w; const float* bias;                             // W packed [N][Kpad] (act dtype), bias f32 [N]
  void* dst; int d_ctot, d_coff, d_P, d_pixoff, d_W;            // output view (d_W: dst row width in pixels)
  const void* res; int r_ctot, r_coff, r_P;                     // optional residual view (same geometry as dst)
  int Hin, Win, Ho, Wo, k, s, pad, Cin8, Kc, N, Kpad, act, shuffle, npr, M, tiles_n;
  // stem only: read the caller's NCHW fp32 input directly, applying LoadTensor's /255 rule on load
  const float* nchw; const float* ctl; float eps;
  // LDS-DMA kernels (csrc/ym_conv_dma.hip): operand extents (elements) and the split-K slab/counter workspace
  long s0_elems, s1_elems;
  FDiv fd_hw, fd_w;            // division by Ho*Wo and by Wo
  float* slab; long slab_cap;  // bytes
  int* cnt; int cnt_cap;       // per-tile arrival counters, zero between launches
};

struct DwArgs {
  const void* src; int s_ctot, s_coff, s_P;
  void* dst; int d_ctot, d_coff, d_P;
  const float* w; const float* bias;  // w: [9][C] f32
  int C, H, W, act, B;
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
  int A, kstride, nm, max_det, max_nms, agnostic, B;
  float max_wh, img_h, img_w;
  double iou;
};

struct PrepArgs {
  const float* in; void* out;  // NCHW fp32 → NHWC act dtype, 8 channels (3 real + 5 zero)
  float* ctl;                  // ctl[0] = running max (ordered-int encoded) of the input
  int* cnt; int cnt_len;       // split-K arrival counters, zeroed at the start of every forward
  int B, C, H, W;
  float eps;                   // LoadTensor rule: /255 when max > 1 + eps
};

struct MaskArgs {
  const float* proto; int MH, MW, nm;   // (B, MH, MW, nm) fp32 NHWC prototypes of the last forward
  const float* dets; int max_det, no;   // (B, max_det, no) rows [x1 y1 x2 y2 conf cls coef_0..coef_nm-1]
  const int* offsets; int B, total;     // offsets[b] = first mask row of image b (prefix of kept counts)
  float* lowres;                        // (total, MH, MW) cropped prototype-space masks
  unsigned char* masks; int H, W;       // (total, H, W) 0/1 masks at input resolution
  int* nonempty;                        // (total) 1 when any pixel of the mask is set
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
hipError_t ym_launch_decode(const DecodeArgs& a, hipStream_t st);
hipError_t ym_launch_nms(const NmsArgs& a, hipStream_t st);
hipError_t ym_launch_stem(int dtype, const ConvArgs& a, hipStream_t st);
hipError_t ym_launch_spin(int usec, hipStream_t st);  // profiling: park the stream for usec (wall clock)
hipError_t ym_launch_conv_dma(int out_f32, const ConvArgs& a, int i, hipStream_t st);  // f16 plans only
int ym_conv_dma_num_cfgs();
hipError_t ym_launch_masks(const MaskArgs& a, hipStream_t st);  // Segment: process_mask(upsample=True)
