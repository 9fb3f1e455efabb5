// Bandwidth-/latency-bound kernels of the YOLO11 inference path on gfx950:
//   input statistics (LoadTensor /255 rule), depthwise 3x3 (Detect cv3 DWConv), fused SPPF max-pool pyramid, C2PSA
//   attention (+ fused positional depthwise conv), anchor-free DFL decode, class-offset greedy NMS.
// Each replaces an upstream Ultralytics/ATen/torchvision op reached from `YOLO11Model.predict`
// (/root/reference/core/model.py:133) — SURVEY §2.2 and §8a rows a2, a8, a9, a11-a14.
#include <stdlib.h>

#include <type_traits>

#include <atomic>

#include "ym_common.h"

namespace {

// ------------------------------------------------------------------------------------------------- input stats
// LoadTensor._single_check: `if im.max() > 1 + finfo(dtype).eps: im = im.float() / 255` over the WHOLE batch.
// ctl[0] holds max as an order-preserving int (ym_input_max reads the YM_CTL_SLOTS slots).
// The division itself happens in the stem conv's loader (csrc/ym_stem.hip), which reads the NCHW batch.
//
// input_stats: the forward's first kernel, one launch.  Every block zeroes its share of the per-image candidate
// counts and the split-K tile counters (csrc/ym_conv_dma.hip; self-resetting, cleared here as a guard against an
// aborted forward), reduces a contiguous chunk of the batch to its max and stores it write-through (sc1) into its
// partial slot; after its `vmcnt(0)` one lane takes an agent-scope ticket, and the block whose ticket is last
// reduces the partials (sc1 loads: the hand-off of MI355X_MICROARCH §inter-workgroup visibility, first table row),
// writes the slots and resets the ticket.  The ticket is two-level: block b counts on group ticket b % 16 and the
// last block of each group on the top ticket — same-address agent-scope atomics serialise at ~10 ns each, so one
// ticket for 1,024 blocks cost ~10 us of the kernel's ~28 (tools/probe_input_stats.hip, profiles/r06j_input_stats.txt:
// 27.9 -> 20.3 us in isolation, 17.9 with no ticket at all).  No per-forward init kernel, no same-address atomicMax storm.  The ticket
// starts at zero (ensure_workspace zeroes the arena it lives in), and a launch can only stop part-way through a device
// fault, which ends the context: a stale ticket cannot carry into a later forward.
// batch_max non-null (multi-GPU shard): the slots take the given global max, x is not read.
constexpr int kStatsBlocks = 1024;  // partial slots (ym_runtime.cpp reserves them behind the ctl slots)
constexpr int kStatsU = 10;         // float4 loads in flight per lane and round
__global__ __launch_bounds__(256) void input_stats(const float* __restrict__ x, long n, float* ctl, int* counts, int B,
                                                   int* cnt, int cnt_len, const float* batch_max) {
  const int tid = threadIdx.x;
  const long gt = blockIdx.x * 256L + tid, gstride = (long)gridDim.x * 256;
  for (long b = gt; b < B; b += gstride) counts[b] = 0;
  int4* c4 = reinterpret_cast<int4*>(cnt);
  for (long i = gt; i < cnt_len / 4; i += gstride) c4[i] = make_int4(0, 0, 0, 0);
  int* slots = reinterpret_cast<int*>(ctl);
  if (batch_max) {
    if (blockIdx.x == 0 && tid < YM_CTL_SLOTS) slots[tid * YM_CTL_STRIDE] = tid == 0 ? f2ord(*batch_max) : f2ord(-INFINITY);
    return;
  }
  int* part = slots + YM_CTL_SLOTS * YM_CTL_STRIDE + 64;  // [kStatsBlocks], after the ticket's 256-byte line
  int* ticket = slots + YM_CTL_SLOTS * YM_CTL_STRIDE;
  int* gticket = part + kStatsBlocks;                     // [YM_STATS_GROUPS][32]
  // contiguous chunk of whole float4s per block; every round issues kStatsU 16-byte loads per lane at once, the
  // indices past the chunk clamped onto its last float4 (a duplicate cannot change a max), so there is no
  // predicated or remainder load: at B = 8, 640² (2400 float4 per block) the whole chunk is ONE round trip
  const long n4 = n >> 2;
  const long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long lo = blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  float m = -INFINITY;
  for (long i = lo + tid; lo < hi && i - tid < hi; i += kStatsU * 256) {
    f32x4 v[kStatsU];
#pragma unroll
    for (int u = 0; u < kStatsU; ++u) {
      const long j = i + u * 256;
      v[u] = x4[j < hi ? j : hi - 1];  // (plain loads: the stem reads the batch next)
    }
#pragma unroll
    for (int u = 0; u < kStatsU; ++u) m = fmaxf(m, fmaxf(fmaxf(v[u][0], v[u][1]), fmaxf(v[u][2], v[u][3])));
  }
  if (blockIdx.x == 0)
    for (long j = (n4 << 2) + tid; j < n; j += 256) m = fmaxf(m, x[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float wm[4];
  __shared__ int last;
  if ((tid & 63) == 0) wm[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    // the sc1 hand-off (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md § visibility, the counter row):
    // the partial is stored write-through (an agent-scope relaxed store is sc1) and drained before the agent-scope
    // ticket; the last block reads every partial with sc1 loads (agent-scope relaxed loads), so neither side needs a
    // fence instruction.  (An acquire-release ticket puts an L2 write-back in every one of the 1,024 blocks: the
    // kernel went 21.8 -> 52.8 us per call under rocprofv3: profiles/r04d_s_b8_x3_summary.json vs r05c.)
    __hip_atomic_store(part + blockIdx.x, f2ord(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int g = blockIdx.x % YM_STATS_GROUPS, ng = ((int)gridDim.x - g + YM_STATS_GROUPS - 1) / YM_STATS_GROUPS;
    const int t = __hip_atomic_fetch_add(gticket + 32 * g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int l = 0;
    if (t == ng - 1) {  // the group's last block: its count is complete, so every partial of the group is stored
      __hip_atomic_store(gticket + 32 * g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int u = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      l = u == min((int)gridDim.x, YM_STATS_GROUPS) - 1;
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below the ticket
  int r = f2ord(-INFINITY);
  for (int b = tid; b < (int)gridDim.x; b += 256)
    r = max(r, __hip_atomic_load(part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) r = max(r, __shfl_xor(r, o));
  __shared__ int wr[4];
  if ((tid & 63) == 0) wr[tid >> 6] = r;
  __syncthreads();
  if (tid < YM_CTL_SLOTS)
    slots[tid * YM_CTL_STRIDE] = tid == 0 ? max(max(wr[0], wr[1]), max(wr[2], wr[3])) : f2ord(-INFINITY);
  if (tid == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void ctl_to_max(const float* ctl, float* out) {
  if (threadIdx.x == 0) *out = ym_input_max(ctl);
}

// ------------------------------------------------------------------------------------------------- depthwise 3x3
// DWConv(c, c, 3) = Conv(g=c): 3x3, stride 1, pad 1, BN folded, SiLU.  One thread = 8 channels of one pixel.
// Every load a thread needs (9 taps x 16 B of activations, 9 x 2 float4 of weights + 2 of bias, the weights L1/L2-
// resident) is independent and issued up front: one memory latency per thread, no LDS staging loop (a strided
// staging loop of 10·C floats was ~10 dependent global round trips for C = 512).
template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3(const DwArgs a) {
  const int C8 = a.C >> 3;
  // 32-bit index math (checked < 2^31 on the host); each XCD owns one contiguous run of blocks (shared tap rows)
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
  const T* src = static_cast<const T*>(a.src);
  typename Vec8<T>::type v[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
    v[t] = ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
               ? Vec8<T>::load(src + (size_t)(b * a.s_P + iy * a.W + ix) * a.s_ctot + a.s_coff + c0)
               : Vec8<T>::zero();
  }
  f32x4 w[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    w[t][0] = *reinterpret_cast<const f32x4*>(a.w + t * a.C + c0);
    w[t][1] = *reinterpret_cast<const f32x4*>(a.w + t * a.C + c0 + 4);
  }
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.bias + c0), b1 = *reinterpret_cast<const f32x4*>(a.bias + c0 + 4);
  float acc[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf((float)v[t][e], w[t][e >> 2][e & 3], acc[e]);
  typename Vec8<T>::type o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {  // f16 plans: the fp16 rounding hides the fast SiLU's ~1 ulp (fp32)
    const float sv = sizeof(T) == 2 ? ym_silu_fast(acc[e]) : (std::is_same<T, P2>::value ? ym_silu_x3(acc[e]) : ym_silu(acc[e]));
    o[e] = (typename Vec8<T>::elem)(a.act ? sv : acc[e]);
  }
  Vec8<T>::store(static_cast<T*>(a.dst) + (size_t)(b * a.d_P + p) * a.d_ctot + a.d_coff + c0, o);
  if (a.raw) {  // f32 calibration run: the pre-activation output
#pragma unroll
    for (int e = 0; e < 8; ++e) a.raw[(size_t)pix * a.C + c0 + e] = acc[e];
  }
}

// Row variant: one thread = 8 channels of PXT consecutive pixels of one row (W % PXT == 0).  The 3 x (PXT + 2)
// activation window and the 9 x 8 weights are loaded once for PXT outputs: (3 (PXT + 2) + 20) vector loads per
// PXT pixels instead of 29 per pixel — the single-pixel kernel is bound by load-instruction issue, not bytes.
// Same fmaf order per output as dwconv3x3 (bias, then taps 0..8): bit-identical results.
template <typename T, int PXT>
__global__ __launch_bounds__(256) void dwconv3x3_row(const DwArgs a) {
  const int C8 = a.C >> 3;
  const int Wq = a.W / PXT;
  const int idx = ym_xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // contiguous run per XCD
  const int total = a.B * a.H * Wq * C8;
  if (idx >= total) return;
  const int q = idx / C8;
  const int cg = idx - q * C8;
  const int row = q / Wq;  // b * H + y
  const int x0 = (q - row * Wq) * PXT;
  const int b = row / a.H, y = row - b * a.H;
  const int c0 = cg * 8;
  const T* src = static_cast<const T*>(a.src) + (size_t)b * a.s_P * a.s_ctot + a.s_coff + c0;
  typename Vec8<T>::type v[3][PXT + 2];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int iy = y + r - 1;
#pragma unroll
    for (int cc = 0; cc < PXT + 2; ++cc) {
      const int ix = x0 + cc - 1;
      v[r][cc] = ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                     ? Vec8<T>::load(src + (size_t)(iy * a.W + ix) * a.s_ctot)
                     : Vec8<T>::zero();
    }
  }
  f32x4 w[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    w[t][0] = *reinterpret_cast<const f32x4*>(a.w + t * a.C + c0);
    w[t][1] = *reinterpret_cast<const f32x4*>(a.w + t * a.C + c0 + 4);
  }
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.bias + c0), b1 = *reinterpret_cast<const f32x4*>(a.bias + c0 + 4);
#pragma unroll
  for (int px = 0; px < PXT; ++px) {
    float acc[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf((float)v[t / 3][px + t % 3][e], w[t][e >> 2][e & 3], acc[e]);
    typename Vec8<T>::type o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sv = sizeof(T) == 2 ? ym_silu_fast(acc[e]) : (std::is_same<T, P2>::value ? ym_silu_x3(acc[e]) : ym_silu(acc[e]));
      o[e] = (typename Vec8<T>::elem)(a.act ? sv : acc[e]);
    }
    const int p = y * a.W + x0 + px;
    Vec8<T>::store(static_cast<T*>(a.dst) + (size_t)(b * a.d_P + p) * a.d_ctot + a.d_coff + c0, o);
    if (a.raw) {
#pragma unroll
      for (int e = 0; e < 8; ++e) a.raw[((size_t)b * a.H * a.W + p) * a.C + c0 + e] = acc[e];
    }
  }
}

// Column-strip variant: one thread = 8 channels of PXT consecutive pixels in RT consecutive rows.  The 3-row window
// rolls down the strip: each new output row loads one input row of PXT + 2 pixels, so (RT + 2)(PXT + 2) vector loads
// serve RT·PXT outputs (PXT 4, RT 4: 2.25 loads per output against 4.5 for the row variant).  Same fmaf order per
// output as dwconv3x3 (bias, then taps 0..8): bit-identical results.
template <typename T, int PXT, int RT>
__global__ __launch_bounds__(256) void dwconv3x3_strip(const DwArgs a) {
  const int C8 = a.C >> 3;
  const int Wq = a.W / PXT, Hq = (a.H + RT - 1) / RT;
  const int idx = ym_xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // contiguous run per XCD
  const int total = a.B * Hq * Wq * C8;
  if (idx >= total) return;
  const int q = idx / C8;
  const int cg = idx - q * C8;
  const int rb = q / Wq;  // b * Hq + row block
  const int x0 = (q - rb * Wq) * PXT;
  const int b = rb / Hq, y0 = (rb - b * Hq) * RT;
  const int c0 = cg * 8;
  const T* src = static_cast<const T*>(a.src) + (size_t)b * a.s_P * a.s_ctot + a.s_coff + c0;
  typedef typename Vec8<T>::type V;
  auto load_row = [&](V* r, int iy) {
#pragma unroll
    for (int cc = 0; cc < PXT + 2; ++cc) {
      const int ix = x0 + cc - 1;
      r[cc] = ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                  ? Vec8<T>::load(src + (size_t)(iy * a.W + ix) * a.s_ctot)
                  : Vec8<T>::zero();
    }
  };
  f32x4 w[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    w[t][0] = *reinterpret_cast<const f32x4*>(a.w + t * a.C + c0);
    w[t][1] = *reinterpret_cast<const f32x4*>(a.w + t * a.C + c0 + 4);
  }
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.bias + c0), b1 = *reinterpret_cast<const f32x4*>(a.bias + c0 + 4);
  V v[3][PXT + 2];  // v[(y - y0 + 1 + r) % 3] holds input row y + r - 1 while output row y is computed
  load_row(v[0], y0 - 1);
  load_row(v[1], y0);
#pragma unroll
  for (int j = 0; j < RT; ++j) {
    const int y = y0 + j;
    if (y >= a.H) break;
    load_row(v[(j + 2) % 3], y + 1);
#pragma unroll
    for (int px = 0; px < PXT; ++px) {
      float acc[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf((float)v[(j + t / 3) % 3][px + t % 3][e], w[t][e >> 2][e & 3], acc[e]);
      V o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sv = sizeof(T) == 2 ? ym_silu_fast(acc[e]) : (std::is_same<T, P2>::value ? ym_silu_x3(acc[e]) : ym_silu(acc[e]));
        o[e] = (typename Vec8<T>::elem)(a.act ? sv : acc[e]);
      }
      const int p = y * a.W + x0 + px;
      Vec8<T>::store(static_cast<T*>(a.dst) + (size_t)(b * a.d_P + p) * a.d_ctot + a.d_coff + c0, o);
      if (a.raw) {
#pragma unroll
        for (int e = 0; e < 8; ++e) a.raw[((size_t)b * a.H * a.W + p) * a.C + c0 + e] = acc[e];
      }
    }
  }
}

// LDS-tile variant: a workgroup owns TH x TW output pixels x CG 8-channel chunks of one image.  Phase 1: the
// (TH + 2) x (TW + 2) input window of those chunks (zeros outside the map) and the tile's weights / bias go into LDS,
// every global load of the workgroup issued before the barrier — one memory round trip per workgroup, each input
// chunk fetched ~(TH+2)(TW+2)/(TH·TW) times instead of the 9 (one-pixel) or 3(PXT+2)/PXT (row variant) per output.
// Phase 2: each thread computes its outputs from LDS in the fmaf order of dwconv3x3 (bias, then taps 0..8):
// bit-identical results.  LDS holds the values as the other variants compute with them (fp16, or fp32 = hi + lo).
template <typename T, int TH, int TW, int CG>
__global__ __launch_bounds__(256) void dwconv3x3_lds(const DwArgs a) {
  typedef typename std::conditional<sizeof(T) == 2, f16x8, f32x8>::type LV;  // one chunk as the kernel computes it
  constexpr int IH = TH + 2, IW = TW + 2;
  __shared__ LV xin[IH * IW * CG];
  __shared__ f32x8 wl[10 * CG];  // taps 0..8, then the bias
  const int C8 = a.C >> 3;
  const int ntx = (a.W + TW - 1) / TW, nty = (a.H + TH - 1) / TH, ncg = (C8 + CG - 1) / CG;
  int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // neighbouring tiles (shared halo rows) on one XCD
  const int cgi = vb % ncg; vb /= ncg;
  const int tx = vb % ntx; vb /= ntx;
  const int ty = vb % nty;
  const int b = vb / nty;
  const int x0 = tx * TW, y0 = ty * TH, c0 = cgi * CG;  // c0: first chunk
  const T* src = static_cast<const T*>(a.src) + (size_t)b * a.s_P * a.s_ctot + a.s_coff;
  constexpr int NIN = IH * IW * CG;
  constexpr int PER = (NIN + 255) / 256;
  LV v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int c = i % CG, q = i / CG;
    const int iy = y0 - 1 + q / IW, ix = x0 - 1 + q % IW;
    LV z;
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = 0;
    if (i < NIN && c0 + c < C8 && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) {
      const auto t = Vec8<T>::load(src + (size_t)(iy * a.W + ix) * a.s_ctot + 8 * (c0 + c));
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = t[e];
    }
    v[u] = z;
  }
  if (threadIdx.x < 10 * CG) {
    const int t = threadIdx.x / CG, c = threadIdx.x % CG;
    f32x8 w8;
#pragma unroll
    for (int e = 0; e < 8; ++e) w8[e] = 0.f;
    if (c0 + c < C8) {
      const float* p = t < 9 ? a.w + t * a.C + 8 * (c0 + c) : a.bias + 8 * (c0 + c);
      const f32x4 lo4 = *reinterpret_cast<const f32x4*>(p), hi4 = *reinterpret_cast<const f32x4*>(p + 4);
      w8 = f32x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
    }
    wl[threadIdx.x] = w8;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < NIN) xin[i] = v[u];
  }
  __syncthreads();
  constexpr int NOUT = TH * TW * CG;
  T* dst = static_cast<T*>(a.dst);
#pragma unroll
  for (int u = 0; u < (NOUT + 255) / 256; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int c = i % CG, q = i / CG;
    const int oy = q / TW, ox = q % TW;
    const int y = y0 + oy, x = x0 + ox;
    if (i >= NOUT || y >= a.H || x >= a.W || c0 + c >= C8) continue;
    const f32x8 bv = wl[9 * CG + c];
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = bv[e];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const LV xv = xin[((oy + t / 3) * IW + ox + t % 3) * CG + c];
      const f32x8 wv = wl[t * CG + c];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf((float)xv[e], wv[e], acc[e]);
    }
    typename Vec8<T>::type o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sv = sizeof(T) == 2 ? ym_silu_fast(acc[e]) : (std::is_same<T, P2>::value ? ym_silu_x3(acc[e]) : ym_silu(acc[e]));
      o[e] = (typename Vec8<T>::elem)(a.act ? sv : acc[e]);
    }
    Vec8<T>::store(dst + (size_t)(b * a.d_P + y * a.W + x) * a.d_ctot + a.d_coff + 8 * (c0 + c), o);
  }
}

// ------------------------------------------------------------------------------------------------- SPPF pools
// y1 = max5(y0), y2 = max5(y1) = max9(y0), y3 = max13(y0) (stride 1, -inf padding: the cascade is exactly the
// wider window).  Separable: row maxima of radius 2/4/6 in one pass over the 13-wide row window, then column
// maxima.  One workgroup = one image x 8 channels; pixels move as 16-byte vectors and stay in LDS in the storage
// type (max is exact in any precision).
template <typename V>
__device__ __forceinline__ V vmax(V x, V y) { return __builtin_elementwise_max(x, y); }  // v_pk_max_f16 for fp16

// fp8 e4m3 codes (sign-magnitude bytes) are max-pooled as order keys: key = sign ? -magnitude : magnitude, an int8
// whose order is the values' order (both zeros -> 0, stored back as +0: the same value)
template <typename V>
__device__ __forceinline__ V f8_key(V v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (v[e] & 0x80) ? (signed char)(-(v[e] & 0x7F)) : v[e];
  return v;
}
template <typename V>
__device__ __forceinline__ V f8_unkey(V v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = v[e] < 0 ? (signed char)(0x80 | -v[e]) : v[e];
  return v;
}

template <typename T, bool F8 = false>
__global__ __launch_bounds__(256) void sppf_pool(const PoolArgs a) {
  typedef typename Vec8<T>::type V;
  auto ld = [&](const T* p) { V v = Vec8<T>::load(p); if constexpr (F8) v = f8_key(v); return v; };
  auto st = [&](T* p, V v) { if constexpr (F8) v = f8_unkey(v); Vec8<T>::store(p, v); };
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  V* in = reinterpret_cast<V*>(smraw);  // [HW]
  const int HW = a.H * a.W;
  V* hr = in + HW;                      // [3][HW] row maxima, radius 2, 4, 6
  const int ng = a.C / 8;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // an image's channel groups share cache lines: one XCD
  const int b = vb / ng;
  const int c0 = (vb % ng) * 8;
  T* buf = static_cast<T*>(a.buf);
  {  // all loads in flight before the first LDS store (HW <= 1024 on the separable path's maps)
    V v[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int p = threadIdx.x + 256 * it;
      if (p < HW) v[it] = ld(buf + (size_t)(b * a.P + p) * a.ctot + a.coff + c0);
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int p = threadIdx.x + 256 * it;
      if (p < HW) in[p] = v[it];
    }
    for (int p = threadIdx.x + 1024; p < HW; p += 256)
      in[p] = ld(buf + (size_t)(b * a.P + p) * a.ctot + a.coff + c0);
  }
  __syncthreads();
  if (!a.sep) {  // LDS holds only the input image (large maps in f32): direct 2-D windows
    for (int it = threadIdx.x; it < 3 * HW; it += 256) {
      const int j = it / HW, p = it - (it / HW) * HW;
      const int r = 2 * (j + 1);
      const int y = p / a.W, x = p - (p / a.W) * a.W;
      V m = in[p];
      for (int yy = y - r < 0 ? 0 : y - r; yy <= y + r && yy < a.H; ++yy)
        for (int xx = x - r < 0 ? 0 : x - r; xx <= x + r && xx < a.W; ++xx) m = vmax(m, in[yy * a.W + xx]);
      st(buf + (size_t)(b * a.P + p) * a.ctot + a.coff + (j + 1) * a.C + c0, m);
    }
    return;
  }
  for (int p = threadIdx.x; p < HW; p += 256) {
    const int y = p / a.W, x = p - (p / a.W) * a.W;
    V m2 = in[p], m4 = m2, m6 = m2;
    for (int dx = -6; dx <= 6; ++dx) {
      const int xx = x + dx;
      if (dx == 0 || (unsigned)xx >= (unsigned)a.W) continue;
      const V v = in[y * a.W + xx];
      const int ad = dx < 0 ? -dx : dx;
      m6 = vmax(m6, v);
      if (ad <= 4) m4 = vmax(m4, v);
      if (ad <= 2) m2 = vmax(m2, v);
    }
    hr[p] = m2;
    hr[HW + p] = m4;
    hr[2 * HW + p] = m6;
  }
  __syncthreads();
  for (int it = threadIdx.x; it < 3 * HW; it += 256) {
    const int j = it / HW, p = it - (it / HW) * HW;
    const int r = 2 * (j + 1);
    const int y = p / a.W, x = p - (p / a.W) * a.W;
    const V* h = hr + (size_t)j * HW;
    V m = h[p];
    for (int dy = -r; dy <= r; ++dy) {
      const int yy = y + dy;
      if (dy == 0 || (unsigned)yy >= (unsigned)a.H) continue;
      m = vmax(m, h[yy * a.W + x]);
    }
    st(buf + (size_t)(b * a.P + p) * a.ctot + a.coff + (j + 1) * a.C + c0, m);
  }
}

// ------------------------------------------------------------------------------------------------- attention
// C2PSA Attention, one workgroup = (image, head, QB queries):
//   1. S = (Q·Kᵀ)·kd^-½ for all N keys into LDS (each thread holds one key row in registers, Q is broadcast);
//   2. row softmax in LDS (max-subtracted exp, divide by the sum — as torch.softmax);
//   3. O = P·V: thread = (head dim d, group of QB/4 queries), V rows read coalesced (128 B per key);
//   4. + pe(v): depthwise 3x3 + folded BN on v (the `+ self.pe(v.reshape(B,C,H,W))` term), store.
constexpr int AKD = 32, AHD = 64;

// one element of an activation tensor (x3 pair storage: hi + lo of its chunk)
template <typename T> __device__ __forceinline__ float ld1(const T* p) {
  if constexpr (std::is_same<T, P2>::value) return ym_p2_get(p);
  else return (float)*p;
}
template <typename T> __device__ __forceinline__ void st1(T* p, float v) {
  if constexpr (std::is_same<T, P2>::value) ym_p2_set(p, v);
  else *p = (T)v;
}

template <typename T, int QB>
__global__ __launch_bounds__(256) void attn_psa(const AttnArgs a) {
  extern __shared__ float S[];  // [QB][N], then Q [QB][AKD]
  const int N = a.N;
  float* Qs = S + (size_t)QB * N;
  const int nqb = (N + QB - 1) / QB;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // the query blocks of one (image, head) on one XCD
  const int qb = vb % nqb;
  const int bh = vb / nqb;
  const int h = bh % a.nh;
  const int b = bh / a.nh;
  const int tid = threadIdx.x;
  const int per = 2 * a.kd + a.hd;
  const T* qkv = static_cast<const T*>(a.qkv);
  const size_t img = (size_t)b * a.q_P;
  const int hq = a.q_coff + h * per;
  for (int i = tid; i < QB * AKD; i += 256) {
    const int r = i / AKD, c = i % AKD;
    const int n = qb * QB + r;
    Qs[i] = (n < N && c < a.kd) ? ld1(qkv + (img + n) * a.q_ctot + hq + c) : 0.f;
  }
  __syncthreads();
  // 1. scores
  for (int key = tid; key < N; key += 256) {
    float k[AKD];
    const T* kp = qkv + (img + key) * a.q_ctot + hq + a.kd;
#pragma unroll
    for (int c8 = 0; c8 < AKD / 8; ++c8) {
      const typename Vec8<T>::type v = Vec8<T>::load(kp + c8 * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) k[c8 * 8 + e] = (c8 * 8 + e < a.kd) ? (float)v[e] : 0.f;
    }
#pragma unroll 4
    for (int q = 0; q < QB; ++q) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < AKD; ++c) s = fmaf(Qs[q * AKD + c], k[c], s);
      S[q * N + key] = s * a.scale;
    }
  }
  __syncthreads();
  // 2. softmax: 256/QB threads per row
  {
    constexpr int TPR = 256 / QB;
    const int q = tid / TPR, sub = tid % TPR;
    float* row = S + (size_t)q * N;
    float m = -INFINITY;
    for (int j = sub; j < N; j += TPR) m = fmaxf(m, row[j]);
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float sum = 0.f;
    for (int j = sub; j < N; j += TPR) {
      const float e = expf(row[j] - m);
      row[j] = e;
      sum += e;
    }
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    for (int j = sub; j < N; j += TPR) row[j] = row[j] / sum;
  }
  __syncthreads();
  // 3. O = P·V
  constexpr int QPG = QB / 4;
  const int d = tid & 63, qg = tid >> 6;
  float o[QPG];
#pragma unroll
  for (int i = 0; i < QPG; ++i) o[i] = 0.f;
  const T* vp = qkv + img * a.q_ctot + hq + 2 * a.kd + d;
  float* Vs = Qs + QB * AKD;  // [64 keys][AHD] chunk of V, staged with 16-byte loads
  for (int k0 = 0; k0 < N; k0 += 64) {
    __syncthreads();
    {
      const int kk = tid >> 2, part = tid & 3;  // 64 keys x 4 quarters of 16 dims
      const int key = k0 + kk;
#pragma unroll
      for (int h8 = 0; h8 < 2; ++h8) {
        const int d0 = part * 16 + h8 * 8;
        typename Vec8<T>::type v = Vec8<T>::zero();
        if (key < N && d0 < a.hd) v = Vec8<T>::load(qkv + (img + key) * a.q_ctot + hq + 2 * a.kd + d0);
#pragma unroll
        for (int e = 0; e < 8; ++e) Vs[kk * AHD + d0 + e] = (float)v[e];
      }
    }
    __syncthreads();
    const int kn = N - k0 < 64 ? N - k0 : 64;
    for (int kj = 0; kj < kn; ++kj) {
      const float v = Vs[kj * AHD + d];
#pragma unroll
      for (int i = 0; i < QPG; ++i) o[i] = fmaf(S[(qg + 4 * i) * N + k0 + kj], v, o[i]);
    }
  }
  // 4. + pe(v), store
  if (d >= a.hd) return;
  const int ch = h * a.hd + d;
  T* dst = static_cast<T*>(a.dst);
#pragma unroll
  for (int i = 0; i < QPG; ++i) {
    const int n = qb * QB + qg + 4 * i;
    if (n >= N) continue;
    const int y = n / a.W, x = n - (n / a.W) * a.W;
    float pe = a.pe_b[ch];
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = y + ky - 1;
      if ((unsigned)iy >= (unsigned)a.H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = x + kx - 1;
        if ((unsigned)ix >= (unsigned)a.W) continue;
        pe = fmaf(ld1(vp + (size_t)(iy * a.W + ix) * a.q_ctot), a.pe_w[(ky * 3 + kx) * a.C + ch], pe);
      }
    }
    st1(dst + ((size_t)b * a.d_P + n) * a.d_ctot + a.d_coff + ch, o[i] + pe);
    if (a.raw) a.raw[((size_t)b * N + n) * a.C + ch] = pe;  // f32 calibration run: pe(v) before the add
  }
}

// f16 plans, kd = 32 / hd = 64 (every YOLO11 scale) and N <= 512 tokens (inputs up to 724 px): the same Attention on
// MFMA.  One workgroup = (image, head, 64 queries), one wave = 16 queries:
//   1. K [N][32] and V^T [64][N] of the whole (image, head) are staged in LDS with every load in flight at once
//      (K rows padded to 80 bytes, V^T rows to 16 NKT + 4 halves: the fragment reads below spread over the banks);
//   2. S^T = K·Q^T: one v_mfma_f32_16x16x32_f16 per 16 keys (K = kd = 32), A = K rows from LDS, B = the wave's 16
//      query rows (one 16-byte load); the lane holds S^T[key 16t + 4(l>>4) + r][query l&15], all N keys in registers;
//   3. softmax over keys: in-lane over the tiles, then across the 4 lane groups (fp32, max-subtracted, v_exp_f32
//      on log2-scaled scores);
//   4. O^T = V^T·P^T, K = 32 keys per MFMA in the lane-group order of step 2 (slot j of group g is key
//      32s + 4g + j, or 32s + 16 + 4g + j - 4), so P comes straight from the softmax registers (rounded to fp16)
//      and V^T as two 8-byte LDS reads; a lane ends with 4 consecutive channels of one query: 8-byte NHWC stores;
//   5. + pe(v) (depthwise 3x3 + folded BN) from the staged V^T and LDS taps, store.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));

template <int NKT>  // key tiles of 16 (even): N <= 16 NKT
__global__ __launch_bounds__(256) void attn_psa_mfma(const AttnArgs a) {
  // LDS: V^T [64][LDV] f16, K [16 NKT][LDK] f16, pe weights [9][64] + bias [64] f32
  extern __shared__ __attribute__((aligned(16))) f16 vt[];
  constexpr int LDV = 16 * NKT + 4;
  // 96-byte K rows (6 16-byte slots): the 16-row x 4-chunk fragment reads hit distinct slots in each of ds_read_b128's
  // non-contiguous lane groups (MI355X_MICROARCH §LDS); 80-byte rows were 2-way there
  constexpr int LDK = 48;
  f16* kl = vt + 64 * LDV;
  float* pw = reinterpret_cast<float*>(kl + 16 * NKT * LDK);
  const int N = a.N;
  const int nqb = (N + 63) / 64;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);  // the query blocks of one (image, head) on one XCD
  const int qb = vb % nqb, bh = vb / nqb;
  const int h = bh % a.nh, b = bh / a.nh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const f16* qkv = static_cast<const f16*>(a.qkv);
  const size_t img = (size_t)b * a.q_P;
  const int hq = a.q_coff + h * 128;  // per head: q 32, k 32, v 64 channels
  // 1. K and V^T of the (image, head) into LDS (keys >= N zero), this head's positional-conv taps and bias
  for (int i = tid; i < 640; i += 256)
    pw[i] = i < 576 ? a.pe_w[(i >> 6) * a.C + h * 64 + (i & 63)] : a.pe_b[h * 64 + i - 576];
  {  // all loads in flight before the first LDS store (one memory latency, not NIT): 12 chunks of 8 per key
    constexpr int NIT = (16 * NKT * 12 + 255) / 256;
    f16x8 v[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + 256 * it, key = i / 12, ch = i - key * 12;
      v[it] = key < N ? Vec8<f16>::load(qkv + (img + key) * a.q_ctot + hq + 32 + 8 * ch) : Vec8<f16>::zero();
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + 256 * it, key = i / 12, ch = i - key * 12;
      if (key >= 16 * NKT) break;
      if (ch < 4) {
        *reinterpret_cast<f16x8*>(kl + key * LDK + 8 * ch) = v[it];
      } else {
        const int d0 = 8 * (ch - 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) vt[(d0 + e) * LDV + key] = v[it][e];
      }
    }
  }
  const int q = qb * 64 + wave * 16 + c;
  h8v qf = Vec8<f16>::zero();
  if (q < N) qf = Vec8<f16>::load(qkv + (img + q) * a.q_ctot + hq + 8 * g);
  __syncthreads();
  // 2. scores, in log2 units (scale·log2 e folded in: softmax by exp2)
  const float sl2 = a.scale * 1.4426950408889634f;
  float s[NKT][4];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const h8v kf = *reinterpret_cast<const h8v*>(kl + (16 * t + c) * LDK + 8 * g);
    const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) s[t][r] = 16 * t + 4 * g + r < N ? d[r] * sl2 : -INFINITY;
  }
  // 3. softmax over the keys of query l&15
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, s[t][r]);
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[t][r] = __builtin_amdgcn_exp2f(s[t][r] - m);  // v_exp_f32 (~1 ulp; P is rounded to fp16 below)
      sum += s[t][r];
    }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float rs = 1.0f / sum;
  // 4. O^T = V^T P^T
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKT / 2; ++ks) {
    h8v pf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pf[r] = (f16)(s[2 * ks][r] * rs);
      pf[4 + r] = (f16)(s[2 * ks + 1][r] * rs);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f16* vr = vt + (16 * dt + c) * LDV + 32 * ks + 4 * g;
      const f16x4 lo = *reinterpret_cast<const f16x4*>(vr), hi = *reinterpret_cast<const f16x4*>(vr + 16);
      const h8v vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf, o[dt], 0, 0, 0);
    }
  }
  // 5. + pe(v), store: lane = channels 16dt + 4g .. +3 of query q
  if (q >= N) return;
  const int y = q / a.W, x = q - (q / a.W) * a.W;
  f16* dst = static_cast<f16*>(a.dst) + ((size_t)b * a.d_P + q) * a.d_ctot + a.d_coff + h * 64;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int d0 = 16 * dt + 4 * g;
    float pe[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pe[r] = pw[576 + d0 + r];
#pragma unroll
    for (int t = 0; t < 9; ++t) {  // taps in (ky, kx) order; out-of-image taps skipped, as the zero-padded conv
      const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
      if ((unsigned)iy >= (unsigned)a.H || (unsigned)ix >= (unsigned)a.W) continue;
      const int nb = iy * a.W + ix;
      const f32x4 w = *reinterpret_cast<const f32x4*>(pw + 64 * t + d0);
#pragma unroll
      for (int r = 0; r < 4; ++r) pe[r] = fmaf((float)vt[(d0 + r) * LDV + nb], w[r], pe[r]);
    }
    f16x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = (f16)(o[dt][r] + pe[r]);
    *reinterpret_cast<f16x4*>(dst + d0) = out;
  }
}

// x3 plans, kd = 32 / hd = 64, N <= 512 tokens: attn_psa_mfma's structure on the pair layout, every product split
// (hi·hi + lo·hi + hi·lo on v_mfma_f32_16x16x32_f16, fp32 accumulation).  V^T of the (image, head) is staged in LDS
// as hi and lo planes (the two planes of K as well would not fit beside them), K fragments stream from global
// (32 bytes = the [hi | lo] pair of one key chunk per lane and key tile; L2-resident), P is split in registers.
template <int NKT, int KB>
__global__ __launch_bounds__(256) void attn_psa_x3(const AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) f16 vt[];  // [2][64][LDV]: V^T hi, lo; then pe weights + bias f32
  constexpr int LDV = 16 * NKT + 4;
  f16* vtl = vt + 64 * LDV;
  float* pw = reinterpret_cast<float*>(vtl + 64 * LDV);
  const int N = a.N;
  const int nqb = (N + 63) / 64;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);
  const int qb = vb % nqb, bh = vb / nqb;
  const int h = bh % a.nh, b = bh / a.nh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const P2* qkv = static_cast<const P2*>(a.qkv);
  const size_t img = (size_t)b * a.q_P;
  const int hq = a.q_coff + h * 128;  // per head: q 32, k 32, v 64 logical channels
  for (int i = tid; i < 640; i += 256)
    pw[i] = i < 576 ? a.pe_w[(i >> 6) * a.C + h * 64 + (i & 63)] : a.pe_b[h * 64 + i - 576];
  // 1. V^T hi / lo planes (keys >= N zero): 8 chunks of 8 v channels per key.  Every chunk load is in flight
  // before the first LDS store (one memory latency, not NIT of them: the loop form waited for each load in turn)
  {
    constexpr int NIT = 16 * NKT * 8 / 256;
    static_assert(16 * NKT * 8 % 256 == 0, "V chunks divide over the threads");
    HL v[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + 256 * it, key = i >> 3, ch = i & 7;
      // (an unconditional load of a clamped key, zeroed below: a load under a condition is waited for on the spot)
      v[it] = ym_load_hl(qkv + (img + (key < N ? key : N - 1)) * a.q_ctot + hq + 64 + 8 * ch);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + 256 * it, key = i >> 3, ch = i & 7;
      const bool ok = key < N;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        vt[(8 * ch + e) * LDV + key] = ok ? v[it].hi[e] : (f16)0;
        vtl[(8 * ch + e) * LDV + key] = ok ? v[it].lo[e] : (f16)0;
      }
    }
  }
  const int q = qb * 64 + wave * 16 + c;
  // (queries past N: a clamped row; their outputs are never stored)
  const HL qf = ym_load_hl(qkv + (img + (q < N ? q : N - 1)) * a.q_ctot + hq + 8 * g);
  // 2. scores S^T = K·Q^T (log2 units): lane (g, c) supplies key 16t + c, logical chunk g of K.  The K fragments
  // of KB key tiles are loaded together (unconditional loads of clamped keys: rows past N only feed scores that are
  // masked to -inf), then their MFMAs run: NKT / KB memory round trips instead of one per tile (KB = NKT: one; the
  // kernel runs one wave per SIMD, so the registers are there)
  const float sl2 = a.scale * 1.4426950408889634f;
  float s[NKT][4];
#pragma unroll
  for (int t0 = 0; t0 < NKT; t0 += KB) {
    HL kf[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int key = 16 * (t0 + u) + c;
      if (t0 + u < NKT) kf[u] = ym_load_hl(qkv + (img + (key < N ? key : N - 1)) * a.q_ctot + hq + 32 + 8 * g);
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int t = t0 + u;
      if (t >= NKT) break;
      f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[u].lo, qf.hi, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[u].hi, qf.lo, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[u].hi, qf.hi, d, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) s[t][r] = 16 * t + 4 * g + r < N ? d[r] * sl2 : -INFINITY;
    }
  }
  __syncthreads();
  // 3. softmax over the keys of query l&15 (fp32, exact exp2)
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, s[t][r]);
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[t][r] = exp2f(s[t][r] - m);
      sum += s[t][r];
    }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float rs = 1.0f / sum;
  // 4. O^T = V^T P^T, K = 32 keys per MFMA in the lane-group order of step 2 (as attn_psa_mfma), P split hi / lo
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKT / 2; ++ks) {
    h8v ph, pl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p0 = s[2 * ks][r] * rs, p1 = s[2 * ks + 1][r] * rs;
      ph[r] = (f16)p0;
      pl[r] = (f16)(p0 - (float)ph[r]);
      ph[4 + r] = (f16)p1;
      pl[4 + r] = (f16)(p1 - (float)ph[4 + r]);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int row = (16 * dt + c) * LDV + 32 * ks + 4 * g;
      const f16x4 hlo = *reinterpret_cast<const f16x4*>(vt + row), hhi = *reinterpret_cast<const f16x4*>(vt + row + 16);
      const f16x4 llo = *reinterpret_cast<const f16x4*>(vtl + row), lhi = *reinterpret_cast<const f16x4*>(vtl + row + 16);
      const h8v vh = {hlo[0], hlo[1], hlo[2], hlo[3], hhi[0], hhi[1], hhi[2], hhi[3]};
      const h8v vl = {llo[0], llo[1], llo[2], llo[3], lhi[0], lhi[1], lhi[2], lhi[3]};
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph, o[dt], 0, 0, 0);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pl, o[dt], 0, 0, 0);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph, o[dt], 0, 0, 0);
    }
  }
  // 5. + pe(v) (v = hi + lo from LDS), store in the pair layout: lane = channels 16dt + 4g .. +3 of query q
  if (q >= N) return;
  const int y = q / a.W, x = q - (q / a.W) * a.W;
  P2* dst = static_cast<P2*>(a.dst) + ((size_t)b * a.d_P + q) * a.d_ctot + a.d_coff + h * 64;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int d0 = 16 * dt + 4 * g;
    float pe[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pe[r] = pw[576 + d0 + r];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
      if ((unsigned)iy >= (unsigned)a.H || (unsigned)ix >= (unsigned)a.W) continue;
      const int nb = iy * a.W + ix;
      const f32x4 w = *reinterpret_cast<const f32x4*>(pw + 64 * t + d0);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pe[r] = fmaf((float)vt[(d0 + r) * LDV + nb] + (float)vtl[(d0 + r) * LDV + nb], w[r], pe[r]);
    }
    float out[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = o[dt][r] + pe[r];
    ym_p2_store4(dst + d0, out);
  }
}

// Any N (the 1280² input: 1600 tokens, core/validator.py:188): the MFMA attention with the keys in blocks of 256
// and an online softmax (running max / sum per query, O rescaled when the max grows), so neither the scores nor
// V^T of the whole (image, head) need to fit: per block, V^T (f16, or hi / lo planes for x3) is staged in LDS, K
// fragments stream from global; pe(v) reads its 3x3 taps from global.  X3: every product split as in attn_psa_x3.
template <bool X3>
__global__ __launch_bounds__(256) void attn_psa_flash(const AttnArgs a) {
  constexpr int KB = 256, NKT = KB / 16, LDV = KB + 4;
  typedef typename std::conditional<X3, P2, f16>::type T;
  extern __shared__ __attribute__((aligned(16))) f16 vt[];  // [X3 ? 2 : 1][64][LDV]
  f16* vtl = vt + 64 * LDV;
  const int N = a.N;
  const int nqb = (N + 63) / 64;
  const int vb = ym_xcd_block(blockIdx.x, gridDim.x);
  const int qb = vb % nqb, bh = vb / nqb;
  const int h = bh % a.nh, b = bh / a.nh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const T* qkv = static_cast<const T*>(a.qkv);
  const size_t img = (size_t)b * a.q_P;
  const int hq = a.q_coff + h * 128;  // per head: q 32, k 32, v 64 channels
  auto frag = [&](const T* p) -> HL {  // 8 channels of one token (hi and, for x3, lo)
    if constexpr (X3) return ym_load_hl(p);
    else return HL{Vec8<f16>::load(p), Vec8<f16>::zero()};
  };
  const int q = qb * 64 + wave * 16 + c;
  HL qf{Vec8<f16>::zero(), Vec8<f16>::zero()};
  if (q < N) qf = frag(qkv + (img + q) * a.q_ctot + hq + 8 * g);
  const float sl2 = a.scale * 1.4426950408889634f;
  float m = -INFINITY, l = 0.f;  // running max (log2 units) and this lane's partial sum of its query's weights
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < N; k0 += KB) {
    __syncthreads();  // every wave is done with the previous block's V^T
    for (int i = tid; i < KB * 8; i += 256) {
      const int key = i >> 3, ch = i & 7;
      HL v{Vec8<f16>::zero(), Vec8<f16>::zero()};
      if (k0 + key < N) v = frag(qkv + (img + k0 + key) * a.q_ctot + hq + 64 + 8 * ch);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        vt[(8 * ch + e) * LDV + key] = v.hi[e];
        if constexpr (X3) vtl[(8 * ch + e) * LDV + key] = v.lo[e];
      }
    }
    float s[NKT][4];
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      const int key = k0 + 16 * t + c;
      HL kf{Vec8<f16>::zero(), Vec8<f16>::zero()};
      if (key < N) kf = frag(qkv + (img + key) * a.q_ctot + hq + 32 + 8 * g);
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (X3) {
        d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf.lo, qf.hi, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf.hi, qf.lo, d, 0, 0, 0);
      }
      d = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf.hi, qf.hi, d, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) s[t][r] = k0 + 16 * t + 4 * g + r < N ? d[r] * sl2 : -INFINITY;
    }
    float mb = -INFINITY;
#pragma unroll
    for (int t = 0; t < NKT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mb = fmaxf(mb, s[t][r]);
    mb = fmaxf(mb, __shfl_xor(mb, 16));
    mb = fmaxf(mb, __shfl_xor(mb, 32));
    const float mn = fmaxf(m, mb);
    const float sc = exp2f(m - mn);  // 0 on the first block (m = -inf)
    m = mn;
    l *= sc;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= sc;
#pragma unroll
    for (int t = 0; t < NKT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[t][r] = exp2f(s[t][r] - mn);
        l += s[t][r];
      }
    __syncthreads();  // this block's V^T is staged
#pragma unroll
    for (int ks = 0; ks < NKT / 2; ++ks) {
      h8v ph, pl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ph[r] = (f16)s[2 * ks][r];
        ph[4 + r] = (f16)s[2 * ks + 1][r];
        if constexpr (X3) {
          pl[r] = (f16)(s[2 * ks][r] - (float)ph[r]);
          pl[4 + r] = (f16)(s[2 * ks + 1][r] - (float)ph[4 + r]);
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int row = (16 * dt + c) * LDV + 32 * ks + 4 * g;
        const f16x4 hlo = *reinterpret_cast<const f16x4*>(vt + row), hhi = *reinterpret_cast<const f16x4*>(vt + row + 16);
        const h8v vh = {hlo[0], hlo[1], hlo[2], hlo[3], hhi[0], hhi[1], hhi[2], hhi[3]};
        if constexpr (X3) {
          const f16x4 llo = *reinterpret_cast<const f16x4*>(vtl + row), lhi = *reinterpret_cast<const f16x4*>(vtl + row + 16);
          const h8v vl = {llo[0], llo[1], llo[2], llo[3], lhi[0], lhi[1], lhi[2], lhi[3]};
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph, o[dt], 0, 0, 0);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pl, o[dt], 0, 0, 0);
        }
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph, o[dt], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  const float rs = 1.0f / l;
  if (q >= N) return;
  const int y = q / a.W, x = q - (q / a.W) * a.W;
  T* dst = static_cast<T*>(a.dst) + ((size_t)b * a.d_P + q) * a.d_ctot + a.d_coff + h * 64;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int d0 = 16 * dt + 4 * g;
    float pe[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pe[r] = a.pe_b[h * 64 + d0 + r];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
      if ((unsigned)iy >= (unsigned)a.H || (unsigned)ix >= (unsigned)a.W) continue;
      const T* vp = qkv + (img + iy * a.W + ix) * a.q_ctot + hq + 64 + d0;
      float v[4];
      if constexpr (X3) {
        ym_p2_load4(vp, v);
      } else {
        const f16x4 hv = *reinterpret_cast<const f16x4*>(vp);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (float)hv[r];
      }
      const f32x4 w = *reinterpret_cast<const f32x4*>(a.pe_w + t * a.C + h * 64 + d0);
#pragma unroll
      for (int r = 0; r < 4; ++r) pe[r] = fmaf(v[r], w[r], pe[r]);
    }
    float out[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = o[dt][r] * rs + pe[r];
    if constexpr (X3) {
      ym_p2_store4(dst + d0, out);
    } else {
      *reinterpret_cast<f16x4*>(dst + d0) = f16x4{(f16)out[0], (f16)out[1], (f16)out[2], (f16)out[3]};
    }
  }
}

// ------------------------------------------------------------------------------------------------- decode
// Detect._inference + the candidate stage of non_max_suppression; 4 lanes per anchor (lane s: DFL side s and a
// quarter of the classes):
//   DFL softmax over reg_max bins → ltrb distances → dist2bbox(xywh) · stride → xywh2xyxy;
//   sigmoid class scores → (max, first argmax); candidate iff max > conf (and class in the filter).
// Candidates are appended to a per-image key list: key = score bits << 32 | ~anchor, so a descending sort gives
// score-descending order with ties broken by ascending anchor index (torchvision's stable sort).
// DIRECT (reg_max 16, nc 80: the YOLO11 heads): no LDS staging — lane s of an anchor loads its 16 DFL bins and its
// 20 class logits straight into registers (4 + 5 float4; the 4 lanes of an anchor cover its 576-byte row, so a wave's
// loads are 9.2 KB contiguous), no barrier before the math, and a small LDS footprint (more workgroups in flight).
// Same per-element arithmetic in the same order as the staged variant.
template <bool DIRECT>
__global__ __launch_bounds__(256) void decode_anchors(const DecodeArgs a) {
  float dist, best;
  int bi, b, ai, sub;
  long idx;
  bool valid;
  const long total = (long)a.B * a.A;
  const long a0 = blockIdx.x * 64L;
  if constexpr (DIRECT) {
    const long gidx = a0 + (threadIdx.x >> 2);
    sub = threadIdx.x & 3;
    valid = gidx < total;
    idx = valid ? gidx : 0;
    b = idx / a.A;
    ai = idx - (long)b * a.A;
    const f32x4* row = reinterpret_cast<const f32x4*>(a.anchors + idx * a.no_tot);
    f32x4 bv[4], cv[5];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = row[4 * sub + i];
#pragma unroll
    for (int i = 0; i < 5; ++i) cv[i] = row[16 + 5 * sub + i];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) mx = fmaxf(mx, bv[i >> 2][i & 3]);
    float den = 0.f, num = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float e = expf(bv[i >> 2][i & 3] - mx);
      den += e;
      num = fmaf(e, (float)i, num);
    }
    dist = num / den;
    float lmax = -INFINITY;
#pragma unroll
    for (int c = 0; c < 20; ++c) lmax = fmaxf(lmax, cv[c >> 2][c & 3]);
    const float lthr = lmax < 10.0f ? lmax - 0.5f : -INFINITY;
    best = -INFINITY;
    bi = 0x7FFFFFFF;
#pragma unroll
    for (int c = 0; c < 20; ++c) {
      const float l = cv[c >> 2][c & 3];
      if (!(l >= lthr)) continue;
      const float sc = ym_sigmoid(l);
      if (sc > best) { best = sc; bi = 20 * sub + c; }
    }
  } else {
    // the workgroup's 64 anchor rows are contiguous: stage them in LDS with coalesced 16-byte loads
    extern __shared__ float rows[];  // [64][no_tot + 1]
    const int nrow = total - a0 < 64 ? (int)(total - a0) : 64;
    // LDS rows are padded to an odd pitch (no_tot + 1 floats): the 16 anchors x 4 sides of a wave read 16-float
    // strided bins, which on a 144-float pitch fell into two banks (32-way conflicts)
    const int ldr = a.no_tot + 1;
    {  // every load in flight before the first LDS store (no_tot <= 192: at most 12 per thread)
      const f32x4* src = reinterpret_cast<const f32x4*>(a.anchors + a0 * a.no_tot);
      const int n4 = nrow * a.no_tot / 4, r4 = a.no_tot / 4;
      f32x4 v[12];
#pragma unroll
      for (int it = 0; it < 12; ++it) {
        const int i = threadIdx.x + 256 * it;
        if (i < n4) v[it] = src[i];
      }
#pragma unroll
      for (int it = 0; it < 12; ++it) {
        const int i = threadIdx.x + 256 * it;
        if (i < n4) {
          const int rr = i / r4, cc = 4 * (i - rr * r4);
          float* d = rows + rr * ldr + cc;
          d[0] = v[it][0]; d[1] = v[it][1]; d[2] = v[it][2]; d[3] = v[it][3];
        }
      }
    }
    __syncthreads();
    const long gidx = a0 + (threadIdx.x >> 2);
    sub = threadIdx.x & 3;
    valid = gidx < total;
    idx = valid ? gidx : 0;
    b = idx / a.A;
    ai = idx - (long)b * a.A;
    const float* row = rows + (valid ? (threadIdx.x >> 2) : 0) * ldr;
    {  // DFL: softmax over the bins, expectation of the bin index (one exp per bin, one division)
      const float* r = row + sub * a.reg_max;
      float mx = -INFINITY;
      for (int i = 0; i < a.reg_max; ++i) mx = fmaxf(mx, r[i]);
      float den = 0.f, num = 0.f;
      for (int i = 0; i < a.reg_max; ++i) {
        const float e = expf(r[i] - mx);
        den += e;
        num = fmaf(e, (float)i, num);
      }
      dist = num / den;
    }
    // class score = max sigmoid, first index on ties (torch max).  Sigmoid is monotonic, so only logits near the
    // quarter's max can reach its value: those within 0.5 of it while it is < 10 (there sigmoid' > 4e-5, so a logit
    // 0.5 lower is many ulps lower), every logit otherwise (saturation).
    const int q = (a.nc + 3) / 4;
    const float* cl = row + 4 * a.reg_max;
    const int c0 = sub * q, c1 = (sub + 1) * q < a.nc ? (sub + 1) * q : a.nc;
    float lmax = -INFINITY;
    for (int c = c0; c < c1; ++c) lmax = fmaxf(lmax, cl[c]);
    const float lthr = lmax < 10.0f ? lmax - 0.5f : -INFINITY;
    best = -INFINITY;
    bi = 0x7FFFFFFF;
    for (int c = c0; c < c1; ++c) {
      if (!(cl[c] >= lthr)) continue;
      const float sc = ym_sigmoid(cl[c]);
      if (sc > best) { best = sc; bi = c; }
    }
  }
#pragma unroll
  for (int o = 1; o < 4; o <<= 1) {
    const float ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const int base = threadIdx.x & 60;
  const float d0 = __shfl(dist, base), d1 = __shfl(dist, base + 1), d2 = __shfl(dist, base + 2),
              d3 = __shfl(dist, base + 3);
  // candidates are appended per workgroup: LDS slots first, then ONE global atomic per (workgroup, image) — the 64
  // anchors of a workgroup span at most 5 images (A >= 21).  (Per-candidate atomics on the B per-image counters serialised:
  // thousands of same-address atomics at ~90 per µs.)
  __shared__ int wg_cnt[8], wg_base[8];
  if (threadIdx.x < 8) wg_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int b_first = (int)(a0 / a.A);
  bool cand = false;
  int slot = 0;
  unsigned long long key = 0;
  if (sub == 0 && valid) {
    int l = 0;
    while (l + 1 < a.nl && ai >= a.lvl_off[l + 1]) ++l;
    const int p = ai - a.lvl_off[l];
    const float ax = (float)(p % a.lvl_W[l]) + 0.5f;
    const float ay = (float)(p / a.lvl_W[l]) + 0.5f;
    const float st = a.lvl_stride[l];
    const float x1 = ax - d0, y1 = ay - d1;
    const float x2 = ax + d2, y2 = ay + d3;
    const float cx = (x1 + x2) / 2.0f * st, cy = (y1 + y2) / 2.0f * st;
    const float w = (x2 - x1) * st, hh = (y2 - y1) * st;
    const float hw = w / 2.0f, hh2 = hh / 2.0f;
    a.boxes[idx] = make_float4(cx - hw, cy - hh2, cx + hw, cy + hh2);
    a.scores[idx] = best;
    a.cls[idx] = bi;
    cand = best > a.conf;
    if (cand && a.has_classes) cand = (a.classes[bi >> 5] >> (bi & 31)) & 1u;
    if (cand) {
      slot = atomicAdd(&wg_cnt[b - b_first], 1);
      key = ((unsigned long long)__float_as_uint(best) << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)ai);
  }
  }
  __syncthreads();
  if (threadIdx.x < 8 && wg_cnt[threadIdx.x] > 0)
    wg_base[threadIdx.x] = atomicAdd(&a.counts[b_first + threadIdx.x], wg_cnt[threadIdx.x]);
  __syncthreads();
  if (cand) a.keys[(size_t)b * a.kstride + wg_base[b - b_first] + slot] = key;
}

// ------------------------------------------------------------------------------------------------- NMS
// Per image, one 1024-thread workgroup: bitonic sort of the candidate keys, then greedy suppression exactly as
// torchvision's CPU nms: boxes offset by cls·max_wh (0 if agnostic), areas and IoU in fp32 on the offset boxes,
// suppress iff IoU > iou (compared in double), keep <= max_det, clip to the image.  Up to NMS_LDS candidates
// everything (keys, boxes, areas, flags) lives in LDS, so the serial scan costs LDS latency per candidate;
// larger candidate sets fall back to the same algorithm on global scratch.
constexpr int NMS_T = 1024;
constexpr int NMS_LDS = 4096;
constexpr int NMS_BM = 512;  // bit-matrix path: 512 x 8 words of 64 bits (32 KB) behind the first 512 boxes
// blocked path (NMS_BM < n, up to NMS_BLK_MAX candidates after max_nms, e.g. the validator's conf 0.001 at 640²: up to
// A = 8,400): the keys sorted in LDS, then the greedy scan in blocks of NMS_BLK candidates in score order — a block's
// candidates are first tested against every box kept by earlier blocks (the kept list in LDS), the survivors'
// intra-block IoU bit matrix is built by all waves, and one wave scans it in order (as the bit-matrix path).
// Candidate j is kept iff no kept i < j has IoU > iou: torchvision's greedy result, with a few barriers per block
// instead of one per kept box.  Class filter (not agnostic, iou >= 0, max_wh above the boxes' coordinate range, nc <=
// NMS_NC): boxes of different classes are offset cls * max_wh apart and cannot intersect (IoU 0, never > iou), so a
// candidate is tested only against kept boxes of its class (per-class lists) and a bit-matrix word only where the
// word holds a box of row i's class (per-word class masks).
constexpr int NMS_SORT = 16384;  // keys sorted in LDS (128 KB: the whole LDS arena)
constexpr int NMS_BLK = 256;     // candidates per block (bit matrix 256 x 4 words)
constexpr int NMS_KEEP = 512;    // kept boxes held in LDS: max_det up to this on the blocked path
constexpr int NMS_NC = 128;      // classes of the class filter
constexpr int NMS_W = NMS_BLK / 64;
// the block / kept-list regions (u64 units) sit at the end of the arena, behind the sorted keys they leave in place
constexpr int NR_BB = 0, NR_BA = NR_BB + 2 * NMS_BLK, NR_BAI = NR_BA + NMS_BLK / 2, NR_BSUP = NR_BAI + NMS_BLK / 2,
              NR_BCLS = NR_BSUP + NMS_BLK / 2, NR_BMASK = NR_BCLS + NMS_BLK / 2, NR_CCM = NR_BMASK + NMS_BLK * NMS_W,
              NR_KB = NR_CCM + NMS_W * NMS_NC, NR_KA = NR_KB + 2 * NMS_KEEP, NR_KNEXT = NR_KA + NMS_KEEP / 2,
              NR_KHEAD = NR_KNEXT + NMS_KEEP / 2, NMS_REG = NR_KHEAD + NMS_NC / 2;
constexpr int NMS_BLK_MAX = NMS_SORT - NMS_REG;  // candidates (after max_nms) the blocked path takes: 12,224

// A step whose stride is <= 64 only pairs elements inside the 128-element run a wave's 64 consecutive i cover (i =
// tid + NMS_T m), so consecutive such steps need no workgroup barrier: the wave's own LDS operations are in order.
// A barrier is taken after a step whose stride, or the next step's, is above 64 (LDS layout-independent; n2 a power
// of two >= 2).
__device__ __forceinline__ void bitonic_sort_desc(unsigned long long* k, int n2, int tid) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (n2 >> 1); i += NMS_T) {
        const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));  // (i / stride) * 2 stride + i % stride
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const unsigned long long x = k[lo], y = k[hi];
        if ((x < y) == desc) { k[lo] = y; k[hi] = x; }
      }
      const int next = stride > 1 ? stride >> 1 : (size < n2 ? size : 0);  // the next step's stride (0: done)
      if (stride > 64 || next > 64 || next == 0) {
        __syncthreads();
      } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
}

// one output row [x1 y1 x2 y2 conf cls coef_0 .. coef_nm-1]: box clipped to the image; a Segment head's nm mask
// coefficients are fetched as float4s all issued before the first store (a scalar load-store loop waited one memory
// latency per coefficient)
__device__ __forceinline__ void write_det(const NmsArgs& a, float* r, size_t anc) {
  const float4 v = a.boxes[anc];
  const float sc = a.scores[anc];
  const int cl = a.cls[anc];
  if (a.nm > 0 && a.nm <= 64 && (a.nm & 3) == 0 && ((a.no_tot | a.mask_off) & 3) == 0) {
    const float4* src = reinterpret_cast<const float4*>(a.anchors + anc * a.no_tot + a.mask_off);
    float4 c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (4 * i < a.nm) c[i] = src[i];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (4 * i < a.nm) {
        r[6 + 4 * i] = c[i].x;
        r[7 + 4 * i] = c[i].y;
        r[8 + 4 * i] = c[i].z;
        r[9 + 4 * i] = c[i].w;
      }
  } else {
    for (int m = 0; m < a.nm; ++m) r[6 + m] = a.anchors[anc * a.no_tot + a.mask_off + m];
  }
  r[0] = fminf(fmaxf(v.x, 0.f), a.img_w);
  r[1] = fminf(fmaxf(v.y, 0.f), a.img_h);
  r[2] = fminf(fmaxf(v.z, 0.f), a.img_w);
  r[3] = fminf(fmaxf(v.w, 0.f), a.img_h);
  r[4] = sc;
  r[5] = (float)cl;
}

__device__ __forceinline__ bool iou_gt(const float4 bi, float ai_area, const float4 bj, float aj_area, double thr) {
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.0f, __fsub_rn(xx2, xx1));
  const float h = fmaxf(0.0f, __fsub_rn(yy2, yy1));
  const float inter = ym_opaque(w * h);  // one rounding per operation, as torchvision's CPU kernel (no fused FMA)
  const float ovr = __fdiv_rn(inter, __fsub_rn(__fadd_rn(ai_area, aj_area), inter));
  return (double)ovr > thr;
}

__global__ __launch_bounds__(NMS_T) void nms_image(const NmsArgs a) {
  // one LDS arena (128 KB), carved per path: keys [NMS_LDS], boxes [NMS_LDS], areas [NMS_LDS], flags [NMS_LDS] for the
  // paths up to NMS_LDS candidates; the sort buffer, then the block / kept-list regions for the blocked path
  __shared__ __attribute__((aligned(16))) unsigned long long arena[NMS_SORT];
  unsigned long long* sk = arena;
  float4* sbx = reinterpret_cast<float4*>(arena + NMS_LDS);
  float* sar = reinterpret_cast<float*>(arena + 3 * NMS_LDS);
  unsigned char* ssup = reinterpret_cast<unsigned char*>(arena + 3 * NMS_LDS + NMS_LDS / 2);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (a.dbg == 6) return;
  unsigned long long* gk = a.keys + (size_t)b * a.kstride;
  // the first NMS_BM keys are loaded before the count is known (the key rows hold kstride >= A entries): the count
  // and the keys are ONE memory round trip instead of two dependent ones; entries past the count are ignored
  const unsigned long long kpre = tid < NMS_BM && tid < a.kstride ? gk[tid] : 0ull;
  int n = a.counts[b];
  if (n > a.A) n = a.A;
  if (a.dbg == 7) return;
  const size_t ib = (size_t)b * a.A;
  const int rowlen = 6 + a.nm;
  float* out = a.dets + (size_t)b * a.max_det * rowlen;
  if (n <= 64) {
    // common case at predict thresholds: one wave, everything in registers, no barriers.
    // lane i holds candidate i; bitonic sort by key across lanes, then the greedy scan with shuffles.
    if (tid >= 64) return;
    const int lane = tid;
    unsigned long long key = lane < n ? kpre : 0ull;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const unsigned long long other = __shfl_xor(key, stride);
        const bool desc = (lane & size) == 0 || size == 64;
        const bool lower = (lane & stride) == 0;
        const bool keep_max = lower == desc;
        key = keep_max ? (key > other ? key : other) : (key < other ? key : other);
      }
    }
    const int ne = n < a.max_nms ? n : a.max_nms;
    const unsigned ai = 0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull);
    float4 bx = make_float4(0.f, 0.f, 0.f, 0.f);
    float ar = 0.f;
    if (lane < ne) {
      const float4 v = a.boxes[ib + ai];
      const float off = a.agnostic ? 0.0f : (float)a.cls[ib + ai] * a.max_wh;
      bx = make_float4(v.x + off, v.y + off, v.z + off, v.w + off);
      ar = __fmul_rn(__fsub_rn(bx.z, bx.x), __fsub_rn(bx.w, bx.y));
    }
    int sup = lane >= ne;
    int keep = 0, kept = 0;
    // candidate i is wave-uniform: v_readlane (a VALU -> SGPR move) instead of ds_bpermute round trips
    auto rl = [](float v, int i) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i)); };
    for (int i = 0; i < ne && kept < a.max_det; ++i) {
      if (__builtin_amdgcn_readlane(sup, i)) continue;
      ++kept;
      if (lane == i) keep = 1;
      const float4 bi = make_float4(rl(bx.x, i), rl(bx.y, i), rl(bx.z, i), rl(bx.w, i));
      const float ai_area = rl(ar, i);
      if (lane > i && !sup && iou_gt(bi, ai_area, bx, ar, a.iou)) sup = 1;
    }
    const unsigned long long km = __ballot(keep);
    if (keep) {
      const int pos = __popcll(km & ((1ull << lane) - 1ull));
      write_det(a, out + (size_t)pos * rowlen, ib + ai);
    }
    if (lane == 0) {
      a.out_counts[b] = kept;
      if (a.counts2) a.counts2[b] = kept;
    }
    return;
  }
  if (n <= NMS_BM) {
    // 64 < n <= 512: rank sort (one barrier), the IoU > iou bit matrix computed by all 1024 threads, then ONE
    // wave scans it greedily (torchvision's loop: keep i unless a kept earlier box suppressed it) — no barrier
    // per kept box.  Keys are unique (anchor index in the low word), so the ranks are a permutation.
    unsigned long long* sorted = sk + NMS_BM;
    unsigned long long* mask = reinterpret_cast<unsigned long long*>(sbx + NMS_BM);  // [ne][W]
    unsigned long long ki = 0;
    if (tid < n) sk[tid] = ki = kpre;
    if (tid == n) sk[n] = 0ull;  // pad to an even count (keys are > 0: the score bits of a candidate are)
    __syncthreads();
    if (a.dbg == 1) return;
    if (tid < n) {
      int r = 0;
      const int n2 = (n + 1) >> 1;
#pragma unroll 4
      for (int j = 0; j < n2; ++j) {  // 16-byte LDS reads, two keys each
        const unsigned long long k0 = sk[2 * j], k1 = sk[2 * j + 1];
        r += (k0 > ki) + (k1 > ki);
      }
      sorted[r] = ki;
    }
    __syncthreads();
    if (a.dbg == 2) return;
    const int ne = n < a.max_nms ? n : a.max_nms;
    const int W = (ne + 63) >> 6;
    if (tid < ne) {
      const unsigned ai = 0xFFFFFFFFu - (unsigned)(sorted[tid] & 0xFFFFFFFFull);
      const float4 v = a.boxes[ib + ai];
      const float off = a.agnostic ? 0.0f : (float)a.cls[ib + ai] * a.max_wh;
      const float4 o = make_float4(v.x + off, v.y + off, v.z + off, v.w + off);
      sbx[tid] = o;
      sar[tid] = __fmul_rn(__fsub_rn(o.z, o.x), __fsub_rn(o.w, o.y));
    }
    __syncthreads();
    if (a.dbg == 3) return;
    {  // one IoU per lane: wave item (i, w) has lane l test box j = 64 w + l against row i; the ballot IS word w
      const int wv = tid >> 6, ln = tid & 63;
      for (int pq = wv; pq < ne * W; pq += NMS_T / 64) {
        const int i = pq / W, w = pq - i * W;
        const int j = 64 * w + ln;
        const bool s = 64 * w + 63 > i && j > i && j < ne && iou_gt(sbx[i], sar[i], sbx[j], sar[j], a.iou);
        const unsigned long long bits = __ballot(s);
        if (ln == 0) mask[pq] = bits;
      }
    }
    __syncthreads();
    if (a.dbg == 4) return;
    __shared__ int keep_bm[NMS_BM], kept_bm;
    if (tid < 64) {
      // greedy scan, 64 candidates per block: lane w holds removed-word w.  Within block k the decisions are a
      // wave-uniform chain on scalar registers: rem (the block's removed bits) and each row's own diagonal word are
      // read into SGPRs (readfirstlane / readlane), so a row costs a few scalar instructions, no exec-mask branch;
      // the block's kept rows are then written in parallel and OR-reduced across the wave into the later words.
      const int lane = tid, cap = a.max_det;
      // the removed words live in LDS: a kept row ORs its later mask words in with ds_or_b64 (one LDS atomic per
      // word, no cross-lane reduction)
      __shared__ unsigned long long rem_w[NMS_BM / 64];
      if (lane < W) rem_w[lane] = 0ull;
      int kept = 0;
      for (int k = 0; k < W && kept < cap; ++k) {
        const int row = 64 * k + lane;
        const unsigned long long diag = row < ne ? mask[row * W + k] : 0ull;
        const unsigned dlo = (unsigned)diag, dhi = (unsigned)(diag >> 32);
        const unsigned long long remv = rem_w[k];
        unsigned long long remk =
            ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(remv >> 32)) << 32) |
            (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)remv);
        const int jn = ne - 64 * k < 64 ? ne - 64 * k : 64;
        // visit only the rows that are kept: the next one is the lowest bit of the block's not-yet-removed rows
        // (a row's diagonal word only has bits above the row, so rows below it are final)
        unsigned long long keepbits = 0;
        int kk = kept;
        unsigned long long avail = ~remk & (jn == 64 ? ~0ull : ((1ull << jn) - 1ull));
        while (avail && kk < cap) {
          const int j = __builtin_ctzll(avail);
          keepbits |= 1ull << j;
          ++kk;
          remk |= ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(dhi, j) << 32) |
                  (unsigned long long)(unsigned)__builtin_amdgcn_readlane(dlo, j);
          avail &= ~remk & ~((2ull << j) - 1ull);
        }
        const bool mine = (keepbits >> lane) & 1ull;
        if (mine) keep_bm[kept + __popcll(keepbits & ((1ull << lane) - 1ull))] = row;
        // the block's kept rows OR their later mask words into the removed words: an OR across the wave (shuffles),
        // one LDS write per word (per-lane LDS atomics on one address serialised, ~35 per block)
        for (int w = k + 1; w < W; ++w) {
          const unsigned long long v = mine ? mask[row * W + w] : 0ull;
          unsigned vlo = (unsigned)v, vhi = (unsigned)(v >> 32);
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            vlo |= (unsigned)__shfl_xor((int)vlo, o);
            vhi |= (unsigned)__shfl_xor((int)vhi, o);
          }
          if (lane == 0) rem_w[w] |= ((unsigned long long)vhi << 32) | vlo;
        }
        kept = kk;
      }
      if (lane == 0) kept_bm = kept;
    }
    __syncthreads();
    if (a.dbg == 5) return;
    const int kept = kept_bm;
    for (int q = tid; q < kept; q += NMS_T) {
      const unsigned ai = 0xFFFFFFFFu - (unsigned)(sorted[keep_bm[q]] & 0xFFFFFFFFull);
      write_det(a, out + (size_t)q * rowlen, ib + ai);
    }
    if (tid == 0) {
      a.out_counts[b] = kept;
      if (a.counts2) a.counts2[b] = kept;
    }
    return;
  }
  if (n <= NMS_SORT && (n < a.max_nms ? n : a.max_nms) <= NMS_BLK_MAX && a.max_det <= NMS_KEEP && a.dbg != 9) {
    // the blocked path (YM_NMS_DBG=9: off, for the A/B test against the one-box-per-barrier path below)
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    if (a.dbg == 12) return;  // timing only: the kernel up to the blocked path
    for (int i = tid; i < n2; i += NMS_T) arena[i] = i < n ? gk[i] : 0ull;
    __syncthreads();
    if (a.dbg == 11) return;  // timing only: + the key loads
    // keys sorted ahead of this kernel by several workgroups per image (nms_presort_*, the validator's low conf)
    if (!(a.presorted && n > NMS_BM && n <= NMS_SORT)) bitonic_sort_desc(arena, n2, tid);
    if (a.dbg == 10) return;  // timing only: + the sort
    const int ne = n < a.max_nms ? n : a.max_nms;  // the sorted keys stay in arena[0, ne); the regions follow them
    constexpr int W = NMS_W;
    unsigned long long* reg = arena + NMS_BLK_MAX;
    float4* bb = reinterpret_cast<float4*>(reg + NR_BB);          // [NMS_BLK] class-offset boxes
    float* ba = reinterpret_cast<float*>(reg + NR_BA);            // [NMS_BLK] areas
    int* bai = reinterpret_cast<int*>(reg + NR_BAI);              // [NMS_BLK] anchor indices
    unsigned* bsup = reinterpret_cast<unsigned*>(reg + NR_BSUP);  // [NMS_BLK] removed flags
    int* bcls = reinterpret_cast<int*>(reg + NR_BCLS);            // [NMS_BLK] the class list each joins
    unsigned long long* bmask = reg + NR_BMASK;                   // [NMS_BLK][W]
    unsigned long long* ccm = reg + NR_CCM;                       // [W][NMS_NC] lanes of word w holding class c
    float4* kb = reinterpret_cast<float4*>(reg + NR_KB);          // [NMS_KEEP] kept boxes
    float* ka = reinterpret_cast<float*>(reg + NR_KA);            // [NMS_KEEP] their areas
    int* knext = reinterpret_cast<int*>(reg + NR_KNEXT);          // [NMS_KEEP] per-class kept lists
    int* khead = reinterpret_cast<int*>(reg + NR_KHEAD);          // [NMS_NC]
    __shared__ int blk_keep[NMS_BLK], blk_kept;
    __shared__ unsigned long long blk_rem[W];
    // class filter: exact when the class offsets separate every pair of boxes (decoded coordinates lie within
    // +-reg_max * stride of the image: the 2,048 margin covers 16 bins x 64 px)
    const bool cf = !a.agnostic && a.iou >= 0.0 && a.nc <= NMS_NC &&
                    (double)a.max_wh >= (double)a.img_w + (double)a.img_h + 2048.0;
    const int cap = a.max_det;  // <= NMS_KEEP
    for (int i = tid; i < W * NMS_NC; i += NMS_T) ccm[i] = 0ull;
    if (tid < NMS_NC) khead[tid] = -1;
    __syncthreads();
    int kept = 0;  // uniform: every thread reads blk_kept after the block's barrier
    for (int b0 = 0; b0 < ne && kept < cap; b0 += NMS_BLK) {
      const int nb = ne - b0 < NMS_BLK ? ne - b0 : NMS_BLK;
      if (tid < nb) {
        const unsigned ai = 0xFFFFFFFFu - (unsigned)(arena[b0 + tid] & 0xFFFFFFFFull);
        const float4 v = a.boxes[ib + ai];
        const int cl = a.cls[ib + ai];
        const float off = a.agnostic ? 0.0f : (float)cl * a.max_wh;
        const float4 o = make_float4(v.x + off, v.y + off, v.z + off, v.w + off);
        bb[tid] = o;
        ba[tid] = __fmul_rn(__fsub_rn(o.z, o.x), __fsub_rn(o.w, o.y));
        bai[tid] = (int)ai;
        const int c = cf ? cl : 0;
        bcls[tid] = c;
        if (cf) atomicOr(&ccm[(tid >> 6) * NMS_NC + c], 1ull << (tid & 63));
      }
      if (tid < NMS_BLK) bsup[tid] = tid >= nb;
      __syncthreads();
      if (tid < nb) {  // suppression by the boxes kept in earlier blocks (of this candidate's class)
        bool sj = false;
        for (int q = khead[bcls[tid]]; q >= 0 && !sj; q = knext[q]) sj = iou_gt(kb[q], ka[q], bb[tid], ba[tid], a.iou);
        if (sj) bsup[tid] = 1u;
      }
      __syncthreads();
      {  // the survivors' bit matrix: wave item (i, w) tests row i against boxes 64 w .. 64 w + 63 (ballot = word w);
         // a word without a box of row i's class (or past i) is zero without a test
        const int wv = tid >> 6, ln = tid & 63;
        for (int pq = wv; pq < nb * W; pq += NMS_T / 64) {
          const int i = pq / W, w = pq - i * W;
          const int j = 64 * w + ln;
          const int lo = i + 1 - 64 * w;  // lanes >= lo lie past row i
          const unsigned long long past = lo <= 0 ? ~0ull : (lo >= 64 ? 0ull : ~0ull << lo);
          const int hiw = nb - 64 * w;    // lanes < hiw lie inside the block
          const unsigned long long in = hiw >= 64 ? ~0ull : (hiw <= 0 ? 0ull : ((1ull << hiw) - 1ull));
          const unsigned long long cand = (cf ? ccm[w * NMS_NC + bcls[i]] : ~0ull) & past & in;
          unsigned long long bits = 0ull;
          if (!bsup[i] && cand) {  // (uniform)
            const bool sij = ((cand >> ln) & 1ull) && !bsup[j] && iou_gt(bb[i], ba[i], bb[j], ba[j], a.iou);
            bits = __ballot(sij);
          }
          if (ln == 0) bmask[pq] = bits;
        }
      }
      __syncthreads();
      if (tid < 64) {  // one wave: the block's greedy scan (the bit-matrix path's), removed words seeded by bsup
        const int lane = tid;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const unsigned long long r = __ballot(bsup[64 * w + lane] != 0u);
          if (lane == 0) blk_rem[w] = r;
        }
        int kk = kept;
        for (int k2 = 0; k2 < W && kk < cap; ++k2) {
          const int jn = nb - 64 * k2 < 64 ? nb - 64 * k2 : 64;
          if (jn <= 0) break;
          const int row = 64 * k2 + lane;
          const unsigned long long diag = row < nb ? bmask[row * W + k2] : 0ull;
          const unsigned dlo = (unsigned)diag, dhi = (unsigned)(diag >> 32);
          const unsigned long long remv = blk_rem[k2];
          unsigned long long remk =
              ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(remv >> 32)) << 32) |
              (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)remv);
          unsigned long long keepbits = 0;
          const int q0 = kk - kept;
          unsigned long long avail = ~remk & (jn == 64 ? ~0ull : ((1ull << jn) - 1ull));
          while (avail && kk < cap) {
            const int j = __builtin_ctzll(avail);
            keepbits |= 1ull << j;
            ++kk;
            remk |= ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(dhi, j) << 32) |
                    (unsigned long long)(unsigned)__builtin_amdgcn_readlane(dlo, j);
            avail &= ~remk & ~((2ull << j) - 1ull);
          }
          const bool mine = (keepbits >> lane) & 1ull;
          if (mine) blk_keep[q0 + __popcll(keepbits & ((1ull << lane) - 1ull))] = row;
          for (int w = k2 + 1; w < W; ++w) {
            const unsigned long long v = mine ? bmask[row * W + w] : 0ull;
            unsigned vlo = (unsigned)v, vhi = (unsigned)(v >> 32);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
              vlo |= (unsigned)__shfl_xor((int)vlo, o);
              vhi |= (unsigned)__shfl_xor((int)vhi, o);
            }
            if (lane == 0) blk_rem[w] |= ((unsigned long long)vhi << 32) | vlo;
          }
        }
        if (lane == 0) blk_kept = kk;
      } else if (cf) {  // the other waves clear the class masks for the next block
        for (int i = tid - 64; i < W * NMS_NC; i += NMS_T - 64) ccm[i] = 0ull;
      }
      __syncthreads();
      const int kept2 = blk_kept;
      for (int q = tid; q < kept2 - kept; q += NMS_T) {  // the block's kept boxes join their class lists; rows written
        const int r = blk_keep[q], idx = kept + q;
        kb[idx] = bb[r];
        ka[idx] = ba[r];
        knext[idx] = atomicExch(&khead[bcls[r]], idx);
        write_det(a, out + (size_t)idx * rowlen, ib + (size_t)bai[r]);
      }
      kept = kept2;
      __syncthreads();  // the kept lists are complete before the next block reads them; the block regions are free
    }
    if (tid == 0) {
      a.out_counts[b] = kept;
      if (a.counts2) a.counts2[b] = kept;
    }
    return;
  }
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  const bool lds = n2 <= NMS_LDS;
  unsigned long long* k = lds ? sk : gk;
  if (lds) {
    for (int i = tid; i < n2; i += NMS_T) sk[i] = i < n ? gk[i] : 0ull;
  } else {
    for (int i = n + tid; i < n2; i += NMS_T) gk[i] = 0ull;  // keys have a power-of-two stride >= A
  }
  __syncthreads();
  if (n > 1) bitonic_sort_desc(k, n2, tid);
  if (n > a.max_nms) n = a.max_nms;
  float4* bx = lds ? sbx : a.sboxes + (size_t)b * a.A;
  float* ar = lds ? sar : a.sareas + (size_t)b * a.A;
  unsigned char* sup = lds ? ssup : a.sup + (size_t)b * a.A;
  for (int i = tid; i < n; i += NMS_T) {
    const unsigned ai = 0xFFFFFFFFu - (unsigned)(k[i] & 0xFFFFFFFFull);
    const float4 v = a.boxes[ib + ai];
    const float off = a.agnostic ? 0.0f : (float)a.cls[ib + ai] * a.max_wh;
    const float4 o = make_float4(v.x + off, v.y + off, v.z + off, v.w + off);
    bx[i] = o;
    ar[i] = __fmul_rn(__fsub_rn(o.z, o.x), __fsub_rn(o.w, o.y));
    sup[i] = 0;
  }
  __syncthreads();
  // greedy scan: only LDS traffic inside the loop (a global store here would make every barrier drain vmcnt);
  // the kept sorted positions are recorded and written out in parallel afterwards
  __shared__ int keep_pos[1024];
  const int cap = a.max_det < 1024 ? a.max_det : 1024;
  int kept = 0;
  for (int i = 0; i < n && kept < cap; ++i) {
    if (sup[i]) continue;  // written before the last barrier; uniform across the workgroup
    const float4 bi = bx[i];
    const float ai_area = ar[i];
    if (tid == 0) keep_pos[kept] = i;
    ++kept;
    for (int j = i + 1 + tid; j < n; j += NMS_T)
      if (!sup[j] && iou_gt(bi, ai_area, bx[j], ar[j], a.iou)) sup[j] = 1;
    __syncthreads();
  }
  __syncthreads();
  for (int q = tid; q < kept; q += NMS_T) {
    const int i = keep_pos[q];
    const unsigned ai = 0xFFFFFFFFu - (unsigned)(k[i] & 0xFFFFFFFFull);
    write_det(a, out + (size_t)q * rowlen, ib + ai);
  }
  if (tid == 0) {
    a.out_counts[b] = kept;
    if (a.counts2) a.counts2[b] = kept;
  }
}

// ------------------------------------------------------------------------------------------------- profiling aid
// One wave parks for `ticks` of the constant 100 MHz wall clock.  ym_profile queues it ahead of the per-op event
// pairs so the host enqueues the whole forward while the GPU waits: the events then time device work only, not host
// launch latency.  Always terminates (bounded by the clock, not by memory state).
__global__ void spin_wait(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

}  // namespace

// ------------------------------------------------------------------------------------------------- launchers
hipError_t ym_launch_spin(int usec, hipStream_t st) {
  if (usec < 0) usec = 0;
  if (usec > 200000) usec = 200000;
  hipLaunchKernelGGL(spin_wait, dim3(1), dim3(64), 0, st, (long long)usec * 100);
  return hipGetLastError();
}

hipError_t ym_launch_prep(int dtype, const PrepArgs& a, int* counts, int B, hipStream_t st) {
  (void)dtype;
  // one launch: counters cleared, batch max reduced (or the given global max taken) — input_stats above
  const long n = (long)a.B * a.C * a.H * a.W;
  long blocks = a.batch_max ? 64 : (n / 4 + 2047) / 2048;  // >= 8 float4 per lane
  if (blocks > kStatsBlocks) blocks = kStatsBlocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(input_stats, dim3(blocks), dim3(256), 0, st, a.in, n, a.ctl, counts, B, a.cnt, a.cnt_len,
                     a.batch_max);
  return hipGetLastError();
}

hipError_t ym_launch_input_max(const float* x, long n, float* ctl, float* out, hipStream_t st) {
  long blocks = (n / 4 + 2047) / 2048;
  if (blocks > kStatsBlocks) blocks = kStatsBlocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(input_stats, dim3(blocks), dim3(256), 0, st, x, n, ctl, nullptr, 0, nullptr, 0, nullptr);
  hipLaunchKernelGGL(ctl_to_max, dim3(1), dim3(64), 0, st, ctl, out);
  return hipGetLastError();
}

// process-wide debug switches (ym_set_debug; include/yolomi.h YM_DBG_*): set from the environment once, then only by
// the setter — a launch reads an atomic instead of calling getenv (getenv per launch is not thread-safe
// against setenv and costs time on every eager forward)
namespace {
constexpr int kDbgKeys = 10;  // include/yolomi.h YM_DBG_* keys 1..9
std::atomic<int>* dbg_slots() {
  static std::atomic<int> v[kDbgKeys] = {};
  static const bool init = [] {
    const char* names[kDbgKeys] = {nullptr,       "YM_NMS_DBG", "YM_DW_MODE", "YM_DW_TILE", "YM_CHAIN",
                                   nullptr,       "YM_STEMFUSE", "YM_ATTN_KB", "YM_PAIRST", "YM_CONV_CFG"};
    for (int k = 1; k < kDbgKeys; ++k) {
      if (!names[k]) continue;
      const char* e = getenv(names[k]);
      // keys 8, 9 hold value + 1 (0: unset — the pair-store default mask, no forced tile configuration)
      v[k].store(e && *e ? atoi(e) + (k >= 8 ? 1 : 0) : 0);
    }
    return true;
  }();
  (void)init;
  return v;
}
}  // namespace

int ym_debug_get(int key) { return key > 0 && key < kDbgKeys ? dbg_slots()[key].load(std::memory_order_relaxed) : 0; }
int ym_debug_set(int key, int value) {
  if (key <= 0 || key >= kDbgKeys) return -1;
  return dbg_slots()[key].exchange(value);
}
void ym_debug_add(int key, int d) {
  if (key > 0 && key < kDbgKeys) dbg_slots()[key].fetch_add(d);
}

hipError_t ym_launch_dwconv(int dtype, const DwArgs& a, hipStream_t st) {
  if (ym_dt_q8(dtype)) return ym_launch_dwconv_i8(a, st, dtype == YM_DT_F8);
  const long total = (long)a.B * a.H * a.W * (a.C / 8);
  if (total >= 0x7FFFFFFFL - 256) return hipErrorInvalidValue;  // the kernel indexes in 32 bits
  const dim3 g((total + 255) / 256);
  if (a.C % 8) return hipErrorInvalidValue;
  // pixels per thread: 4 where that still leaves >= 128 workgroups (measured best at 80²/160²), else 2 (20²/40²)
  static const int env_pxt = [] { const char* e = getenv("YM_DW_PXT"); return e ? atoi(e) : 0; }();
  // YM_DBG_DW_MODE (A/B and tests; read at every launch, i.e. at graph capture): 0 = LDS tiles (default), 1 = row /
  // one-pixel variants, 2 = column strips
  const int mode = ym_debug_get(2);
  if (mode == 0 && !a.raw) {
    // LDS tile shape (TH x TW pixels x CG chunks; YM_DBG_DW_TILE 0..3 for A/B, read at every launch): 0 = 8 x 16 x 4
    const int ti = ym_debug_get(3);
    auto go = [&](auto th, auto tw, auto cg) -> hipError_t {
      constexpr int TH = decltype(th)::value, TW = decltype(tw)::value, CG = decltype(cg)::value;
      const long tiles = (long)a.B * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW) * ((a.C / 8 + CG - 1) / CG);
      if (tiles >= 0x7FFFFFFFL) return hipErrorInvalidValue;
      if (dtype == YM_DT_F16) hipLaunchKernelGGL((dwconv3x3_lds<f16, TH, TW, CG>), dim3(tiles), dim3(256), 0, st, a);
      else if (dtype == YM_DT_X3) hipLaunchKernelGGL((dwconv3x3_lds<P2, TH, TW, CG>), dim3(tiles), dim3(256), 0, st, a);
      else hipLaunchKernelGGL((dwconv3x3_lds<float, TH, TW, CG>), dim3(tiles), dim3(256), 0, st, a);
      return hipGetLastError();
    };
    if (ti == 1) return go(std::integral_constant<int, 4>(), std::integral_constant<int, 32>(), std::integral_constant<int, 4>());
    if (ti == 2) return go(std::integral_constant<int, 8>(), std::integral_constant<int, 32>(), std::integral_constant<int, 2>());
    if (ti == 3) return go(std::integral_constant<int, 16>(), std::integral_constant<int, 16>(), std::integral_constant<int, 2>());
    return go(std::integral_constant<int, 8>(), std::integral_constant<int, 16>(), std::integral_constant<int, 4>());
  }
  // column strips (dwconv3x3_strip): rows per thread where the grid keeps >= 256 workgroups (YM_DW_RT forces 2 / 4)
  static const int env_rt = [] { const char* e = getenv("YM_DW_RT"); return e ? atoi(e) : 0; }();
  if (mode == 2 && !a.raw) {
    const bool is16 = dtype == YM_DT_F16, x3 = dtype == YM_DT_X3;
    const int px = (a.W % 4 == 0) ? 4 : (a.W % 2 == 0 ? 2 : 0);
    auto blocks = [&](int p, int rt) { return ((long)a.B * ((a.H + rt - 1) / rt) * (a.W / p) * (a.C / 8) + 255) / 256; };
    int rt = env_rt ? env_rt : 0;
    if (!rt && px) rt = blocks(px, 4) >= 256 ? 4 : (blocks(px, 2) >= 256 ? 2 : 0);
    if (px == 4 && rt == 4) {
      const dim3 gs(blocks(4, 4));
      if (is16) hipLaunchKernelGGL((dwconv3x3_strip<f16, 4, 4>), gs, dim3(256), 0, st, a);
      else if (x3) hipLaunchKernelGGL((dwconv3x3_strip<P2, 4, 4>), gs, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((dwconv3x3_strip<float, 4, 4>), gs, dim3(256), 0, st, a);
      return hipGetLastError();
    }
    if (px && rt == 2) {
      const dim3 gs(blocks(2, 2));
      if (is16) hipLaunchKernelGGL((dwconv3x3_strip<f16, 2, 2>), gs, dim3(256), 0, st, a);
      else if (x3) hipLaunchKernelGGL((dwconv3x3_strip<P2, 2, 2>), gs, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((dwconv3x3_strip<float, 2, 2>), gs, dim3(256), 0, st, a);
      return hipGetLastError();
    }
  }
  const int pxt = env_pxt ? env_pxt : (total / 4 >= 128 * 256 ? 4 : 2);
  if (dtype == YM_DT_F16 && pxt == 4 && a.W % 4 == 0)
    hipLaunchKernelGGL((dwconv3x3_row<f16, 4>), dim3((total / 4 + 255) / 256), dim3(256), 0, st, a);
  else if (pxt >= 2 && a.W % 2 == 0 && dtype == YM_DT_F16)
    hipLaunchKernelGGL((dwconv3x3_row<f16, 2>), dim3((total / 2 + 255) / 256), dim3(256), 0, st, a);
  else if (pxt >= 2 && a.W % 2 == 0 && dtype == YM_DT_X3)
    hipLaunchKernelGGL((dwconv3x3_row<P2, 2>), dim3((total / 2 + 255) / 256), dim3(256), 0, st, a);
  else if (pxt >= 2 && a.W % 2 == 0)
    hipLaunchKernelGGL((dwconv3x3_row<float, 2>), dim3((total / 2 + 255) / 256), dim3(256), 0, st, a);
  else if (dtype == YM_DT_F16) hipLaunchKernelGGL(dwconv3x3<f16>, g, dim3(256), 0, st, a);
  else if (dtype == YM_DT_X3) hipLaunchKernelGGL(dwconv3x3<P2>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(dwconv3x3<float>, g, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_sppf(int dtype, const PoolArgs& a, hipStream_t st) {
  const size_t HW = (size_t)a.H * a.W;
  const size_t img = HW * 8 * (dtype == YM_DT_F16 ? 2 : (ym_dt_q8(dtype) ? 1 : 4));
  PoolArgs b = a;
  b.sep = 4 * img <= 128 * 1024;  // input + 3 row-max images, 8 channels
  const size_t lds = b.sep ? 4 * img : img;
  if (a.C % 8 || lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 g(a.B * (a.C / 8));
  if (dtype == YM_DT_F16) hipLaunchKernelGGL(sppf_pool<f16>, g, dim3(256), lds, st, b);
  else if (dtype == YM_DT_I8) hipLaunchKernelGGL(sppf_pool<i8>, g, dim3(256), lds, st, b);  // max on q - 128: exact
  else if (dtype == YM_DT_F8) hipLaunchKernelGGL((sppf_pool<i8, true>), g, dim3(256), lds, st, b);
  else if (dtype == YM_DT_X3) hipLaunchKernelGGL(sppf_pool<P2>, g, dim3(256), lds, st, b);  // max of hi + lo values
  else hipLaunchKernelGGL(sppf_pool<float>, g, dim3(256), lds, st, b);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_attn_t(const AttnArgs& a, hipStream_t st) {
  const size_t budget = 150 * 1024;
  auto lds = [&](int qb) { return ((size_t)qb * a.N + (size_t)qb * AKD + 64 * AHD) * sizeof(float); };
  // fewer queries per workgroup = more workgroups: with one wave per SIMD nothing hides this kernel's latencies
  auto wgs = [&](int qb) { return (long)a.B * a.nh * ((a.N + qb - 1) / qb); };
  if (lds(32) <= budget && wgs(32) >= 512) {
    hipLaunchKernelGGL((attn_psa<T, 32>), dim3(a.B * a.nh * ((a.N + 31) / 32)), dim3(256), lds(32), st, a);
  } else if (lds(16) <= budget && (wgs(16) >= 512 || lds(8) > budget)) {
    hipLaunchKernelGGL((attn_psa<T, 16>), dim3(a.B * a.nh * ((a.N + 15) / 16)), dim3(256), lds(16), st, a);
  } else if (lds(8) <= budget) {
    hipLaunchKernelGGL((attn_psa<T, 8>), dim3(a.B * a.nh * ((a.N + 7) / 8)), dim3(256), lds(8), st, a);
  } else if (lds(4) <= budget) {
    hipLaunchKernelGGL((attn_psa<T, 4>), dim3(a.B * a.nh * ((a.N + 3) / 4)), dim3(256), lds(4), st, a);
  } else {
    return hipErrorInvalidValue;  // N > ~9,600 tokens (input > 3136 px): not supported
  }
  return hipGetLastError();
}

template <int NKT>
hipError_t launch_attn_mfma(const AttnArgs& a, hipStream_t st) {
  const size_t lds = ((size_t)64 * (16 * NKT + 4) + (size_t)16 * NKT * 48) * sizeof(f16) + 640 * sizeof(float);
  hipLaunchKernelGGL((attn_psa_mfma<NKT>), dim3(a.B * a.nh * ((a.N + 63) / 64)), dim3(256), lds, st, a);
  return hipGetLastError();
}

template <bool X3>
hipError_t launch_attn_flash(const AttnArgs& a, hipStream_t st) {
  static const bool off = [] { const char* e = getenv("YM_ATTN_FLASH_OFF"); return e && *e == '1'; }();
  if (off) return hipErrorInvalidValue;
  const size_t lds = (size_t)(X3 ? 2 : 1) * 64 * (256 + 4) * sizeof(f16);
  hipLaunchKernelGGL((attn_psa_flash<X3>), dim3(a.B * a.nh * ((a.N + 63) / 64)), dim3(256), lds, st, a);
  return hipGetLastError();
}

template <int NKT>
hipError_t launch_attn_x3(const AttnArgs& a, hipStream_t st) {
  const size_t lds = (size_t)2 * 64 * (16 * NKT + 4) * sizeof(f16) + 640 * sizeof(float);
  const dim3 g(a.B * a.nh * ((a.N + 63) / 64));
  // K fragments of every key tile in flight at once (up to 26 tiles); YM_DBG_ATTN_KB = 1: 8 tiles per round trip
  constexpr int KBALL = NKT <= 26 ? NKT : 16;
  if (ym_debug_get(7) == 1) hipLaunchKernelGGL((attn_psa_x3<NKT, 8>), g, dim3(256), lds, st, a);
  else hipLaunchKernelGGL((attn_psa_x3<NKT, KBALL>), g, dim3(256), lds, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_attn(int dtype, const AttnArgs& a, hipStream_t st) {
  if (ym_dt_q8(dtype)) return ym_launch_attn_i8(a, st, dtype == YM_DT_F8);
  if (dtype == YM_DT_X3 && a.kd == 32 && a.hd == 64 && !a.raw && a.nh * 128 <= a.q_ctot && a.d_ctot % 4 == 0 &&
      a.d_coff % 4 == 0 && a.q_ctot % 8 == 0 && a.q_coff % 8 == 0) {
    const int nkt = (a.N + 15) / 16;
    if (nkt <= 8) return launch_attn_x3<8>(a, st);
    if (nkt <= 16) return launch_attn_x3<16>(a, st);
    if (nkt <= 26) return launch_attn_x3<26>(a, st);
    if (nkt <= 32) return launch_attn_x3<32>(a, st);
    const hipError_t e = launch_attn_flash<true>(a, st);
    if (e != hipErrorInvalidValue) return e;
  }
  if (dtype == YM_DT_F16 && a.kd == 32 && a.hd == 64 && !a.raw && a.nh * 128 <= a.q_ctot && a.d_ctot % 4 == 0 &&
      a.d_coff % 4 == 0 && a.q_ctot % 8 == 0 && a.q_coff % 8 == 0) {
    const int nkt = (a.N + 15) / 16;
    if (nkt <= 8) return launch_attn_mfma<8>(a, st);
    if (nkt <= 16) return launch_attn_mfma<16>(a, st);
    if (nkt <= 26) return launch_attn_mfma<26>(a, st);
    if (nkt <= 32) return launch_attn_mfma<32>(a, st);
    const hipError_t e = launch_attn_flash<false>(a, st);  // N > 512 tokens (inputs above 724 px)
    if (e != hipErrorInvalidValue) return e;  // (YM_ATTN_FLASH_OFF=1: the scalar kernel, tests)
  }
  if (a.kd > AKD || a.hd > AHD) return hipErrorInvalidValue;
  if (dtype == YM_DT_X3) return launch_attn_t<P2>(a, st);
  return dtype == YM_DT_F16 ? launch_attn_t<f16>(a, st) : launch_attn_t<float>(a, st);
}

hipError_t ym_launch_decode(const DecodeArgs& a, hipStream_t st) {
  const long total = (long)a.B * a.A;
  if (a.no_tot % 4) return hipErrorInvalidValue;
  // YM_DECODE_STAGED=1 forces the general LDS-staged variant (tests: both variants agree bit for bit)
  static const bool staged = [] {
    const char* e = getenv("YM_DECODE_STAGED");
    return e && *e == '1';
  }();
  if (a.reg_max == 16 && a.nc == 80 && !staged) {
    hipLaunchKernelGGL(decode_anchors<true>, dim3((total + 63) / 64), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(decode_anchors<false>, dim3((total + 63) / 64), dim3(256), (size_t)64 * (a.no_tot + 1) * sizeof(float), st,
                     a);
  return hipGetLastError();
}

hipError_t ym_launch_nms(const NmsArgs& a0, hipStream_t st) {
  NmsArgs a = a0;
  a.dbg = ym_debug_get(1);  // YM_DBG_NMS (a test switches the blocked path off between eager runs)
  hipLaunchKernelGGL(nms_image, dim3(a.B), dim3(NMS_T), 0, st, a);
  return hipGetLastError();
}

const void* ym_nms_kernel() { return reinterpret_cast<const void*>(&nms_image); }

// ---- multi-workgroup presort of the NMS keys (verdict r5 item 6: at the validator's conf 0.001 the blocked path's
// one-workgroup sort of up to 16,384 keys took ~130 of nms_image's ~254 us, profiles/r05ad_nms_sort_probe.txt).
// Phase 1: NMS_SORT / PS_CH workgroups per image each sort one 2,048-key chunk in LDS (descending; padding keys 0,
// a real key is never 0: its score bits are those of a positive float) into keys2.  Phase 2: each workgroup stages
// all of its image's sorted chunks in LDS (<= 128 KB) and gives each key of its own chunk its final position —
// its index in its chunk plus, per other chunk, the number of larger keys there (a binary search; keys are unique,
// the anchor index is in their low bits) — and writes it back to keys.  Both phases exit at once for an image with
// <= NMS_BM or > NMS_SORT candidates, where nms_image keeps its own sort (NmsArgs::presorted is checked alike).
constexpr int PS_CH = 2048;
constexpr int PS_NCH = NMS_SORT / PS_CH;

__global__ __launch_bounds__(NMS_T) void nms_presort_chunks(const NmsArgs a) {
  __shared__ unsigned long long k[PS_CH];
  const int b = blockIdx.x / PS_NCH, c = blockIdx.x % PS_NCH, tid = threadIdx.x;
  int n = a.counts[b];
  if (n > a.A) n = a.A;
  if (n <= NMS_BM || n > NMS_SORT || c * PS_CH >= n) return;
  const unsigned long long* gk = a.keys + (size_t)b * a.kstride + c * PS_CH;
  const int m = n - c * PS_CH;
  for (int i = tid; i < PS_CH; i += NMS_T) k[i] = i < m ? gk[i] : 0ull;
  __syncthreads();
  bitonic_sort_desc(k, PS_CH, tid);
  unsigned long long* out = a.keys2 + (size_t)b * a.kstride + c * PS_CH;
  for (int i = tid; i < PS_CH; i += NMS_T) out[i] = k[i];
}

__global__ __launch_bounds__(NMS_T) void nms_presort_merge(const NmsArgs a) {
  __shared__ unsigned long long s[NMS_SORT];
  const int b = blockIdx.x / PS_NCH, c = blockIdx.x % PS_NCH, tid = threadIdx.x;
  int n = a.counts[b];
  if (n > a.A) n = a.A;
  if (n <= NMS_BM || n > NMS_SORT || c * PS_CH >= n) return;
  const int nc = (n + PS_CH - 1) / PS_CH;
  const unsigned long long* src = a.keys2 + (size_t)b * a.kstride;
  for (int i = tid; i < nc * PS_CH; i += NMS_T) s[i] = src[i];
  __syncthreads();
  unsigned long long* gk = a.keys + (size_t)b * a.kstride;
  for (int j = tid; j < PS_CH; j += NMS_T) {
    const unsigned long long key = s[c * PS_CH + j];
    if (key == 0ull) continue;  // chunk padding
    int rank = j;
    for (int c2 = 0; c2 < nc; ++c2) {
      if (c2 == c) continue;
      const unsigned long long* q = s + c2 * PS_CH;
      int lo = 0, hi = PS_CH;  // the first index whose key is smaller (descending order)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (q[mid] > key) lo = mid + 1;
        else hi = mid;
      }
      rank += lo;
    }
    gk[rank] = key;
  }
}

hipError_t ym_launch_nms_presort(const NmsArgs& a, hipStream_t st) {
  if (!a.keys2 || a.kstride < NMS_SORT) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nms_presort_chunks, dim3(a.B * PS_NCH), dim3(NMS_T), 0, st, a);
  hipLaunchKernelGGL(nms_presort_merge, dim3(a.B * PS_NCH), dim3(NMS_T), 0, st, a);
  return hipGetLastError();
}
