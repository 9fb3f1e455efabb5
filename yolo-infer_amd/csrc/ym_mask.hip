// Instance-mask assembly of the Segment head: Ultralytics `ops.process_mask(proto, coef, boxes, shape, upsample=True)`
// as the segmentation predictor calls it for tensor sources (reached from `YOLO11Model.predict`,
// /root/reference/core/model.py:133), then the non-empty filter of the predictor's result construction.
//   1. mask_lowres: m[d](y, x) = Σ_c coef[d][c] · proto[b](y, x, c), zeroed outside the box scaled to prototype
//      resolution (crop_mask: x1·r ≤ x < x2·r, same for y, compared in fp32 as torch does on float aranges);
//   2. mask_upsample: bilinear resize to (H, W) with align_corners=False (torch upsample_bilinear2d source index
//      (dst + 0.5)·in/out − 0.5 clamped at 0, neighbour clamped at in − 1), then > 0 → one byte per pixel; a
//      ballot per wave sets the detection's non-empty flag.
// Both kernels are bandwidth-light per pixel; the (n, H, W) byte masks are the dominant traffic (n · H · W bytes).
// When a workgroup's source rows fit in LDS (the usual 4x prototype scale), mask_upsample16 does both steps in one
// launch: it computes the prototype-resolution rows it reads straight into LDS and writes 16 mask bytes per thread.
#include "ym_common.h"

namespace {

__device__ __forceinline__ int image_of(const int* off, int B, int d) {
  int b = 0;
  while (b + 1 < B && off[b + 1] <= d) ++b;
  return b;
}

// the detection row of mask d, or null for an unused slot (slot mode); b = its image
__device__ __forceinline__ const float* det_row(const MaskArgs& a, int d, int& b) {
  if (a.counts) {
    b = d / a.cap;
    const int i = d - b * a.cap;
    return i < a.counts[b] ? a.dets + ((size_t)b * a.max_det + i) * a.no : nullptr;
  }
  b = image_of(a.offsets, a.B, d);
  return a.dets + ((size_t)b * a.max_det + (d - a.offsets[b])) * a.no;
}

__global__ __launch_bounds__(256) void mask_lowres(const MaskArgs a) {
  const int d = blockIdx.y;
  int b;
  const float* row = det_row(a, d, b);
  if (!row) return;  // unused slot (uniform per workgroup)
  __shared__ float coef[64];
  if (threadIdx.x < a.nm) coef[threadIdx.x] = row[6 + threadIdx.x];
  __syncthreads();
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= a.MH * a.MW) return;
  const int y = p / a.MW, x = p - (p / a.MW) * a.MW;
  // crop_mask on boxes scaled by (mw / iw, mh / ih)
  const float rw = (float)a.MW / (float)a.W, rh = (float)a.MH / (float)a.H;
  const float bx1 = row[0] * rw, by1 = row[1] * rh, bx2 = row[2] * rw, by2 = row[3] * rh;
  const bool in = (float)x >= bx1 && (float)x < bx2 && (float)y >= by1 && (float)y < by2;
  float v = 0.f;
  if (in) {
    const f32x4* pr = reinterpret_cast<const f32x4*>(a.proto + ((size_t)b * a.MH * a.MW + p) * a.nm);
#pragma unroll 8
    for (int c4 = 0; c4 < a.nm / 4; ++c4) {
      const f32x4 q = pr[c4];
      v = fmaf(coef[4 * c4], q[0], v);
      v = fmaf(coef[4 * c4 + 1], q[1], v);
      v = fmaf(coef[4 * c4 + 2], q[2], v);
      v = fmaf(coef[4 * c4 + 3], q[3], v);
    }
  }
  a.lowres[(size_t)d * a.MH * a.MW + p] = v;
}

__device__ __forceinline__ bool upsample_px(const MaskArgs& a, const float* m, int oy, int ox) {
  const float sy_ = (float)a.MH / (float)a.H, sx_ = (float)a.MW / (float)a.W;
  float fy = ((float)oy + 0.5f) * sy_ - 0.5f, fx = ((float)ox + 0.5f) * sx_ - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 < a.MH - 1 ? y0 + 1 : y0, x1 = x0 < a.MW - 1 ? x0 + 1 : x0;
  const float ly = fy - (float)y0, lx = fx - (float)x0;
  const float v = (1.f - ly) * ((1.f - lx) * m[y0 * a.MW + x0] + lx * m[y0 * a.MW + x1]) +
                  ly * ((1.f - lx) * m[y1 * a.MW + x0] + lx * m[y1 * a.MW + x1]);
  return v > 0.f;
}

// one pixel per thread (any W)
__global__ __launch_bounds__(256) void mask_upsample(const MaskArgs a) {
  const int d = blockIdx.y;
  int b;
  if (!det_row(a, d, b)) return;  // unused slot (uniform per workgroup)
  const int p = blockIdx.x * 256 + threadIdx.x;
  bool on = false;
  if (p < a.H * a.W) {
    const int oy = p / a.W, ox = p - (p / a.W) * a.W;
    on = upsample_px(a, a.lowres + (size_t)d * a.MH * a.MW, oy, ox);
    a.masks[(size_t)d * a.H * a.W + p] = on ? 1 : 0;
  }
  const unsigned long long bal = __ballot(on);  // every lane reaches this (no early return above)
  if (bal && (threadIdx.x & 63) == __builtin_ctzll(bal)) a.nonempty[d] = 1;
}

// 16 consecutive pixels of a row per thread and run (W % 16 == 0): one 16-byte store instead of 16 byte stores; the
// prototype-resolution rows the workgroup's output rows read (at most LROWS) are staged in LDS once, so a pixel's four
// bilinear taps are LDS reads; 16-pixel runs wholly outside the box (scaled to prototype resolution, plus the
// bilinear reach) are all zero — crop_mask zeroes the prototype mask there — and are stored without evaluation.
// A workgroup covers RPT x 256 runs (~26 rows at 640 px): its dependent chain (detection row -> coefficients ->
// prototype rows -> masks) is paid once per 16 KB of mask instead of once per 4 KB (yolo11s-seg B=4: 25,600
// workgroups of ~5 us chains made the masks ~130 us per predict, well above their ~12 us of stores).
constexpr int LROWS = 12, LMW = 512, RPT = 4;
__global__ __launch_bounds__(256) void mask_upsample16(const MaskArgs a) {
  __shared__ float tile[LROWS * LMW];
  const int d = blockIdx.y;
  const int runs = a.W >> 4;
  const int q0 = blockIdx.x * 256 * RPT;  // first 16-pixel run of the workgroup
  int b;
  const float* row = det_row(a, d, b);
  if (!row) return;  // unused slot (uniform per workgroup)
  const float sx = (float)a.W / (float)a.MW, sy = (float)a.H / (float)a.MH;
  const float rw = (float)a.MW / (float)a.W, rh = (float)a.MH / (float)a.H;
  // lowres crop [floor(x1 r), ceil(x2 r)) in output pixels, widened by two source pixels each side (the bilinear
  // reach is one; the second is margin for the float bounds)
  const float lo_x = (floorf(row[0] * rw) - 2.f) * sx, hi_x = (ceilf(row[2] * rw) + 2.f) * sx;
  const float lo_y = (floorf(row[1] * rh) - 2.f) * sy, hi_y = (ceilf(row[3] * rh) + 2.f) * sy;
  // source rows of this workgroup's output rows
  const int oyA = q0 / runs, oyB = min((q0 + 256 * RPT - 1) / runs, a.H - 1);
  auto src_y = [&](int oy) { const float f = ((float)oy + 0.5f) * rh - 0.5f; return f < 0.f ? 0 : (int)f; };
  const int ya = src_y(oyA), yb = min(src_y(oyB) + 1, a.MH - 1);
  const bool rows_hit = (float)oyB >= lo_y && (float)oyA < hi_y;
  // the prototype-resolution mask of rows ya..yb, computed here (mask_lowres's arithmetic: crop test in fp32, the
  // coefficient dot product as the same fmaf chain), so no (total, MH, MW) intermediate is written or re-read
  __shared__ float coef[64];
  if (threadIdx.x < a.nm) coef[threadIdx.x] = row[6 + threadIdx.x];
  __syncthreads();
  if (rows_hit) {
    const float bx1 = row[0] * rw, by1 = row[1] * rh, bx2 = row[2] * rw, by2 = row[3] * rh;
    // crop_mask's integer ranges (x >= bx1 and x < bx2 in fp32 <=> ceil(bx1) <= x < ceil(bx2)), clipped to the tile:
    // out-of-box entries are zeroed first, then only the in-box ones are computed — a narrow box's few pixels spread
    // over all threads instead of one dependent prototype load round per 256 tile entries
    const int cx0 = max(0, (int)ceilf(bx1)), cx1 = min(a.MW, (int)ceilf(bx2));
    const int cy0 = max(ya, (int)ceilf(by1)), cy1 = min(yb + 1, (int)ceilf(by2));
    for (int i = threadIdx.x; i < (yb - ya + 1) * a.MW; i += 256) {
      const int y = ya + i / a.MW, x = i - (i / a.MW) * a.MW;
      if (!(x >= cx0 && x < cx1 && y >= cy0 && y < cy1)) tile[i] = 0.f;
    }
    const int bw = cx1 - cx0, nin = cx1 > cx0 && cy1 > cy0 ? (cy1 - cy0) * bw : 0;
    for (int j = threadIdx.x; j < nin; j += 256) {
      const int y = cy0 + j / bw, x = cx0 + (j - (j / bw) * bw);
      const f32x4* pr = reinterpret_cast<const f32x4*>(a.proto + ((size_t)b * a.MH * a.MW + (size_t)y * a.MW + x) * a.nm);
      float v = 0.f;
#pragma unroll 8
      for (int c4 = 0; c4 < a.nm / 4; ++c4) {
        const f32x4 p4 = pr[c4];
        v = fmaf(coef[4 * c4], p4[0], v);
        v = fmaf(coef[4 * c4 + 1], p4[1], v);
        v = fmaf(coef[4 * c4 + 2], p4[2], v);
        v = fmaf(coef[4 * c4 + 3], p4[3], v);
      }
      tile[(y - ya) * a.MW + x] = v;
    }
  }
  __syncthreads();
  bool on = false;
#pragma unroll 1
  for (int r = 0; r < RPT; ++r) {
    const int q = q0 + 256 * r + threadIdx.x;  // consecutive threads: consecutive runs (coalesced 16-byte stores)
    if (q >= a.H * runs) break;
    const int oy = q / runs, ox0 = (q - oy * runs) * 16;
    unsigned w[4] = {0u, 0u, 0u, 0u};
    if (rows_hit && (float)oy >= lo_y && (float)oy < hi_y && (float)(ox0 + 16) > lo_x && (float)ox0 < hi_x) {
      float fy = ((float)oy + 0.5f) * rh - 0.5f;
      fy = fy < 0.f ? 0.f : fy;
      const int y0 = (int)fy, y1 = y0 < a.MH - 1 ? y0 + 1 : y0;
      const float ly = fy - (float)y0;
      const float* t0 = tile + (y0 - ya) * a.MW;
      const float* t1 = tile + (y1 - ya) * a.MW;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float fx = ((float)(ox0 + i) + 0.5f) * rw - 0.5f;
        fx = fx < 0.f ? 0.f : fx;
        const int x0 = (int)fx, x1 = x0 < a.MW - 1 ? x0 + 1 : x0;
        const float lx = fx - (float)x0;
        const float v = (1.f - ly) * ((1.f - lx) * t0[x0] + lx * t0[x1]) + ly * ((1.f - lx) * t1[x0] + lx * t1[x1]);
        if (v > 0.f) w[i >> 2] |= 1u << (8 * (i & 3));
      }
      on = on || (w[0] | w[1] | w[2] | w[3]) != 0u;
    }
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<u32x4*>(a.masks + (size_t)d * a.H * a.W + (size_t)oy * a.W + ox0) = u32x4{w[0], w[1], w[2], w[3]};
  }
  const unsigned long long bal = __ballot(on);
  if (bal && (threadIdx.x & 63) == __builtin_ctzll(bal)) a.nonempty[d] = 1;
}

}  // namespace

// host-side: can the rows a 256-run workgroup reads be staged (at most LROWS prototype rows of at most LMW)?
bool ym_masks_fused(const MaskArgs& a) {
  if (a.W % 16 || a.MW > LMW) return false;
  const int runs = a.W / 16;
  const int rows_out = 256 * RPT / runs + 2;  // output rows one workgroup touches
  return (int)ceilf((float)rows_out * a.MH / a.H) + 2 <= LROWS;
}

namespace {
__global__ void mask_flags_init(const MaskArgs a) {  // slot mode: flags zeroed, the counts copied behind them
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.total) a.nonempty[i] = 0;
  else if (i < a.total + a.B) a.nonempty[i] = a.counts[i - a.total];
}
}  // namespace

hipError_t ym_launch_masks(const MaskArgs& a, hipStream_t st) {
  if (a.total <= 0) return hipSuccess;
  if (a.nm > 64 || a.nm % 4) return hipErrorInvalidValue;
  if (a.counts)
    hipLaunchKernelGGL(mask_flags_init, dim3((a.total + a.B + 255) / 256), dim3(256), 0, st, a);
  else
    (void)hipMemsetAsync(a.nonempty, 0, (size_t)a.total * sizeof(int), st);
  if (ym_masks_fused(a)) {  // fused: prototype masks computed per workgroup in LDS
    hipLaunchKernelGGL(mask_upsample16, dim3((a.H * (a.W / 16) + 256 * RPT - 1) / (256 * RPT), a.total), dim3(256), 0,
                       st, a);
  } else {
    hipLaunchKernelGGL(mask_lowres, dim3((a.MH * a.MW + 255) / 256, a.total), dim3(256), 0, st, a);
    hipLaunchKernelGGL(mask_upsample, dim3((a.H * a.W + 255) / 256, a.total), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}
