// Bandwidth-/latency-bound kernels of the YOLO11 inference path on gfx950:
//   input prep (LoadTensor /255 rule + NCHW fp32 → NHWC), depthwise 3x3 (Detect cv3 DWConv), fused SPPF max-pool
//   pyramid, C2PSA attention (+ fused positional depthwise conv), anchor-free DFL decode, class-offset greedy NMS.
// Each replaces an upstream Ultralytics/ATen/torchvision op reached from `YOLO11Model.predict`
// (/root/reference/core/model.py:133) — SURVEY §2.2 and §8a rows a2, a8, a9, a11-a14.
#include "ym_common.h"

namespace {

// ------------------------------------------------------------------------------------------------- input prep
// LoadTensor._single_check: `if im.max() > 1 + finfo(dtype).eps: im = im.float() / 255` over the WHOLE batch.
// ctl[0] holds max as an order-preserving int; ctl is reset by the init kernel at the start of every forward.
__device__ __forceinline__ int f2ord(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

__global__ void init_ctl(float* ctl, int* counts, int B) {
  const int t = threadIdx.x;
  if (t == 0) reinterpret_cast<int*>(ctl)[0] = f2ord(-INFINITY);
  for (int b = t; b < B; b += blockDim.x) counts[b] = 0;
}

__global__ __launch_bounds__(256) void max_reduce(const float* __restrict__ x, long n, float* ctl) {
  float m = -INFINITY;
  const long n4 = n >> 2;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f32x4 v = x4[i];
    m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
  }
  for (long i = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    m = fmaxf(m, x[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    atomicMax(reinterpret_cast<int*>(ctl), f2ord(m));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void prep_nhwc(const PrepArgs a) {
  const long HW = (long)a.H * a.W;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)a.B * HW) return;
  const long b = i / HW, p = i - b * HW;
  const float mx = ord2f(reinterpret_cast<const int*>(a.ctl)[0]);
  const bool div = mx > 1.0f + a.eps;
  typename Vec8<T>::type v = Vec8<T>::zero();
  for (int c = 0; c < a.C; ++c) {
    float x = a.in[(b * a.C + c) * HW + p];
    if (div) x = x / 255.0f;
    v[c] = (T)x;
  }
  Vec8<T>::store(static_cast<T*>(a.out) + i * 8, v);
}

// ------------------------------------------------------------------------------------------------- depthwise 3x3
// DWConv(c, c, 3) = Conv(g=c): 3x3, stride 1, pad 1, BN folded, SiLU.  One thread = 8 channels of one pixel.
template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3(const DwArgs a) {
  const int C8 = a.C >> 3;
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)a.B * a.H * a.W * C8;
  if (idx >= total) return;
  const int cg = idx % C8;
  const long pix = idx / C8;
  const int HW = a.H * a.W;
  const int b = pix / HW;
  const int p = pix - (long)b * HW;
  const int y = p / a.W, x = p - (p / a.W) * a.W;
  const int c0 = cg * 8;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = a.bias[c0 + e];
  const T* src = static_cast<const T*>(a.src);
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = y + ky - 1;
    if ((unsigned)iy >= (unsigned)a.H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = x + kx - 1;
      if ((unsigned)ix >= (unsigned)a.W) continue;
      const typename Vec8<T>::type v =
          Vec8<T>::load(src + (size_t)(b * a.s_P + iy * a.W + ix) * a.s_ctot + a.s_coff + c0);
      const float* wr = a.w + (ky * 3 + kx) * a.C + c0;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf((float)v[e], wr[e], acc[e]);
    }
  }
  typename Vec8<T>::type o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (T)(a.act ? ym_silu(acc[e]) : acc[e]);
  Vec8<T>::store(static_cast<T*>(a.dst) + (size_t)(b * a.d_P + p) * a.d_ctot + a.d_coff + c0, o);
}

// ------------------------------------------------------------------------------------------------- SPPF pools
// y1 = max5(y0), y2 = max5(y1) = max9(y0), y3 = max13(y0): stride 1, -inf padding, all three in one pass.
template <typename T>
__global__ __launch_bounds__(256) void sppf_pool(const PoolArgs a) {
  const int C8 = a.C >> 3;
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)a.B * a.H * a.W * C8;
  if (idx >= total) return;
  const int cg = idx % C8;
  const long pix = idx / C8;
  const int HW = a.H * a.W;
  const int b = pix / HW;
  const int p = pix - (long)b * HW;
  const int y = p / a.W, x = p - (p / a.W) * a.W;
  const int c0 = cg * 8;
  T* buf = static_cast<T*>(a.buf);
  float m5[8], m9[8], m13[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) m5[e] = m9[e] = m13[e] = -INFINITY;
  for (int dy = -6; dy <= 6; ++dy) {
    const int iy = y + dy;
    if ((unsigned)iy >= (unsigned)a.H) continue;
    const int ady = dy < 0 ? -dy : dy;
    for (int dx = -6; dx <= 6; ++dx) {
      const int ix = x + dx;
      if ((unsigned)ix >= (unsigned)a.W) continue;
      const int adx = dx < 0 ? -dx : dx;
      const int r = ady > adx ? ady : adx;
      const typename Vec8<T>::type v =
          Vec8<T>::load(buf + (size_t)(b * a.P + iy * a.W + ix) * a.ctot + a.coff + c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = (float)v[e];
        m13[e] = fmaxf(m13[e], f);
        if (r <= 4) m9[e] = fmaxf(m9[e], f);
        if (r <= 2) m5[e] = fmaxf(m5[e], f);
      }
    }
  }
  typename Vec8<T>::type o5, o9, o13;
#pragma unroll
  for (int e = 0; e < 8; ++e) { o5[e] = (T)m5[e]; o9[e] = (T)m9[e]; o13[e] = (T)m13[e]; }
  T* base = buf + (size_t)(b * a.P + p) * a.ctot + a.coff + c0;
  Vec8<T>::store(base + a.C, o5);
  Vec8<T>::store(base + 2 * a.C, o9);
  Vec8<T>::store(base + 3 * a.C, o13);
}

// ------------------------------------------------------------------------------------------------- attention
// C2PSA Attention: per (image, head): softmax((qᵀk)·kd^-½) over N = H·W tokens, o = v·Aᵀ, plus pe(v) (depthwise
// 3x3 + folded BN, no act) — the `(v @ attn.T).view(B,C,H,W) + self.pe(v)` of the upstream module.
// One workgroup = 64 queries of one (b, head); keys streamed in chunks of 64 with an online softmax (fp32).
constexpr int AQ = 64, AK = 64, AKD = 32, AHD = 64;

template <typename T>
__global__ __launch_bounds__(256) void attn_psa(const AttnArgs a) {
  __shared__ float Qs[AQ][AKD + 1];
  __shared__ float Ks[AK][AKD + 1];
  __shared__ float Vs[AK][AHD + 1];
  __shared__ float Ps[AQ][AK + 1];
  const int nqb = (a.N + AQ - 1) / AQ;
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int h = bh % a.nh;
  const int b = bh / a.nh;
  const int tid = threadIdx.x;
  const int per = 2 * a.kd + a.hd;
  const T* qkv = static_cast<const T*>(a.qkv);
  const size_t img = (size_t)b * a.q_P;
  const int hq = a.q_coff + h * per;

  for (int i = tid; i < AQ * AKD; i += 256) {
    const int r = i / AKD, c = i % AKD;
    const int n = qb * AQ + r;
    Qs[r][c] = (n < a.N && c < a.kd) ? (float)qkv[(img + n) * a.q_ctot + hq + c] : 0.f;
  }
  const int qr = tid >> 2;    // query row owned (4 threads per row)
  const int sub = tid & 3;    // key quarter for scores, dim quarter for the output
  const int d0 = sub * (AHD / 4);
  float mrow = -INFINITY, lrow = 0.f;
  float o[AHD / 4];
#pragma unroll
  for (int e = 0; e < AHD / 4; ++e) o[e] = 0.f;

  for (int k0 = 0; k0 < a.N; k0 += AK) {
    __syncthreads();
    for (int i = tid; i < AK * AKD; i += 256) {
      const int r = i / AKD, c = i % AKD;
      const int n = k0 + r;
      Ks[r][c] = (n < a.N && c < a.kd) ? (float)qkv[(img + n) * a.q_ctot + hq + a.kd + c] : 0.f;
    }
    for (int i = tid; i < AK * AHD; i += 256) {
      const int r = i / AHD, c = i % AHD;
      const int n = k0 + r;
      Vs[r][c] = (n < a.N && c < a.hd) ? (float)qkv[(img + n) * a.q_ctot + hq + 2 * a.kd + c] : 0.f;
    }
    __syncthreads();
    float s[AK / 4];
    float cmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < AK / 4; ++j) {
      const int kj = sub * (AK / 4) + j;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < AKD; ++c) acc = fmaf(Qs[qr][c], Ks[kj][c], acc);
      acc *= a.scale;
      if (k0 + kj >= a.N) acc = -INFINITY;
      s[j] = acc;
      cmax = fmaxf(cmax, acc);
    }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 1));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 2));
    const float mnew = fmaxf(mrow, cmax);
    const float alpha = expf(mrow - mnew);
    float psum = 0.f;
#pragma unroll
    for (int j = 0; j < AK / 4; ++j) {
      const float pj = expf(s[j] - mnew);
      psum += pj;
      Ps[qr][sub * (AK / 4) + j] = pj;
    }
    psum += __shfl_xor(psum, 1);
    psum += __shfl_xor(psum, 2);
    lrow = lrow * alpha + psum;
    mrow = mnew;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < AHD / 4; ++e) o[e] *= alpha;
    for (int kj = 0; kj < AK; ++kj) {
      const float pj = Ps[qr][kj];
#pragma unroll
      for (int e = 0; e < AHD / 4; ++e) o[e] = fmaf(pj, Vs[kj][d0 + e], o[e]);
    }
  }
  const int n = qb * AQ + qr;
  if (n >= a.N) return;
  const int y = n / a.W, x = n - (n / a.W) * a.W;
  T* dst = static_cast<T*>(a.dst);
  const float inv = 1.0f / lrow;
  for (int e = 0; e < AHD / 4; ++e) {
    const int d = d0 + e;
    if (d >= a.hd) break;
    const int ch = h * a.hd + d;
    float pe = a.pe_b[ch];
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = y + ky - 1;
      if ((unsigned)iy >= (unsigned)a.H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = x + kx - 1;
        if ((unsigned)ix >= (unsigned)a.W) continue;
        pe = fmaf((float)qkv[(img + iy * a.W + ix) * a.q_ctot + hq + 2 * a.kd + d], a.pe_w[(ky * 3 + kx) * a.C + ch],
                  pe);
      }
    }
    dst[((size_t)b * a.d_P + n) * a.d_ctot + a.d_coff + ch] = (T)(o[e] * inv + pe);
  }
}

// ------------------------------------------------------------------------------------------------- decode
// Detect._inference + the candidate stage of non_max_suppression, one thread per anchor:
//   DFL softmax over reg_max bins per side → ltrb distances → dist2bbox(xywh) · stride → xywh2xyxy;
//   sigmoid class scores → (max, first argmax); candidate iff max > conf (and class in the filter).
// Candidates are appended to a per-image key list: key = score bits << 32 | ~anchor, so a descending sort gives
// score-descending order with ties broken by ascending anchor index (torchvision's stable sort).
__global__ __launch_bounds__(256) void decode_anchors(const DecodeArgs a) {
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)a.B * a.A) return;
  const int b = idx / a.A;
  const int ai = idx - (long)b * a.A;
  const float* row = a.anchors + idx * a.no_tot;
  int l = 0;
  while (l + 1 < a.nl && ai >= a.lvl_off[l + 1]) ++l;
  const int p = ai - a.lvl_off[l];
  const float ax = (float)(p % a.lvl_W[l]) + 0.5f;
  const float ay = (float)(p / a.lvl_W[l]) + 0.5f;
  const float st = a.lvl_stride[l];
  float dist[4];
  for (int s = 0; s < 4; ++s) {
    const float* r = row + s * a.reg_max;
    float mx = -INFINITY;
    for (int i = 0; i < a.reg_max; ++i) mx = fmaxf(mx, r[i]);
    float den = 0.f, num = 0.f;
    for (int i = 0; i < a.reg_max; ++i) {
      const float e = expf(r[i] - mx);
      den += e;
    }
    for (int i = 0; i < a.reg_max; ++i) num = fmaf(expf(r[i] - mx) / den, (float)i, num);
    dist[s] = num;
  }
  const float x1 = ax - dist[0], y1 = ay - dist[1];
  const float x2 = ax + dist[2], y2 = ay + dist[3];
  const float cx = (x1 + x2) / 2.0f * st, cy = (y1 + y2) / 2.0f * st;
  const float w = (x2 - x1) * st, hh = (y2 - y1) * st;
  const float hw = w / 2.0f, hh2 = hh / 2.0f;
  a.boxes[idx] = make_float4(cx - hw, cy - hh2, cx + hw, cy + hh2);
  const float* cl = row + 4 * a.reg_max;
  float best = -INFINITY;
  int bi = 0;
  for (int c = 0; c < a.nc; ++c) {
    const float sc = ym_sigmoid(cl[c]);
    if (sc > best) { best = sc; bi = c; }
  }
  a.scores[idx] = best;
  a.cls[idx] = bi;
  bool cand = best > a.conf;
  if (cand && a.has_classes) cand = (a.classes[bi >> 5] >> (bi & 31)) & 1u;
  if (cand) {
    const int slot = atomicAdd(&a.counts[b], 1);
    a.keys[(size_t)b * a.kstride + slot] =
        ((unsigned long long)__float_as_uint(best) << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)ai);
  }
}

// ------------------------------------------------------------------------------------------------- NMS
// Per image, one 1024-thread workgroup: bitonic sort of the candidate keys (LDS when they fit), then greedy
// suppression exactly as torchvision's CPU nms: boxes offset by cls·max_wh (0 if agnostic), areas and IoU in fp32
// on the offset boxes, suppress iff IoU > iou (compared in double), keep ≤ max_det, clip to the image.
constexpr int NMS_T = 1024;
constexpr int NMS_LDS_KEYS = 8192;

__device__ void bitonic_sort_desc(unsigned long long* k, int n2, int tid) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (n2 >> 1); i += NMS_T) {
        const int lo = (i / stride) * stride * 2 + (i % stride);
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const unsigned long long x = k[lo], y = k[hi];
        if ((x < y) == desc) { k[lo] = y; k[hi] = x; }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(NMS_T) void nms_image(const NmsArgs a) {
  __shared__ unsigned long long sk[NMS_LDS_KEYS];

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  int n = a.counts[b];
  if (n > a.A) n = a.A;
  unsigned long long* gk = a.keys + (size_t)b * a.kstride;
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  const bool in_lds = n2 <= NMS_LDS_KEYS;
  unsigned long long* k = in_lds ? sk : gk;
  if (in_lds) {
    for (int i = tid; i < n2; i += NMS_T) sk[i] = i < n ? gk[i] : 0ull;
  } else {
    // the key list of each image has a power-of-two stride >= A (runtime), so padding up to n2 is in bounds
    for (int i = n + tid; i < n2; i += NMS_T) gk[i] = 0ull;
  }
  __syncthreads();
  if (n > 1) bitonic_sort_desc(k, n2, tid);
  if (n > a.max_nms) n = a.max_nms;

  // sorted, class-offset boxes and areas
  float4* sb = a.sboxes + (size_t)b * a.A;
  float* sa = a.sareas + (size_t)b * a.A;
  unsigned char* sup = a.sup + (size_t)b * a.A;
  const size_t ib = (size_t)b * a.A;
  for (int i = tid; i < n; i += NMS_T) {
    const unsigned ai = 0xFFFFFFFFu - (unsigned)(k[i] & 0xFFFFFFFFull);
    const float4 bx = a.boxes[ib + ai];
    const float off = a.agnostic ? 0.0f : (float)a.cls[ib + ai] * a.max_wh;
    const float4 o = make_float4(bx.x + off, bx.y + off, bx.z + off, bx.w + off);
    sb[i] = o;
    sa[i] = __fmul_rn(__fsub_rn(o.z, o.x), __fsub_rn(o.w, o.y));
    sup[i] = 0;
  }

  __syncthreads();

  const int rowlen = 6 + a.nm;
  float* out = a.dets + (size_t)b * a.max_det * rowlen;
  int kept = 0;
  for (int i = 0; i < n && kept < a.max_det; ++i) {
    if (sup[i]) continue;  // written before the last barrier; uniform across the workgroup
    const float4 bi = sb[i];
    const float ai_area = sa[i];
    if (tid == 0) {
      const unsigned ai = 0xFFFFFFFFu - (unsigned)(k[i] & 0xFFFFFFFFull);
      const float4 bx = a.boxes[ib + ai];
      float* r = out + (size_t)kept * rowlen;
      r[0] = fminf(fmaxf(bx.x, 0.f), a.img_w);
      r[1] = fminf(fmaxf(bx.y, 0.f), a.img_h);
      r[2] = fminf(fmaxf(bx.z, 0.f), a.img_w);
      r[3] = fminf(fmaxf(bx.w, 0.f), a.img_h);
      r[4] = a.scores[ib + ai];
      r[5] = (float)a.cls[ib + ai];
      for (int m = 0; m < a.nm; ++m) r[6 + m] = a.anchors[(ib + ai) * a.no_tot + a.mask_off + m];
    }
    ++kept;
    for (int j = i + 1 + tid; j < n; j += NMS_T) {
      if (sup[j]) continue;
      const float4 bj = sb[j];
      const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
      const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
      const float w = fmaxf(0.0f, __fsub_rn(xx2, xx1));
      const float h = fmaxf(0.0f, __fsub_rn(yy2, yy1));
      const float inter = __fmul_rn(w, h);
      const float ovr = __fdiv_rn(inter, __fsub_rn(__fadd_rn(ai_area, sa[j]), inter));
      if ((double)ovr > a.iou) sup[j] = 1;
    }
    __syncthreads();
  }
  if (tid == 0) a.out_counts[b] = kept;
}

}  // namespace

// ------------------------------------------------------------------------------------------------- launchers
hipError_t ym_launch_prep(int dtype, const PrepArgs& a, int* counts, int B, hipStream_t st) {
  hipLaunchKernelGGL(init_ctl, dim3(1), dim3(64), 0, st, a.ctl, counts, B);
  const long n = (long)a.B * a.C * a.H * a.W;
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(max_reduce, dim3(blocks), dim3(256), 0, st, a.in, n, a.ctl);
  const long np = (long)a.B * a.H * a.W;
  if (dtype == YM_DT_F16)
    hipLaunchKernelGGL(prep_nhwc<f16>, dim3((np + 255) / 256), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(prep_nhwc<float>, dim3((np + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_dwconv(int dtype, const DwArgs& a, hipStream_t st) {
  const long total = (long)a.B * a.H * a.W * (a.C / 8);
  const dim3 g((total + 255) / 256);
  if (dtype == YM_DT_F16) hipLaunchKernelGGL(dwconv3x3<f16>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(dwconv3x3<float>, g, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_sppf(int dtype, const PoolArgs& a, hipStream_t st) {
  const long total = (long)a.B * a.H * a.W * (a.C / 8);
  const dim3 g((total + 255) / 256);
  if (dtype == YM_DT_F16) hipLaunchKernelGGL(sppf_pool<f16>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(sppf_pool<float>, g, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_attn(int dtype, const AttnArgs& a, hipStream_t st) {
  if (a.kd > AKD || a.hd > AHD) return hipErrorInvalidValue;
  const int nqb = (a.N + AQ - 1) / AQ;
  const dim3 g(a.B * a.nh * nqb);
  if (dtype == YM_DT_F16) hipLaunchKernelGGL(attn_psa<f16>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_psa<float>, g, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_decode(const DecodeArgs& a, hipStream_t st) {
  const long total = (long)a.B * a.A;
  hipLaunchKernelGGL(decode_anchors, dim3((total + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t ym_launch_nms(const NmsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(nms_image, dim3(a.B), dim3(NMS_T), 0, st, a);
  return hipGetLastError();
}
