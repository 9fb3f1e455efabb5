// Probe of the fp8 MFMA accumulation on gfx950: what does v_mfma_f32_32x32x16_fp8_fp8 (and the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 with unit scales) compute for D = C + A·B, exactly?  The fp8 PTQ plan's convs
// differ from an exact (float64) restatement in ~0.1 % of the output codes (tests/test_gpu_fp8.py), more than fp32
// accumulation explains; tools/f8_mfma_model.py fits candidate rounding models to the data this writes.
//
//   hipcc --offload-arch=gfx950 -O2 tools/f8_mfma_probe.hip -o tools/ab/f8_mfma_probe
//   tools/ab/f8_mfma_probe out.bin [instances per distribution]
//
// Output: header (magic, n, nkinds, ndist), then per kind k (0: 32x32x16 fp8, 1: 32x32x64 f8f6f4 unit scales, 2: the
// e4m3 values on the 32x32x16 f16 MFMA) and
// instance: the 64 lanes' A bytes, B bytes (as fed: 8 or 32 per lane), C (32x32 fp32, row-major [row][col]) and D.
// Lane l feeds A[row l&31][k = KL*(l>>5) + j] and B[k = KL*(l>>5) + j][col l&31] (KL = 8 or 32 bytes per lane):
// the analysis re-checks that mapping against the data.  C/D: lane l, register i = row (i&3) + 8(i>>2) + 4(l>>5),
// column l&31.  One wave per instance, no LDS, no atomics.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void probe_f8(const uint8_t* A, const uint8_t* B, const float* C, float* D) {
  const int inst = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
  long a, b;
  memcpy(&a, A + ((size_t)inst * 64 + l) * 8, 8);
  memcpy(&b, B + ((size_t)inst * 64 + l) * 8, 8);
  v16f c;
  for (int i = 0; i < 16; ++i) c[i] = C[(size_t)inst * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  const v16f d = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) D[(size_t)inst * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = d[i];
}

__global__ void probe_f8s(const uint8_t* A, const uint8_t* B, const float* C, float* D, int scale) {
  const int inst = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
  v8i a, b;
  memcpy(&a, A + ((size_t)inst * 64 + l) * 32, 32);
  memcpy(&b, B + ((size_t)inst * 64 + l) * 32, 32);
  v16f c;
  for (int i = 0; i < 16; ++i) c[i] = C[(size_t)inst * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  // cbsz = blgp = 0: both operands e4m3; opsel 0; E8M0 block scales `scale` (127 = 2^0) for A and B
  const v16f d = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, scale, 0, scale);
  for (int i = 0; i < 16; ++i) D[(size_t)inst * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = d[i];
}

// kind 2: the same e4m3 values on the f16 MFMA (v_mfma_f32_32x32x16_f16), each converted exactly to fp16 scaled by 2^-8
// (fp16 bits = sign << 15 | (code & 0x7F) << 7: the e4m3 exponent and mantissa fields land in fp16's, subnormals
// included), so D = C + 2^-16 · sum of the products
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
__device__ inline h8 f8x8_to_h8(long v) {
  h8 r;
  for (int j = 0; j < 8; ++j) {
    const unsigned c = (unsigned)(v >> (8 * j)) & 0xFF;
    const unsigned short bits = (unsigned short)(((c & 0x80) << 8) | ((c & 0x7F) << 7));
    r[j] = __builtin_bit_cast(_Float16, bits);
  }
  return r;
}
__global__ void probe_f16(const uint8_t* A, const uint8_t* B, const float* C, float* D) {
  const int inst = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
  long a, b;
  memcpy(&a, A + ((size_t)inst * 64 + l) * 8, 8);
  memcpy(&b, B + ((size_t)inst * 64 + l) * 8, 8);
  v16f c;
  for (int i = 0; i < 16; ++i) c[i] = C[(size_t)inst * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  const v16f d = __builtin_amdgcn_mfma_f32_32x32x16_f16(f8x8_to_h8(a), f8x8_to_h8(b), c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) D[(size_t)inst * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = d[i];
}

static double e4m3(uint8_t c) {
  const int e = (c >> 3) & 15, m = c & 7;
  const double v = e == 0 ? std::ldexp((double)m, -9) : std::ldexp((double)(8 + m), e - 10);
  return (c & 0x80) ? -v : v;
}

// one random e4m3 code of distribution `dist`: 0 any finite code, 1 exponent spread over the whole range (incl.
// subnormals), 2 codes near 1 (small spread: carries and rounding inside one binade)
static uint8_t code(std::mt19937& g, int dist) {
  for (;;) {
    uint8_t c;
    if (dist == 2) c = (uint8_t)(0x30 + (g() % 32)) | (uint8_t)((g() & 1) << 7);  // |v| in [0.5, 2)
    else c = (uint8_t)(g() & 0xFF);
    if ((c & 0x7F) == 0x7F) continue;  // NaN
    if (dist == 0 && (c & 0x78) == 0) continue;  // no subnormals in the plain random set
    return c;
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s out.bin [n]\n", argv[0]);
    return 2;
  }
  const int n_per = argc > 2 ? atoi(argv[2]) : 128;
  const int ndist = 4;  // 0 random, 1 spread, 2 near one, 3 random with cancelling pairs
  const int n = n_per * ndist;
  FILE* f = fopen(argv[1], "wb");
  if (!f) return 1;
  const int hdr[4] = {0x38465059, n, 3, ndist};
  fwrite(hdr, 4, 4, f);
  std::mt19937 g(12345);
  for (int kind = 0; kind < 3; ++kind) {
    const int KL = kind == 1 ? 32 : 8;  // bytes per lane
    std::vector<uint8_t> A((size_t)n * 64 * KL), B((size_t)n * 64 * KL);
    std::vector<float> C((size_t)n * 1024), D((size_t)n * 1024);
    for (int inst = 0; inst < n; ++inst) {
      const int dist = inst / n_per;
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < KL; ++j) {
          A[((size_t)inst * 64 + l) * KL + j] = code(g, dist == 3 ? 0 : dist);
          B[((size_t)inst * 64 + l) * KL + j] = code(g, dist == 3 ? 0 : dist);
        }
      if (dist == 3)  // make the second half of each lane's K run cancel the first half's products approximately
        for (int l = 0; l < 64; ++l)
          for (int j = KL / 2; j < KL; ++j)
            if (g() & 1) {
              A[((size_t)inst * 64 + l) * KL + j] = A[((size_t)inst * 64 + l) * KL + j - KL / 2] ^ 0x80;
              B[((size_t)inst * 64 + l) * KL + j] = B[((size_t)inst * 64 + l) * KL + j - KL / 2];
            }
      for (int i = 0; i < 1024; ++i) {
        // C: zero for a third of the instances, else of the order of a product sum
        const int mode = inst % 3;
        C[(size_t)inst * 1024 + i] = mode == 0 ? 0.0f
                                               : (float)((double)(int)(g() % 2000001 - 1000000) * (mode == 1 ? 1e-6 : 1e-2));
      }
    }
    uint8_t *dA, *dB;
    float *dC, *dD;
    if (hipMalloc(&dA, A.size()) || hipMalloc(&dB, B.size()) || hipMalloc(&dC, C.size() * 4) ||
        hipMalloc(&dD, D.size() * 4))
      return 1;
    hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    if (kind == 0) hipLaunchKernelGGL(probe_f8, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD);
    else if (kind == 1) hipLaunchKernelGGL(probe_f8s, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD, 127);
    else hipLaunchKernelGGL(probe_f16, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD);
    if (hipDeviceSynchronize() != hipSuccess) {
      fprintf(stderr, "kernel failed\n");
      return 1;
    }
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    fwrite(A.data(), 1, A.size(), f);
    fwrite(B.data(), 1, B.size(), f);
    fwrite(C.data(), 4, C.size(), f);
    fwrite(D.data(), 4, D.size(), f);
    // quick self-check against the exact sum rounded once (the analysis does the full fit)
    long same = 0;
    for (int inst = 0; inst < n; ++inst)
      for (int row = 0; row < 32; ++row)
        for (int col = 0; col < 32; ++col) {
          double s = C[(size_t)inst * 1024 + row * 32 + col];
          const double sc = kind == 2 ? 1.0 / 65536.0 : 1.0;
          for (int k = 0; k < 2 * KL; ++k) {
            const int la = (k / KL) * 32 + row, lb = (k / KL) * 32 + col, j = k % KL;
            s += sc * e4m3(A[((size_t)inst * 64 + la) * KL + j]) * e4m3(B[((size_t)inst * 64 + lb) * KL + j]);
          }
          same += (float)s == D[(size_t)inst * 1024 + row * 32 + col];
        }
    printf("kind %d (K=%d): %.4f%% of outputs equal (float)(C + exact sum in double)\n", kind, 2 * KL,
           100.0 * same / ((double)n * 1024));
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
  }
  fclose(f);
  return 0;
}
