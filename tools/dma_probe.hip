// Stand-alone probe of one LDS-DMA conv launch (csrc/ym_conv_dma.hip built with YM_DMA_STAMPS): cycle stamps of
// workgroup 0 / wave 0 around the prologue, every K stage's wait and compute, and the epilogue; plus the event time
// of the launch.  Synthetic fp16 operands; NHWC input B x H x W x C, 3x3 (or 1x1) conv to N channels.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DYM_DMA_STAMPS tools/dma_probe.hip -o tools/dma_probe
//   ./tools/dma_probe B H W C N k cfg [stride]   (cfg = index into the DMA table; PROBE_X3=1: the x3 plan's pair
//   layout — operands of twice the fp16 elements, pair-layout output, cfg >= 30: the x3-only configurations)
#include "../yolo-infer_amd/csrc/ym_conv_dma.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));            \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8, H = argc > 2 ? atoi(argv[2]) : 20, W = argc > 3 ? atoi(argv[3]) : 20;
  const int C = argc > 4 ? atoi(argv[4]) : 128, N = argc > 5 ? atoi(argv[5]) : 128, k = argc > 6 ? atoi(argv[6]) : 3;
  const int cfg = argc > 7 ? atoi(argv[7]) : 0;
  const int S = argc > 8 ? atoi(argv[8]) : 1, CT = argc > 9 ? atoi(argv[9]) : C, Ho = (H + 2 * (k / 2) - k) / S + 1, Wo = (W + 2 * (k / 2) - k) / S + 1;
  const int x3 = getenv("PROBE_X3") ? atoi(getenv("PROBE_X3")) : 0, XS = x3 ? 2 : 1;
  const int K = k * k * C * XS, Kpad = (K + 63) / 64 * 64;  // storage K
  const size_t nin = (size_t)B * H * W * CT * XS, nout = (size_t)B * Ho * Wo * N * XS;
  std::vector<f16> hin(nin), hw((size_t)N * Kpad);
  for (size_t i = 0; i < nin; ++i) hin[i] = (f16)((int)(i * 2654435761u % 2001) * 0.001f - 1.f);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (f16)((int)(i * 40503u % 2001) * 0.0005f - 0.5f);
  f16 *din, *dw, *dout;
  float *dbias, *slab;
  int* cnt;
  unsigned long long* stamps;
  CK(hipMalloc(&din, nin * 2));
  CK(hipMalloc(&dw, hw.size() * 2));
  CK(hipMalloc(&dout, nout * 2));
  CK(hipMalloc(&dbias, N * 4));
  CK(hipMalloc(&slab, 64 << 20));
  CK(hipMalloc(&cnt, 65536 * 4));
  CK(hipMalloc(&stamps, 512 * 8));  // [0..3] phases, [8 + 4 it + p] stage it
  CK(hipMemset(dbias, 0, N * 4));
  CK(hipMemset(cnt, 0, 65536 * 4));
  CK(hipMemset(stamps, 0, 512 * 8));
  CK(hipMemcpy(din, hin.data(), nin * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
#ifdef YM_DMA_STAMPS
  CK(hipMemcpyToSymbol(HIP_SYMBOL(ym_dma_stamps), &stamps, sizeof(stamps)));
#endif
  ConvArgs a{};
  a.src0 = din; a.s0_ctot = CT; a.s0_coff = 0; a.C0 = C; a.s0_W = W; a.s0_P = H * W; a.up0 = 0;
  a.w = dw; a.bias = dbias;
  a.dst = dout; a.d_ctot = N; a.d_coff = 0; a.d_P = Ho * Wo; a.d_pixoff = 0; a.d_W = Wo;
  a.Hin = H; a.Win = W; a.Ho = Ho; a.Wo = Wo; a.k = k; a.s = S; a.pad = k / 2;
  a.Cin8 = XS * C / 8; a.Kc = K / 8; a.N = N; a.Kpad = Kpad; a.act = 1; a.npr = N; a.M = B * Ho * Wo;
  a.x3 = x3; a.wsc = a.wsc2 = 1.0f;
  a.s0_elems = (long)nin; a.s1_elems = 0;
  a.fd_hw = ym_fdiv(Ho * Wo); a.fd_w = ym_fdiv(Wo);
  a.slab = slab; a.slab_cap = 64 << 20; a.cnt = cnt; a.cnt_cap = 65536;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (int i = 0; i < 5; ++i) CK(ym_launch_conv_dma(0, a, cfg, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = getenv("PROBE_REPS") ? atoi(getenv("PROBE_REPS")) : 50;
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) CK(ym_launch_conv_dma(0, a, cfg, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> hs(512);
  CK(hipMemcpy(hs.data(), stamps, 512 * 8, hipMemcpyDeviceToHost));
  const int nk = Kpad / 64;
  constexpr DmaCfg kX3[] = {
#define YM_X(id, bm, bn, sp, kg, ns, sub) {bm, bn, sp, kg, ns, sub},
      YM_DMA_X3_CFGS(YM_X)
#undef YM_X
  };
  const DmaCfg dc = cfg < kNumDma ? kDma[cfg] : kX3[cfg - kNumDma];
  printf("B=%d %dx%d C=%d N=%d k=%d s=%d x3=%d cfg=%d (BM=%d BN=%d split=%d kg=%d ns=%d sub=%d): %d sub-stages, "
         "%.2f us/launch (stream, eager)\n", B, H, W, C, N, k, S, x3, cfg, dc.bm, dc.bn, dc.split, dc.kg, dc.ns, dc.sub,
         nk, ms * 1e3 / reps);
  const unsigned long long t0 = hs[0];
  printf("  prologue: index setup %llu cyc, first stages issued %llu cyc\n", hs[4] - t0, hs[1] - hs[4]);
  const int per = nk / dc.split / dc.sub;
  for (int it = 0; it < per && it < 64; ++it) {
    const unsigned long long* q = &hs[8 + 4 * it];
    const unsigned long long prev = it ? hs[8 + 4 * (it - 1) + 3] : hs[1];
    printf("  stage %3d at %6llu: wait %5lld  barrier %5lld  issue %5lld  compute %5lld\n", it, q[0] - t0,
           (long long)(q[0] - prev), (long long)(q[1] - q[0]), (long long)(q[2] - q[1]), (long long)(q[3] - q[2]));
  }
  printf("  loop end %llu, epilogue end %llu (epilogue %lld cyc: wave-group reduction %lld, split-K hand-off %lld, "
         "bias / act / stores %lld)\n", hs[2] - t0, hs[3] - t0, (long long)(hs[3] - hs[2]), (long long)(hs[5] - hs[2]),
         (long long)(hs[6] - hs[5]), (long long)(hs[3] - hs[6]));
  return 0;
}
