// Semantics probe of gfx950's v_permlane16_swap / v_permlane32_swap builtins as used for the x3 lane-pair stores:
// both called with the same register as vdst and vsrc; prints, per lane, which lane's value each result half holds.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/permlane_probe tools/permlane_probe.hip && /tmp/permlane_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(unsigned* o) {
  const unsigned x = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  o[4 * x] = r[0];
  o[4 * x + 1] = r[1];
  o[4 * x + 2] = q[0];
  o[4 * x + 3] = q[1];
}

int main() {
  unsigned* d = nullptr;
  if (hipMalloc(&d, 64 * 4 * sizeof(unsigned)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int ok16 = 1, ok32 = 1;
  for (int l = 0; l < 64; ++l) {
    const unsigned p16 = (l >> 4) & 1 ? h[4 * l] : h[4 * l + 1];   // partner value if the halves work as assumed
    const unsigned p32 = (l >> 5) & 1 ? h[4 * l + 2] : h[4 * l + 3];
    ok16 &= p16 == (unsigned)(l ^ 16);
    ok32 &= p32 == (unsigned)(l ^ 32);
    if (l % 8 == 0) printf("lane %2d: p16 {%2u %2u} p32 {%2u %2u}\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  }
  printf("permlane16_swap partner rule %s, permlane32_swap partner rule %s\n", ok16 ? "OK" : "WRONG", ok32 ? "OK" : "WRONG");
  (void)hipFree(d);
  return 0;
}
