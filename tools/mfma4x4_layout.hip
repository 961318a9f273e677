// Probe of the v_mfma_f32_4x4x1_16b_f32 operand/accumulator layout on gfx950 (tools/, not product).
// Lane l supplies a = 1 + l (A operand) and b = 1000 * (1 + l) (B operand); prints, per lane,
// which (a-lane, b-lane) product each of the 4 accumulator registers holds.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out) {
  const int l = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(1 + l), 1000.f * (float)(1 + l), c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) out[l * 4 + v] = c[v];
}
int main() {
  float* d;
  (void)hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int ok = 1;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int v = 0; v < 4; ++v) {
      // value = (1+la)*1000*(1+lb); try the hypothesis la = 4*(l/4) + v, lb = l
      const float hyp = (float)(1 + 4 * (l / 4) + v) * 1000.f * (float)(1 + l);
      printf(" %g%s", h[l * 4 + v], h[l * 4 + v] == hyp ? "" : "(!)");
      if (h[l * 4 + v] != hyp) ok = 0;
    }
    printf("\n");
  }
  printf("hypothesis D[block=l/4][i=v][j=l%%4], A lane=4*block+i, B lane=4*block+j: %s\n", ok ? "HOLDS" : "FAILS");
  return 0;
}
