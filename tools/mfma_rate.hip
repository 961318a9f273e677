// Issue-rate probe of the f32 MFMA forms on gfx950 (tools/, not product): one wave per SIMD,
// 8 independent accumulators, back-to-back; prints cycles per instruction (s_memtime ticks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int KIND>
__global__ void k(float* out, long long* cyc, int iters) {
  f4 c[8];
  for (int i = 0; i < 8; ++i) c[i] = f4{0.f, 0.f, 0.f, 0.f};
  const float a = 1.0f + threadIdx.x * 1e-3f, b = 0.5f;
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (KIND == 0) c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
      else c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float* o;
  long long* cy;
  (void)hipMalloc(&o, 1 << 20);
  (void)hipMalloc(&cy, 1 << 12);
  const int iters = 4096;
  for (int kind = 0; kind < 2; ++kind) {
    for (int wps = 1; wps <= 2; ++wps) {  // waves per SIMD: block of 256 or 512 threads, 1 block per CU
      const int threads = 256 * wps;
      for (int rep = 0; rep < 2; ++rep) {
        if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(threads), 0, 0, o, cy, iters);
        else hipLaunchKernelGGL(k<1>, dim3(256), dim3(threads), 0, 0, o, cy, iters);
      }
      long long h = 0;
      (void)hipMemcpy(&h, cy, 8, hipMemcpyDeviceToHost);
      printf("%s waves/SIMD=%d: %.2f cycles per MFMA per wave (%.2f per SIMD)\n",
             kind == 0 ? "v_mfma_f32_4x4x1_16b_f32" : "v_mfma_f32_16x16x4_f32", wps,
             (double)h / (iters * 8.0), (double)h / (iters * 8.0 * wps));
    }
  }
  return 0;
}
