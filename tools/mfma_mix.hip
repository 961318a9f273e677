// Issue-rate probe of MFMA instruction MIXES on gfx950 (tools/, not product): one wave per SIMD
// (256-thread blocks, one per CU), the patterns of the spectral 4-wave kernel's inner loops, each
// instruction fenced in program order; prints cycles per pattern repetition.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
#define F() __builtin_amdgcn_sched_barrier(0)
#define M16(c, a, b) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0)
#define M4(c, a, b) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0)
template <int P>
__global__ __launch_bounds__(512) void k(float* out, long long* cyc, int iters) {
  __shared__ float lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = i * 1e-3f;
  __syncthreads();
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0;
  float a = 1.0f + threadIdx.x * 1e-3f, b = 0.5f;
  float x0 = a, x1 = b, x2 = a * b, x3 = a + b;
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
    if (P == 0) {  // 16x16x4, two accumulators alternating
      M16(c0, a, b); F(); M16(c1, a, b); F();
    } else if (P == 1) {  // 16x16x4, one dependent chain
      M16(c0, a, b); F(); M16(c0, a, b); F();
    } else if (P == 2) {  // 4x4x1, four accumulators
      M4(c0, a, b); F(); M4(c1, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F();
    } else if (P == 3) {  // forward step: 16x16 T0, 4x4 x2, 16x16 T1, 4x4 x2
      M16(c0, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F(); M16(c1, a, b); F(); M4(c4, a, b); F(); M4(c5, a, b); F();
    } else if (P == 4) {  // backward: one 16x16 chain with 4x4 x2 between
      M16(c0, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F(); M16(c0, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F();
    } else if (P == 5) {  // forward step + its two ds_read_b64
      const float2 v = *reinterpret_cast<const float2*>(lds + ((threadIdx.x * 2 + it * 64) & 4095));
      const float2 w = *reinterpret_cast<const float2*>(lds + ((threadIdx.x * 2 + it * 32 + 7) & 4094));
      x0 += v.x; x1 += w.y;
      M16(c0, x0, b); F(); M4(c2, x1, b); F(); M4(c3, x0, b); F(); M16(c1, x1, b); F(); M4(c4, x0, b); F(); M4(c5, x1, b); F();
    } else if (P == 6) {  // 4x4x1, two accumulators
      M4(c0, a, b); F(); M4(c1, a, b); F();
    } else if (P == 8) {  // octo backward v: gacc, lin x4 (2 acc), gacc, lin x4
      M16(c0, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F();
      M16(c0, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F(); M4(c2, a, b); F(); M4(c3, a, b); F();
    } else if (P == 7) {  // 4x4x1, one chain
      M4(c0, a, b); F(); M4(c0, a, b); F();
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  f4 s = c0 + c1 + c2 + c3 + c4 + c5;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3] + x0 + x1 + x2 + x3;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int P>
void run(const char* name, float* o, long long* cy, int threads = 256) {
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k<P>, dim3(256), dim3(threads), 0, 0, o, cy, iters);
  long long h[256];
  (void)hipMemcpy(h, cy, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  printf("%-58s %8.1f cycles per repetition\n", name, m / 256 / iters);
}
int main() {
  float* o;
  long long* cy;
  (void)hipMalloc(&o, 1 << 20);
  (void)hipMalloc(&cy, 1 << 12);
  run<0>("16x16x4 x2, two accumulators", o, cy);
  run<1>("16x16x4 x2, one dependent chain", o, cy);
  run<2>("4x4x1 x4, four accumulators", o, cy);
  run<6>("4x4x1 x2, two accumulators", o, cy);
  run<7>("4x4x1 x2, one chain", o, cy);
  run<3>("fwd step: 16x16, 4x4, 4x4, 16x16, 4x4, 4x4 (6 acc)", o, cy);
  run<4>("bwd: 16x16 chain with 4x4 x2 between (x2)", o, cy);
  run<5>("fwd step + two ds_read_b64", o, cy);
  printf("two waves per SIMD (512-thread blocks): cycles per repetition per wave\n");
  run<0>("16x16x4 x2, two accumulators", o, cy, 512);
  run<2>("4x4x1 x4, four accumulators", o, cy, 512);
  run<3>("fwd step: 16x16, 4x4, 4x4, 16x16, 4x4, 4x4 (6 acc)", o, cy, 512);
  run<4>("bwd: 16x16 chain with 4x4 x2 between (x2)", o, cy, 512);
  run<1>("16x16x4 x2, one dependent chain", o, cy, 512);
  run<8>("bwd octo: 16x16 x2 chain + 4x4 x8 (2 acc)", o, cy, 512);
  run<8>("bwd octo: 16x16 x2 chain + 4x4 x8 (2 acc), 1 wave/SIMD", o, cy, 256);
  return 0;
}
