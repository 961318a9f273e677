// Issue cost of the VALU instructions the exact bf16x3 split is made of (tools/, not product):
// cycles per wave-instruction for 64 independent instructions per loop trip (8 registers x 8),
// with one wave per SIMD (256-thread blocks) and two waves per SIMD (512-thread blocks), alone
// and between v_mfma_f32_16x16x32_bf16 (one MFMA per 4 / 8 VALU).  One block per CU.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/_valu_rate && ./tools/_valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

#define R8(OP)                                                                                       \
  asm volatile(OP " %0, %8, %0\n\t" OP " %1, %8, %1\n\t" OP " %2, %8, %2\n\t" OP " %3, %8, %3\n\t"    \
               OP " %4, %8, %4\n\t" OP " %5, %8, %5\n\t" OP " %6, %8, %6\n\t" OP " %7, %8, %7"        \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)       \
               : "v"(k))
#define R8_3(OP)                                                                                      \
  asm volatile(OP " %0, %8, %0, %9\n\t" OP " %1, %8, %1, %9\n\t" OP " %2, %8, %2, %9\n\t"            \
               OP " %3, %8, %3, %9\n\t" OP " %4, %8, %4, %9\n\t" OP " %5, %8, %5, %9\n\t"            \
               OP " %6, %8, %6, %9\n\t" OP " %7, %8, %7, %9"                                          \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)       \
               : "v"(k), "v"(k2))

template <int OP, int MF>
__global__ __launch_bounds__(512) void kv(unsigned* out, long long* cyc, int iters) {
  unsigned r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6,
           r7 = r0 + 7;
  const unsigned k = 0x3f800000u ^ threadIdx.x, k2 = 0x07060302u;
  f4 c = {0, 0, 0, 0};
  u4 a = {r0, r1, r2, r3}, b = {r4, r5, r6, r7};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int m = 0; m < MF; ++m)  // MF MFMAs per 8 VALU
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0, 0);
      if (OP == 0) R8("v_and_b32");
      if (OP == 1) R8("v_sub_f32");
      if (OP == 2) R8_3("v_perm_b32");
      if (OP == 3) R8("v_cvt_pk_bf16_f32");
      if (OP == 4) R8("v_lshlrev_b32");
      if (OP == 5) R8_3("v_bfi_b32");
      if (OP == 6) R8("v_add_u32");
      if (OP == 7) R8_3("v_fma_f32");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7 + (unsigned)c[0];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP, int MF>
void run(const char* name, unsigned* o, long long* cy, int threads) {
  const int iters = 2048;
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((kv<OP, MF>), dim3(256), dim3(threads), 0, 0, o, cy, iters);
  long long h[256];
  (void)hipMemcpy(h, cy, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  m /= 256.0 * iters;
  printf("%-20s MFMAs per 8 VALU %d  waves/SIMD %d: %7.1f cycles per trip (64 VALU%s) = %5.2f per VALU\n", name, MF,
         threads / 256, m, MF ? " + MFMAs" : "", m / 64);
}
#define ALL(OP, NAME)                 \
  run<OP, 0>(NAME, o, cy, 256);       \
  run<OP, 0>(NAME, o, cy, 512);       \
  run<OP, 1>(NAME, o, cy, 256);       \
  run<OP, 1>(NAME, o, cy, 512);       \
  run<OP, 2>(NAME, o, cy, 256);       \
  run<OP, 2>(NAME, o, cy, 512);
int main() {
  unsigned* o;
  long long* cy;
  (void)hipMalloc(&o, 256 * 512 * 4);
  (void)hipMalloc(&cy, 256 * 8);
  ALL(0, "v_and_b32")
  ALL(1, "v_sub_f32")
  ALL(2, "v_perm_b32")
  ALL(3, "v_cvt_pk_bf16_f32")
  ALL(4, "v_lshlrev_b32")
  ALL(5, "v_bfi_b32")
  ALL(6, "v_add_u32")
  ALL(7, "v_fma_f32")
  return 0;
}
