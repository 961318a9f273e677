// LDS-DMA issue-cost probe 3 (tools/, not product): is the ~220-cycle per-instruction issue cost
// of global_load_lds_dwordx4 (tools/ldsdma_probe2.hip, even with one wave per CU) tied to
// rewriting M0 between consecutive LDS-DMA instructions?  Variants, 16 instructions per burst:
//   0: m0 saved / set / s_nop / dma / restored around every instruction (the kernels' form)
//   1: m0 set once per burst, the LDS destinations advanced by the instruction offset (which
//      also offsets the global address: vaddr compensates)
//   2: m0 set before every instruction, no save / restore, no s_nop
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}

template <int V>
__global__ __launch_bounds__(512) void k_burst(const float* src, long long* cyc, int bursts, int64_t span) {
  extern __shared__ __attribute__((aligned(16))) float s[];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* mine = s + wv * 256 * 16;
  const float* g = src + ((int64_t)blockIdx.x * (blockDim.x / 64) + wv) * span;
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(mine));
  long long issue = 0;
  for (int b = 0; b < bursts; ++b) {
    const float* gb = g + ((int64_t)b * 16 * 256) % span + 4 * l + 1;
    const long long t0 = __builtin_readcyclecounter();
    if (V == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(gb + q * 256), "s"(base + q * 1024)
                     : "memory");
      }
    } else if (V == 1) {
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0" : "=&s"(keep) : "s"(base) : "memory");
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // offsets 0, 1024, 2048, 3072 (13-bit signed immediate)
        const float* p = gb + q * 4 * 256;
        asm volatile(
            "global_load_lds_dwordx4 %0, off nt\n\t"
            "global_load_lds_dwordx4 %0, off offset:1024 nt\n\t"
            "global_load_lds_dwordx4 %0, off offset:2048 nt\n\t"
            "global_load_lds_dwordx4 %0, off offset:3072 nt"
            :
            : "v"(p)
            : "memory");
        asm volatile("s_add_u32 m0, m0, 4096" ::: "memory");
      }
      asm volatile("s_mov_b32 m0, %0" ::"s"(keep) : "memory");
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" : : "v"(gb + q * 256), "s"(base + q * 1024)
                     : "memory", "m0");
    }
    issue += __builtin_readcyclecounter() - t0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (l == 0) cyc[blockIdx.x * 8 + wv] = issue;
}

int main() {
  const int64_t span = 1 << 19;
  const size_t bytes = (size_t)256 * 8 * span * 4;
  float* big;
  long long* cy;
  if (hipMalloc(&big, bytes) != hipSuccess) return 1;
  (void)hipMemset(big, 0, bytes);
  (void)hipMalloc(&cy, 256 * 8 * 8);
  const void* ks[3] = {reinterpret_cast<const void*>(&k_burst<0>), reinterpret_cast<const void*>(&k_burst<1>),
                       reinterpret_cast<const void*>(&k_burst<2>)};
  for (int v = 0; v < 3; ++v)
    (void)hipFuncSetAttribute(ks[v], hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 256 * 16 * 4);
  const int bursts = 32;
  for (int v = 0; v < 3; ++v)
    for (int waves : {1, 8}) {
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(k_burst<0>, dim3(256), dim3(64 * waves), waves * 65536, 0, big, cy, bursts, span);
        if (v == 1) hipLaunchKernelGGL(k_burst<1>, dim3(256), dim3(64 * waves), waves * 65536, 0, big, cy, bursts, span);
        if (v == 2) hipLaunchKernelGGL(k_burst<2>, dim3(256), dim3(64 * waves), waves * 65536, 0, big, cy, bursts, span);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
      }
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      std::vector<long long> c(256 * 8, 0);
      (void)hipMemcpy(c.data(), cy, c.size() * 8, hipMemcpyDeviceToHost);
      double iss = 0;
      for (int b = 0; b < 256; ++b)
        for (int w = 0; w < waves; ++w) iss += c[b * 8 + w];
      iss /= 256.0 * waves * bursts * 16;
      printf("variant %d waves/CU %d: issue %.1f cyc/instr, %.2f TB/s\n", v, waves, iss,
             256.0 * waves * bursts * 16 * 1024 / (ms * 1e-3) / 1e12);
    }
  return 0;
}
