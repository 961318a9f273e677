// LDS-DMA issue-cost probe 2 (tools/, not product): how long does a global_load_lds_dwordx4
// block the issuing wave, as a function of the number of issuing waves per CU and of the spacing
// between a wave's DMA instructions (VALU filler between them)?  Every CU streams its own
// region of a 4 GiB buffer; prints per-instruction issue cycles (wave view) and chip TB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}
__device__ __forceinline__ void dma16(const float* g, const float* l) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
               : "memory");
}

// each wave: `total` DMA instructions into a 16-slot ring of its own (1 KiB each), `gap` dependent
// VALU ops between consecutive instructions, at most `depth` outstanding (vmcnt wait)
__global__ __launch_bounds__(512) void k_issue(const float* src, long long* cyc, int total, int gap, int depth,
                                               int64_t span, float* sink) {
  extern __shared__ __attribute__((aligned(16))) float s[];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* mine = s + wv * 256 * 16;
  const float* g = src + ((int64_t)blockIdx.x * (blockDim.x / 64) + wv) * span;
  long long issue = 0;
  float acc = (float)l;
  const long long t0 = __builtin_readcyclecounter();
  for (int q = 0; q < total; ++q) {
    for (int k = 0; k < gap; ++k) acc = fmaf(acc, 1.0000001f, 0.5f);
    if (q >= depth) {
      if (depth == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (depth == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    }
    const long long a = __builtin_readcyclecounter();
    dma16(g + ((int64_t)q * 256) % span + 4 * l + 1, mine + (q & 15) * 256);
    issue += __builtin_readcyclecounter() - a;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t1 = __builtin_readcyclecounter();
  if (l == 0) {
    cyc[2 * (blockIdx.x * 8 + wv)] = issue;
    cyc[2 * (blockIdx.x * 8 + wv) + 1] = t1 - t0;
  }
  if (acc == 12345.f) sink[0] = acc;
}

int main() {
  const int64_t span = 1 << 19;  // floats per wave
  const size_t bytes = (size_t)256 * 8 * span * 4;
  float *big, *sink;
  long long* cy;
  if (hipMalloc(&big, bytes) != hipSuccess) return 1;
  (void)hipMemset(big, 0, bytes);
  (void)hipMalloc(&cy, 256 * 8 * 2 * 8);
  (void)hipMalloc(&sink, 64);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_issue), hipFuncAttributeMaxDynamicSharedMemorySize,
                            8 * 256 * 16 * 4);
  const int total = 256;
  for (int waves : {1, 2, 4, 8})
    for (int depth : {4, 8, 16})
      for (int gap : {0, 64, 256}) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        for (int rep = 0; rep < 2; ++rep) {
          (void)hipEventRecord(e0);
          hipLaunchKernelGGL(k_issue, dim3(256), dim3(64 * waves), waves * 256 * 16 * 4, 0, big, cy, total, gap, depth,
                             span, sink);
          (void)hipEventRecord(e1);
          (void)hipEventSynchronize(e1);
        }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> c(256 * 8 * 2, 0);
        (void)hipMemcpy(c.data(), cy, c.size() * 8, hipMemcpyDeviceToHost);
        double iss = 0, tot = 0;
        int nw = 0;
        for (int b = 0; b < 256; ++b)
          for (int w = 0; w < waves; ++w) {
            iss += c[2 * (b * 8 + w)];
            tot += c[2 * (b * 8 + w) + 1];
            ++nw;
          }
        const double moved = 256.0 * waves * total * 1024;
        printf("waves/CU %d depth %2d gap %3d: issue %6.1f cyc/instr, total %6.1f cyc/instr/wave, %.2f TB/s\n", waves,
               depth, gap, iss / nw / total, tot / nw / total, moved / (ms * 1e-3) / 1e12);
      }
  return 0;
}
