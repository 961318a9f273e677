// LDS-DMA probe (tools/, not product): (1) does global_load_lds_dwordx4 accept a source that is
// 4-B but not 16-B aligned, and land the 16 bytes at m0 + 16 * lane?  (2) what does one LDS-DMA
// wave-instruction cost the issuing wave (dword vs dwordx4), with every CU streaming?
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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
__device__ __forceinline__ void dma4(const float* g, const float* l) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
               : "memory");
}

// (1) one wave: lane l fetches 16 B at src + off + 7 * l floats (row stride 7: scattered, 4-B aligned)
__global__ void k_align(const float* src, float* out, int off) {
  __shared__ __attribute__((aligned(16))) float s[256];
  const int l = threadIdx.x;
  s[l] = -1.f;
  s[l + 64] = -1.f;
  s[l + 128] = -1.f;
  s[l + 192] = -1.f;
  __syncthreads();
  dma16(src + off + 7 * l, s);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int e = l; e < 256; e += 64) out[e] = s[e];
}

// (2) issue cost: every wave issues `n` DMA instructions of its own 1 KiB (x4) / 256 B (x1)
// region per round, rounds of waits in between; cycles per instruction from the wave's view
template <int X4>
__global__ __launch_bounds__(512) void k_rate(const float* src, long long* cyc, int rounds, int n, int64_t span) {
  extern __shared__ __attribute__((aligned(16))) float s[];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* mine = s + wv * (X4 ? 256 * 16 : 64 * 16);
  const float* g = src + ((int64_t)blockIdx.x * 8 + wv) * span;
  long long issue = 0;
  const long long t0 = __builtin_readcyclecounter();
  for (int r = 0; r < rounds; ++r) {
    const long long a = __builtin_readcyclecounter();
    for (int q = 0; q < n; ++q) {
      const float* gp = g + ((int64_t)r * n + q) * (X4 ? 256 : 64) % span + (X4 ? 4 * l + 1 : l);
      if (X4)
        dma16(gp, mine + (q & 15) * 256);
      else
        dma4(gp, mine + (q & 15) * 64);
    }
    issue += __builtin_readcyclecounter() - a;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const long long t1 = __builtin_readcyclecounter();
  if (l == 0) {
    cyc[2 * (blockIdx.x * 8 + wv)] = issue;
    cyc[2 * (blockIdx.x * 8 + wv) + 1] = t1 - t0;
  }
}

int main() {
  const int NF = 1 << 20;
  std::vector<float> h(NF);
  for (int i = 0; i < NF; ++i) h[i] = (float)i;
  float *d, *o;
  (void)hipMalloc(&d, NF * 4);
  (void)hipMalloc(&o, 256 * 4);
  (void)hipMemcpy(d, h.data(), NF * 4, hipMemcpyHostToDevice);
  for (int off = 0; off < 4; ++off) {
    hipLaunchKernelGGL(k_align, dim3(1), dim3(64), 0, 0, d, o, off);
    std::vector<float> r(256);
    (void)hipMemcpy(r.data(), o, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 4; ++e)
        if (r[4 * l + e] != (float)(off + 7 * l + e)) ++bad;
    printf("dwordx4 LDS-DMA, source offset %d floats (%s-aligned): %s (%d wrong of 256)\n", off,
           off == 0 ? "16-B" : "4-B", bad ? "WRONG" : "exact", bad);
  }
  // rate: 256 CUs x 8 waves, each streaming its own region of a 2 GiB buffer
  const int64_t span = 1 << 18;  // floats per wave
  const size_t bytes = (size_t)256 * 8 * span * 4;
  float* big;
  long long* cy;
  if (hipMalloc(&big, bytes) != hipSuccess) return 1;
  (void)hipMemset(big, 0, bytes);
  (void)hipMalloc(&cy, 256 * 8 * 2 * 8);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rate<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            8 * 256 * 16 * 4);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rate<0>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            8 * 64 * 16 * 4);
  for (int x4 = 0; x4 < 2; ++x4) {
    for (int n : {8, 16, 32}) {
      const int rounds = 64;
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        if (x4)
          hipLaunchKernelGGL(k_rate<1>, dim3(256), dim3(512), 8 * 256 * 16 * 4, 0, big, cy, rounds, n, span);
        else
          hipLaunchKernelGGL(k_rate<0>, dim3(256), dim3(512), 8 * 64 * 16 * 4, 0, big, cy, rounds, n, span);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
      }
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      std::vector<long long> c(256 * 8 * 2);
      (void)hipMemcpy(c.data(), cy, c.size() * 8, hipMemcpyDeviceToHost);
      double iss = 0, tot = 0;
      for (int w = 0; w < 256 * 8; ++w) {
        iss += c[2 * w];
        tot += c[2 * w + 1];
      }
      iss /= 256 * 8;
      tot /= 256 * 8;
      const double moved = 256.0 * 8 * rounds * n * (x4 ? 1024 : 256);
      printf("%s  %2d instr/round: issue %.1f cyc/instr (wave view), %.2f TB/s chip, %.1f cyc/instr incl. wait\n",
             x4 ? "dwordx4" : "dword  ", n, iss / (rounds * n), moved / (ms * 1e-3) / 1e12, tot / (rounds * n));
    }
  }
  return 0;
}
