// hbm_probe.hip — measure the achievable streaming-read bandwidth on this MI355X, to calibrate
// the roofline of the X-streaming kernels (a known-good reference on the same hardware,
// cdna_hip_programming.md §5.4 rule 10).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip && tools/hbm_probe [GiB]
//
// Variants: grid-stride float4 reads (plain / nontemporal) at several grid sizes, and a
// row-streaming variant shaped like k_linear_fused (one workgroup per CU, buffer loads).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));          \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int NT, int U>
__global__ __launch_bounds__(256) void read_gs(const float4* __restrict__ p, size_t n4, float* out) {
  float acc = 0.f;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p + i + u * stride));
        v[u] = make_float4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = p[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  for (; i < n4; i += stride) {
    const float4 v = p[i];
    acc += (v.x + v.y) + (v.z + v.w);
  }
  if (acc == 12345.678f) out[0] = acc;  // keep the loads alive
}

// one workgroup streams a contiguous block of rows of `row4` float4 each (like k_linear_fused)
template <int T, int CH, int AUX>
__global__ __launch_bounds__(T) void read_rows(const float* __restrict__ X, size_t nrows, size_t rows_per_wg,
                                               int row_bytes, float* out) {
  const size_t r0 = blockIdx.x * rows_per_wg;
  size_t r1 = r0 + rows_per_wg;
  if (r1 > nrows) r1 = nrows;
  float acc = 0.f;
  for (size_t r = r0; r < r1; ++r) {
    const char* base = reinterpret_cast<const char*>(X) + r * (size_t)row_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, row_bytes, 0x00020000);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16, c * T * 16, AUX));
      acc += (v.x + v.y) + (v.z + v.w);
    }
  }
  if (acc == 12345.678f) out[0] = acc;
}

template <typename F>
static double time_ms(F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? std::atof(argv[1]) : 8.0;
  const size_t bytes = (size_t)(gib * 1024 * 1024 * 1024) / 131072 * 131072;
  float* X = nullptr;
  float* out = nullptr;
  CHECK(hipMalloc(&X, bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(X, 0x3c, bytes));
  const size_t n4 = bytes / 16;
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("buffer %.2f GB, %d CUs\n", bytes / 1e9, ncu);
  const int reps = 10;
  for (int wpc : {4, 8, 16, 32}) {
    const int grid = ncu * wpc;
    double ms = time_ms([&] { hipLaunchKernelGGL((read_gs<0, 8>), dim3(grid), dim3(256), 0, 0, (const float4*)X, n4, out); }, reps);
    std::printf("grid-stride plain  U=8 WG/CU=%2d: %.3f ms  %.1f GB/s\n", wpc, ms, bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((read_gs<1, 8>), dim3(grid), dim3(256), 0, 0, (const float4*)X, n4, out); }, reps);
    std::printf("grid-stride nt     U=8 WG/CU=%2d: %.3f ms  %.1f GB/s\n", wpc, ms, bytes / ms / 1e6);
  }
  const int row_bytes = 131072;  // 32768 floats (config 2 row)
  const size_t nrows = bytes / row_bytes;
  {
    const size_t rpw = (nrows + ncu - 1) / ncu;
    double ms = time_ms([&] { hipLaunchKernelGGL((read_rows<512, 16, 0>), dim3(ncu), dim3(512), 0, 0, X, nrows, rpw, row_bytes, out); }, reps);
    std::printf("rows T=512 CH=16 aux=0, 1 WG/CU : %.3f ms  %.1f GB/s\n", ms, bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((read_rows<512, 16, 2>), dim3(ncu), dim3(512), 0, 0, X, nrows, rpw, row_bytes, out); }, reps);
    std::printf("rows T=512 CH=16 aux=2, 1 WG/CU : %.3f ms  %.1f GB/s\n", ms, bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((read_rows<1024, 8, 0>), dim3(ncu), dim3(1024), 0, 0, X, nrows, rpw, row_bytes, out); }, reps);
    std::printf("rows T=1024 CH=8 aux=0, 1 WG/CU : %.3f ms  %.1f GB/s\n", ms, bytes / ms / 1e6);
    const size_t rpw2 = (nrows + 2 * ncu - 1) / (2 * ncu);
    ms = time_ms([&] { hipLaunchKernelGGL((read_rows<512, 16, 0>), dim3(2 * ncu), dim3(512), 0, 0, X, nrows, rpw2, row_bytes, out); }, reps);
    std::printf("rows T=512 CH=16 aux=0, 2 WG/CU : %.3f ms  %.1f GB/s\n", ms, bytes / ms / 1e6);
  }
  CHECK(hipFree(X));
  CHECK(hipFree(out));
  return 0;
}
