// tr_common.h — shared device helpers for the gfx950 CP tensor-regression kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TR_WAVE 64
#define TR_MAXF 8     // max factors (modes of the dense coefficient tensor)
#define TR_MAXR 1024  // max CP rank (MTTKRP tiles ranks by 64; the reference has no limit)
// stop-flag value written by k_update when the pass it was about to apply failed on the device
// (gradient-arena status slot set): TR_STOP_DEVICE_ERROR - iteration.  Distinct from the plateau
// stop (iterations completed, > 0) and the spectral NaN stop (-(iterations run) > -2^30).
#define TR_STOP_DEVICE_ERROR (-(1 << 30))

// Description of the dense coefficient tensor B and its Kruskal factors, passed by value.
//
// Factors are listed in the REFERENCE's list order (standard: A_1..A_K; multinomial:
// A_1..A_K, A_C).  B's value at factor indices (i_0..i_{F-1}) is
//     sum_r w_r * prod_f Phi_f[i_f, r]
// with the reference's association order (cp_to_tensor: (Phi_0 * w) @ KR(Phi_1..)^T,
// KR folded left).  `stride[f]` gives where that element lives in OUR dense buffer:
// row-major over the feature modes, and for the multinomial class factor the slowest
// (class-major, Bt[c][p]) so every class column is a contiguous P-vector.
struct FactorSet {
  int nf;                    // number of factors F
  int rank;                  // R
  int64_t dim[TR_MAXF];      // I_f (rows of factor f)
  int64_t off[TR_MAXF];      // offset of factor f in the parameter / phi arenas
  int64_t stride[TR_MAXF];   // dense-buffer stride of index i_f
  int64_t rstride[TR_MAXF];  // stride of i_f in the reference's row-major enumeration
  int nonneg[TR_MAXF];       // softplus applied to this factor
  int64_t total;             // prod_f I_f
  int64_t nfelem;            // sum_f I_f * R
  int8_t others[TR_MAXF][TR_MAXF];  // for each f: the other factors, by decreasing dense stride
};

// torch.nn.functional.softplus(x, beta, threshold) and its derivative
// (ATen softplus / softplus_backward CPU kernels).
__device__ __forceinline__ float tr_softplus(float a, float beta, float thr) {
  const float ab = a * beta;
  return ab > thr ? a : log1pf(expf(ab)) / beta;
}
__device__ __forceinline__ float tr_softplus_grad(float a, float beta, float thr) {
  const float ab = a * beta;
  if (ab > thr) return 1.0f;
  const float z = expf(ab);
  return z / (z + 1.0f);
}

// All-reduce across the 64 lanes of a wave without address VGPRs: ds_swizzle xor-butterfly
// inside each 32-lane half (bit-mask mode, offset = xor<<10 | and 0x1F), then the two half
// sums through readlane.  Commutativity of IEEE addition makes every lane of a half hold the
// bitwise-identical value, so the result is the same scalar in every lane (deterministic).
template <int PATTERN>
__device__ __forceinline__ float tr_swz_xor(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), PATTERN));
}
__device__ __forceinline__ float tr_wave_allreduce(float v) {
  v += tr_swz_xor<0x401F>(v);  // xor 16
  v += tr_swz_xor<0x201F>(v);  // xor 8
  v += tr_swz_xor<0x101F>(v);  // xor 4
  v += tr_swz_xor<0x081F>(v);  // xor 2
  v += tr_swz_xor<0x041F>(v);  // xor 1
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  return a + b;
}
__device__ __forceinline__ float tr_wave_allreduce_max(float v) {
  v = fmaxf(v, tr_swz_xor<0x401F>(v));
  v = fmaxf(v, tr_swz_xor<0x201F>(v));
  v = fmaxf(v, tr_swz_xor<0x101F>(v));
  v = fmaxf(v, tr_swz_xor<0x081F>(v));
  v = fmaxf(v, tr_swz_xor<0x041F>(v));
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  return fmaxf(a, b);
}
__device__ __forceinline__ double tr_wave_allreduce_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float tr_dot4(const float4 a, const float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  acc = fmaf(a.w, b.w, acc);
  return acc;
}
__device__ __forceinline__ void tr_axpy4(float s, const float4 x, float4& acc) {
  acc.x = fmaf(s, x.x, acc.x);
  acc.y = fmaf(s, x.y, acc.y);
  acc.z = fmaf(s, x.z, acc.z);
  acc.w = fmaf(s, x.w, acc.w);
}

// Non-temporal 16-B load for the once-per-pass X stream (X >> 256 MiB Infinity Cache).
typedef float tr_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 tr_ld_stream(const float4* p) {
  const tr_f4 v = __builtin_nontemporal_load(reinterpret_cast<const tr_f4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// HIP loads every translation unit's code object (one per .hip file of the library) on the first
// use of any of its kernels: loading tr_kernels.hip's took 10.5 ms inside the first fit's first
// iteration on the GPU box.  Each file defines one touch function; tr_api.hip calls them all once
// per device when a plan is created.
namespace tr {
hipError_t touch_code_object_kernels();
hipError_t touch_code_object_update();
hipError_t touch_code_object_cluster();
hipError_t touch_code_object_spectral();
hipError_t touch_code_object_spectral_slice();
hipError_t touch_code_object_spectral_gen();
hipError_t touch_code_object_mnl();
hipError_t touch_code_object_mnl_duo();
hipError_t touch_code_object_fp64();
}  // namespace tr
