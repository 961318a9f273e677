// update_bench.hip — layout study for the one-workgroup Adam step (k_update, tr_kernels.hip).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I tensor_regression_amd/csrc tools/update_bench.hip -o tools/_update_bench
//   rocprofv3 --kernel-trace --stats -d gpurun_out/ub -o ub -- tools/_update_bench
//
// The step is tiny (3-8 K parameters) but runs after a pass that streamed GBs through L2 and the
// Infinity Cache, so every global access is a cold HBM round trip; a 1 GiB memset between
// launches reproduces that.  Variants (all compute the same Adam step; v0 is the round-3 kernel):
//   v0  one element per loop iteration (round trip per iteration)
//   v2  U = 8 elements per thread loaded before use, fully unrolled
//   v3  float4 per thread per round, rolled loop
//   v4  float4, the first two rounds of all arrays loaded up front (params reused by the norms)
// Parameter counts: c2 3073 (2 factors), c3 1616 (3 factors), c5 8242 (6 factors + 2 bias).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tr_common.h"
#ifndef TR_UPD_PROFILE
#define TR_UPD_PROFILE 0
#endif
#include "tr_update.hip"  // the library kernel (v5)

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

namespace ub {


struct Args {
  float lam, omb1, b2, omb2, eps, step, bc2;
  int amsgrad;
};

__device__ __forceinline__ int factor_of(const FactorSet& fs, int64_t e) {
  int f = 0;
#pragma unroll
  for (int g = 1; g < TR_MAXF; ++g)
    if (g < fs.nf && e >= fs.off[g]) f = g;
  return f;
}

__device__ __forceinline__ void norms_finish(const FactorSet& fs, float (&accn)[TR_MAXF], float* wsum, float* norms) {
  const int t = threadIdx.x, lane = t & 63, q = t >> 6, NWV = blockDim.x >> 6;
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f)
    if (f < fs.nf) {
      const float v = tr_wave_allreduce(accn[f]);
      if (lane == 0) wsum[f * 16 + q] = v;
    }
  __syncthreads();
  if (t < fs.nf) {
    float tot = 0.f;
    for (int k = 0; k < NWV; ++k) tot += wsum[t * 16 + k];
    norms[t] = sqrtf(tot);
  }
  __syncthreads();
}

__device__ __forceinline__ void acc1(const FactorSet& fs, float (&accn)[TR_MAXF], int64_t k, float a) {
  const int f = factor_of(fs, k);
#pragma unroll
  for (int g = 0; g < TR_MAXF; ++g)
    if (g == f) accn[g] = fmaf(a, a, accn[g]);
}

__device__ __forceinline__ void step1(const FactorSet& fs, const Args& ua, const float* norms, int64_t e, float g,
                                      float p, float mm, float vv, float vmo, float* params, float* m, float* v,
                                      float* vmax) {
#pragma clang fp contract(off)
  if (e < fs.nfelem) {
    const int f = factor_of(fs, e);
    g = g + ua.lam / (2.0f * norms[f]) * (2.0f * p);
  }
  mm = fmaf(ua.omb1, g - mm, mm);
  vv = vv * ua.b2;
  vv = vv + ua.omb2 * g * g;
  float den = vv;
  if (ua.amsgrad) {
    den = fmaxf(vmo, vv);
    vmax[e] = den;
  }
  const float denom = sqrtf(den) / ua.bc2 + ua.eps;
  p = p + (-ua.step) * (mm / denom);
  m[e] = mm;
  v[e] = vv;
  params[e] = p;
}

__global__ __launch_bounds__(1024) void v0(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF];
  if (*stop != 0) return;
  if (grad[fs.nfelem + nb + 1] != 0.f) return;
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  for (int64_t k = threadIdx.x; k < fs.nfelem; k += blockDim.x) acc1(fs, accn, k, params[k]);
  norms_finish(fs, accn, wsum, norms);
  const int64_t np = fs.nfelem + nb;
  for (int64_t e = threadIdx.x; e < np; e += blockDim.x)
    step1(fs, ua, norms, e, grad[e], params[e], m[e], v[e], ua.amsgrad ? vmax[e] : 0.f, params, m, v, vmax);
}

__global__ __launch_bounds__(1024) void v2(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF];
  constexpr int U = 8;
  const int64_t B = blockDim.x, t = threadIdx.x, nfe = fs.nfelem, np = nfe + nb;
  const int32_t s0 = *stop;
  const float st = grad[nfe + nb + 1];
  float g0[U], p0[U], m0[U], v0_[U], vm0[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int64_t e = t + j * B;
    const bool in = e < np;
    p0[j] = in ? params[e] : 0.f;
    g0[j] = in ? grad[e] : 0.f;
    m0[j] = in ? m[e] : 0.f;
    v0_[j] = in ? v[e] : 0.f;
    vm0[j] = in && ua.amsgrad ? vmax[e] : 0.f;
  }
  if (s0 != 0 || st != 0.f) return;
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (t + j * B < nfe) acc1(fs, accn, t + j * B, p0[j]);
  for (int64_t k0 = t + U * B; k0 < nfe; k0 += U * B) {
    float a[U];
#pragma unroll
    for (int j = 0; j < U; ++j) a[j] = k0 + j * B < nfe ? params[k0 + j * B] : 0.f;
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (k0 + j * B < nfe) acc1(fs, accn, k0 + j * B, a[j]);
  }
  norms_finish(fs, accn, wsum, norms);
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (t + j * B < np) step1(fs, ua, norms, t + j * B, g0[j], p0[j], m0[j], v0_[j], vm0[j], params, m, v, vmax);
  for (int64_t e0 = t + U * B; e0 < np; e0 += U * B) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int64_t e = e0 + j * B;
      const bool in = e < np;
      p0[j] = in ? params[e] : 0.f;
      g0[j] = in ? grad[e] : 0.f;
      m0[j] = in ? m[e] : 0.f;
      v0_[j] = in ? v[e] : 0.f;
      vm0[j] = in && ua.amsgrad ? vmax[e] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (e0 + j * B < np) step1(fs, ua, norms, e0 + j * B, g0[j], p0[j], m0[j], v0_[j], vm0[j], params, m, v, vmax);
  }
}

// float4 rounds: thread t owns elements 4 * (t + r * B) .. +3 of round r
__device__ __forceinline__ float4 ld4(const float* p, int64_t e, int64_t n) {
  if (e + 4 <= n) return *reinterpret_cast<const float4*>(p + e);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n) r.x = p[e];
  if (e + 1 < n) r.y = p[e + 1];
  if (e + 2 < n) r.z = p[e + 2];
  return r;
}
__device__ __forceinline__ void acc4(const FactorSet& fs, float (&accn)[TR_MAXF], int64_t e, float4 a, int64_t nfe) {
  if (e < nfe) acc1(fs, accn, e, a.x);
  if (e + 1 < nfe) acc1(fs, accn, e + 1, a.y);
  if (e + 2 < nfe) acc1(fs, accn, e + 2, a.z);
  if (e + 3 < nfe) acc1(fs, accn, e + 3, a.w);
}
__device__ __forceinline__ void step4(const FactorSet& fs, const Args& ua, const float* norms, int64_t e, int64_t np,
                                      float4 g, float4 p, float4 mm, float4 vv, float4 vm, float* params, float* m,
                                      float* v, float* vmax) {
  const float* gg = &g.x;
  const float* pp = &p.x;
  const float* m4 = &mm.x;
  const float* v4 = &vv.x;
  const float* w4 = &vm.x;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (e + c < np) step1(fs, ua, norms, e + c, gg[c], pp[c], m4[c], v4[c], w4[c], params, m, v, vmax);
}

__global__ __launch_bounds__(1024) void v3(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF];
  const int64_t B4 = 4 * (int64_t)blockDim.x, nfe = fs.nfelem, np = nfe + nb;
  const int32_t s0 = *stop;
  const float st = grad[nfe + nb + 1];
  if (s0 != 0 || st != 0.f) return;
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  for (int64_t e = 4 * threadIdx.x; e < nfe; e += B4) acc4(fs, accn, e, ld4(params, e, nfe), nfe);
  norms_finish(fs, accn, wsum, norms);
  for (int64_t e = 4 * threadIdx.x; e < np; e += B4) {
    const float4 g = ld4(grad, e, np), p = ld4(params, e, np), mm = ld4(m, e, np), vv = ld4(v, e, np);
    const float4 vm = ua.amsgrad ? ld4(vmax, e, np) : make_float4(0.f, 0.f, 0.f, 0.f);
    step4(fs, ua, norms, e, np, g, p, mm, vv, vm, params, m, v, vmax);
  }
}

__global__ __launch_bounds__(1024) void v4(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF];
  const int64_t B4 = 4 * (int64_t)blockDim.x, nfe = fs.nfelem, np = nfe + nb;
  const int64_t e0 = 4 * threadIdx.x, e1 = e0 + B4;
  const int32_t s0 = *stop;
  const float st = grad[nfe + nb + 1];
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 p0 = ld4(params, e0, np), g0 = ld4(grad, e0, np), m0 = ld4(m, e0, np), w0 = ld4(v, e0, np);
  const float4 p1 = ld4(params, e1, np), g1 = ld4(grad, e1, np), m1 = ld4(m, e1, np), w1 = ld4(v, e1, np);
  const float4 x0 = ua.amsgrad ? ld4(vmax, e0, np) : z, x1 = ua.amsgrad ? ld4(vmax, e1, np) : z;
  if (s0 != 0 || st != 0.f) return;
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  acc4(fs, accn, e0, p0, nfe);
  acc4(fs, accn, e1, p1, nfe);
  for (int64_t e = e1 + B4; e < nfe; e += B4) acc4(fs, accn, e, ld4(params, e, nfe), nfe);
  norms_finish(fs, accn, wsum, norms);
  step4(fs, ua, norms, e0, np, g0, p0, m0, w0, x0, params, m, v, vmax);
  step4(fs, ua, norms, e1, np, g1, p1, m1, w1, x1, params, m, v, vmax);
  for (int64_t e = e1 + B4; e < np; e += B4) {
    const float4 g = ld4(grad, e, np), p = ld4(params, e, np), mm = ld4(m, e, np), vv = ld4(v, e, np);
    const float4 vm = ua.amsgrad ? ld4(vmax, e, np) : z;
    step4(fs, ua, norms, e, np, g, p, mm, vv, vm, params, m, v, vmax);
  }
}


// probes: launch floor, norm phase only, loads only
__global__ __launch_bounds__(1024) void pe(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  if (*stop != 0) params[0] = 1.f;
}
__global__ __launch_bounds__(1024) void pn(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF];
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  for (int64_t k = threadIdx.x; k < fs.nfelem; k += blockDim.x) acc1(fs, accn, k, params[k]);
  norms_finish(fs, accn, wsum, norms);
  if (threadIdx.x < fs.nf && *stop != 0) params[threadIdx.x] = norms[threadIdx.x];
}
__global__ __launch_bounds__(1024) void pl(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
  const int64_t np = fs.nfelem + nb;
  float s = 0.f;
  for (int64_t e = threadIdx.x; e < np; e += blockDim.x) s += grad[e] + params[e] + m[e] + v[e];
  if (*stop != 0) params[threadIdx.x] = s;
}
// full step with plain (no factor lookup) L2 term: isolates the per-element factor search
__global__ __launch_bounds__(1024) void pf(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
#pragma clang fp contract(off)
  const int64_t np = fs.nfelem + nb;
  for (int64_t e = threadIdx.x; e < np; e += blockDim.x) {
    float g = grad[e], p = params[e], mm = m[e], vv = v[e];
    g = g + ua.lam * p;
    mm = fmaf(ua.omb1, g - mm, mm);
    vv = vv * ua.b2 + ua.omb2 * g * g;
    p = p + (-ua.step) * (mm / (sqrtf(vv) / ua.bc2 + ua.eps));
    m[e] = mm;
    v[e] = vv;
    params[e] = p;
  }
}


// v6: v0's rolled loops (compact code: the step runs from a cold instruction cache) with the
// per-element branches removed: branch-free norm selection, L2 coefficient per factor from LDS
__global__ __launch_bounds__(1024) void v6(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
#pragma clang fp contract(off)
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF], coef[TR_MAXF];
  const int t = threadIdx.x, lane = t & 63, q = t >> 6, NWV = blockDim.x >> 6;
  const int32_t s0 = *stop;
  const float st = grad[fs.nfelem + nb + 1];
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  for (int64_t k = t; k < fs.nfelem; k += blockDim.x) {
    const float a = params[k];
    const int f = factor_of(fs, k);
#pragma unroll
    for (int g = 0; g < TR_MAXF; ++g) accn[g] = g == f ? fmaf(a, a, accn[g]) : accn[g];
  }
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f)
    if (f < fs.nf) {
      const float r = tr_wave_allreduce(accn[f]);
      if (lane == 0) wsum[f * 16 + q] = r;
    }
  __syncthreads();
  if (t < fs.nf) {
    float tot = 0.f;
    for (int k = 0; k < NWV; ++k) tot += wsum[t * 16 + k];
    norms[t] = sqrtf(tot);
    coef[t] = ua.lam / (2.0f * norms[t]);
  }
  __syncthreads();
  if (s0 != 0 || st != 0.f) return;
  const int64_t np = fs.nfelem + nb;
  for (int64_t e = threadIdx.x; e < np; e += blockDim.x) {
    float g = grad[e], p = params[e], mm = m[e], vv = v[e];
    const float vmo = ua.amsgrad ? vmax[e] : 0.f;
    const int f = factor_of(fs, e);
    g = e < fs.nfelem ? g + coef[f] * (2.0f * p) : g;
    mm = fmaf(ua.omb1, g - mm, mm);
    vv = vv * ua.b2;
    vv = vv + ua.omb2 * g * g;
    const float vm = fmaxf(vmo, vv);
    if (ua.amsgrad) vmax[e] = vm;
    const float denom = sqrtf(ua.amsgrad ? vm : vv) / ua.bc2 + ua.eps;
    p = p + (-ua.step) * (mm / denom);
    m[e] = mm;
    v[e] = vv;
    params[e] = p;
  }
}

// v7: v6 with two elements per trip (loads of both in flight)'s rolled loops (compact code: the step runs from a cold instruction cache) with the
// per-element branches removed: branch-free norm selection, L2 coefficient per factor from LDS
__global__ __launch_bounds__(1024) void v7(FactorSet fs, int nb, float* params, const float* grad, Args ua, float* m,
                                           float* v, float* vmax, int32_t* stop) {
#pragma clang fp contract(off)
  __shared__ float wsum[TR_MAXF * 16], norms[TR_MAXF], coef[TR_MAXF];
  const int t = threadIdx.x, lane = t & 63, q = t >> 6, NWV = blockDim.x >> 6;
  const int32_t s0 = *stop;
  const float st = grad[fs.nfelem + nb + 1];
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  const int64_t B = blockDim.x;
  int64_t k = t;
  for (; k + B < fs.nfelem; k += 2 * B) {
    const float a = params[k], b = params[k + B];
    const int f = factor_of(fs, k), h = factor_of(fs, k + B);
#pragma unroll
    for (int g = 0; g < TR_MAXF; ++g) accn[g] = g == f ? fmaf(a, a, accn[g]) : accn[g];
#pragma unroll
    for (int g = 0; g < TR_MAXF; ++g) accn[g] = g == h ? fmaf(b, b, accn[g]) : accn[g];
  }
  if (k < fs.nfelem) {
    const float a = params[k];
    const int f = factor_of(fs, k);
#pragma unroll
    for (int g = 0; g < TR_MAXF; ++g) accn[g] = g == f ? fmaf(a, a, accn[g]) : accn[g];
  }
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f)
    if (f < fs.nf) {
      const float r = tr_wave_allreduce(accn[f]);
      if (lane == 0) wsum[f * 16 + q] = r;
    }
  __syncthreads();
  if (t < fs.nf) {
    float tot = 0.f;
    for (int k = 0; k < NWV; ++k) tot += wsum[t * 16 + k];
    norms[t] = sqrtf(tot);
    coef[t] = ua.lam / (2.0f * norms[t]);
  }
  __syncthreads();
  if (s0 != 0 || st != 0.f) return;
  const int64_t np = fs.nfelem + nb;
  auto step = [&](int64_t e, float g, float p, float mm, float vv, float vmo) {
    const int f = factor_of(fs, e);
    g = e < fs.nfelem ? g + coef[f] * (2.0f * p) : g;
    mm = fmaf(ua.omb1, g - mm, mm);
    vv = vv * ua.b2;
    vv = vv + ua.omb2 * g * g;
    const float vm = fmaxf(vmo, vv);
    if (ua.amsgrad) vmax[e] = vm;
    const float denom = sqrtf(ua.amsgrad ? vm : vv) / ua.bc2 + ua.eps;
    p = p + (-ua.step) * (mm / denom);
    m[e] = mm;
    v[e] = vv;
    params[e] = p;
  };
  int64_t e = t;
  for (; e + B < np; e += 2 * B) {
    const float g0 = grad[e], g1 = grad[e + B], p0 = params[e], p1 = params[e + B];
    const float m0 = m[e], m1 = m[e + B], w0 = v[e], w1 = v[e + B];
    const float x0 = ua.amsgrad ? vmax[e] : 0.f, x1 = ua.amsgrad ? vmax[e + B] : 0.f;
    step(e, g0, p0, m0, w0, x0);
    step(e + B, g1, p1, m1, w1, x1);
  }
  if (e < np) step(e, grad[e], params[e], m[e], v[e], ua.amsgrad ? vmax[e] : 0.f);
}

// stand-in for the pass before the step: a streaming read of 4 GiB (L2, Infinity Cache and the
// address-translation caches all turn over, as after the real X pass)
__global__ __launch_bounds__(256) void stream_read(const float4* __restrict__ x, int64_t n4, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}
}  // namespace ub

int main() {
  struct Case { const char* name; std::vector<int64_t> rows; int rank; int nb; };
  const Case cases[] = {{"c2", {256, 128}, 8, 1}, {"c3", {128, 64, 10}, 8, 0},
                        {"c5", {256 * 1, 129, 2, 256 * 2, 129, 2}, 8, 2}};
  const size_t flush_bytes = size_t(4) << 30;
  void* flush = nullptr;
  CK(hipMalloc(&flush, flush_bytes));
  CK(hipMemset(flush, 0, flush_bytes));
  int32_t* stop = nullptr;
  CK(hipMalloc(&stop, 4));
  CK(hipMemset(stop, 0, 4));
  using KernT = void (*)(FactorSet, int, float*, const float*, ub::Args, float*, float*, float*, int32_t*);
  const KernT kerns[] = {ub::v0, ub::v2, ub::v3, ub::v4, ub::pe, ub::pn, ub::pl, ub::pf, ub::v6, ub::v7};
  const char* names[] = {"v0", "v2", "v3", "v4", "pe", "pn", "pl", "pf", "v6", "v7", "v5"};
  const int nk = 11;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (const Case& c : cases) {
    FactorSet fs{};
    fs.nf = (int)c.rows.size();
    fs.rank = c.rank;
    int64_t off = 0;
    for (int f = 0; f < fs.nf; ++f) {
      fs.dim[f] = c.rows[f];
      fs.off[f] = off;
      off += c.rows[f] * c.rank;
    }
    fs.nfelem = off;
    const int64_t np = off + c.nb, ng = np + 2;
    std::vector<float> h(ng);
    for (int64_t i = 0; i < ng; ++i) h[i] = 0.01f * (float)((i * 7919) % 201 - 100);
    h[np + 1] = 0.f;  // status slot
    float *params, *grad, *m, *v, *vmax;
    CK(hipMalloc(&params, ng * 4));
    CK(hipMalloc(&grad, ng * 4));
    CK(hipMalloc(&m, ng * 4));
    CK(hipMalloc(&v, ng * 4));
    CK(hipMalloc(&vmax, ng * 4));
    ub::Args ua{0.01f, 0.1f, 0.999f, 0.001f, 1e-8f, 0.01f, 0.03f, 0};
    for (int amsgrad = 0; amsgrad < 1; ++amsgrad) {
      ua.amsgrad = amsgrad;
      for (int kv = 0; kv < nk; ++kv) {
        CK(hipMemcpy(params, h.data(), ng * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(grad, h.data(), ng * 4, hipMemcpyHostToDevice));
        CK(hipMemset(m, 0, ng * 4));
        CK(hipMemset(v, 0, ng * 4));
        CK(hipMemset(vmax, 0, ng * 4));
        double tot = 0.0;
        const int reps = 50;
        for (int r = 0; r < reps + 5; ++r) {
          hipLaunchKernelGGL(ub::stream_read, dim3(4096), dim3(256), 0, 0, (const float4*)flush, (int64_t)(flush_bytes / 16),
                             (float*)flush);
          CK(hipEventRecord(a, 0));
          if (kv < 10) {
            hipLaunchKernelGGL(kerns[kv], dim3(1), dim3(1024), 0, 0, fs, c.nb, params, grad, ua, m, v, vmax, stop);
          } else {
            tr::UpdateArgs u;
            std::memset(&u, 0, sizeof(u));
            u.lambda_l2 = ua.lam;
            u.one_minus_b1 = ua.omb1;
            u.beta2 = ua.b2;
            u.one_minus_b2 = ua.omb2;
            u.eps = ua.eps;
            u.step_size = ua.step;
            u.bc2_sqrt = ua.bc2;
            u.amsgrad = ua.amsgrad;
            u.iter = r;
            CK(tr::launch_update(fs, c.nb, params, grad, u, m, v, vmax, nullptr, nullptr, nullptr, stop, 0, nullptr));
          }
          CK(hipGetLastError());
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, a, b));
          if (r >= 5) tot += ms;
        }
#if TR_UPD_PROFILE
        if (kv == 10) {
          long long prof[64][8];
          CK(hipMemcpyFromSymbol(prof, HIP_SYMBOL(tr::g_upd_prof), sizeof(prof)));
          double acc[6] = {0, 0, 0, 0, 0, 0};
          for (int r = 10; r < 50; ++r)
            for (int i = 1; i < 6; ++i) acc[i] += 10.0 * (prof[r][i] - prof[r][0]);
          std::printf("%s v5 phases (ns from entry, mean of 40): norms-issued+reduced %.0f  synced %.0f  updated %.0f  "
                      "loss %.0f  end %.0f\n", c.name, acc[1] / 40, acc[2] / 40, acc[3] / 40, acc[4] / 40, acc[5] / 40);
        }
#endif
        if (kv == 10 || kv == 4 || kv == 8 || kv == 9 || kv == 0) {  // warm-cache relaunches (kernel trace only): same kernel 20x back to back
          for (int r = 0; r < 20; ++r) {
            if (kv != 10) {
              hipLaunchKernelGGL(kerns[kv], dim3(1), dim3(1024), 0, 0, fs, c.nb, params, grad, ua, m, v, vmax, stop);
            } else {
              tr::UpdateArgs u;
              std::memset(&u, 0, sizeof(u));
              u.lambda_l2 = ua.lam;
              u.one_minus_b1 = ua.omb1;
              u.beta2 = ua.b2;
              u.one_minus_b2 = ua.omb2;
              u.eps = ua.eps;
              u.step_size = ua.step;
              u.bc2_sqrt = ua.bc2;
              u.iter = 100 + r;
              CK(tr::launch_update(fs, c.nb, params, grad, u, m, v, vmax, nullptr, nullptr, nullptr, stop, 0, nullptr));
            }
          }
          CK(hipDeviceSynchronize());
        }
        std::vector<float> out(np);
        CK(hipMemcpy(out.data(), params, np * 4, hipMemcpyDeviceToHost));
        double cs = 0.0;
        for (float x : out) cs += x;
        std::printf("%s amsgrad=%d %s: %.2f us/launch (events), checksum %.9g\n", c.name, amsgrad, names[kv],
                    1e3 * tot / reps, cs);
      }
    }
    CK(hipFree(params));
    CK(hipFree(grad));
    CK(hipFree(m));
    CK(hipFree(v));
    CK(hipFree(vmax));
  }
  CK(hipFree(flush));
  CK(hipFree(stop));
  return 0;
}
