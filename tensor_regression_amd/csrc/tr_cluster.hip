// tr_cluster.hip — single pass over X for linear models whose dense B does not fit one CU's LDS
// (BASELINE config 4: X (N, 64, 64, 32), P = 131072 floats = 512 KiB per sample).
//
// Replaces, like k_linear_fused, the forward `inner(X, cp_to_tensor(B))` + MSE + autograd
// backward of standard_tensor_regression.py:87-130, 455-462 — but where the reference (and our
// two-pass path) reads X twice per iteration, this reads it once.
//
// A CLUSTER of S workgroups owns a contiguous row range; member s owns feature slice
// [s*PS, (s+1)*PS) of every row: its B slice sits in LDS, its G slice in VGPRs.  Per row each
// member forms its partial dot, and the members exchange partials as tagged 8-byte granules
// ({tag, fp32}: the data is the flag, cdna_hip_programming.md §6 Guideline 16 R2).  Every member
// sums the S partials in slice order, so all of them derive the bitwise-identical residual and
// apply G_s += r * X_n[slice] while the slice is still in registers.
//
// Wave roles (512 threads): waves 1..7 stream X (CH float4 per lane per row, the next row in
// flight while the current one is reduced); wave 0 is the exchange wave.  It issues no X loads,
// so its granule polls do not queue behind a row of vmcnt-counted X loads; the hop overlaps the
// next row's HBM transfer.
//
// Co-residency: the plan launches S * floor(ncu / S) <= ncu workgroups of one workgroup per CU
// (occupancy >= 1 checked at plan time), so on an unshared GPU every member is resident.
// Safety when it is not: a spin that sees no partner for err[1] polls (2^16 by default; the plan
// takes TR_CLUSTER_SPIN_LIMIT for tests) sets err[0], marks the workgroup dead (NaN partials from
// then on) and runs to completion.  k_reduce_slabs copies err[0] into the gradient arena's status
// slot, where k_update sees it on every rank after the all-reduce: it stops the fit before
// applying the step, and the host falls back to the two-pass path from the untouched
// parameters.  Tags grow monotonically per plan (host-side counter), so granules left by earlier
// launches never match.
#include "tr_common.h"
#include "tr_kernels.h"

namespace tr {

namespace {
constexpr int CL_T = 512;               // threads per workgroup
constexpr int CL_NW = CL_T / TR_WAVE;   // 8 waves
constexpr int CL_TC = CL_T - TR_WAVE;   // 448 streaming threads (waves 1..7)

__device__ __forceinline__ void cl_barrier() {
  // LDS-only barrier: the streaming waves' next-row X loads stay in flight across it.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
}  // namespace

template <int CH>
__global__ __launch_bounds__(CL_T) void k_linear_cluster(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t xld, const float* __restrict__ B,
    const float* __restrict__ bias_p, const float* __restrict__ y, float scale, float* __restrict__ gpart,
    double* __restrict__ dpart, int S, int ncl, int64_t rows_per_cl, int reverse, uint32_t tag0,
    unsigned long long* __restrict__ gran, uint32_t* __restrict__ err, const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float4 lds_b[];
  if (stop != nullptr && *stop != 0) return;
  const int cl = (int)blockIdx.x / S;
  const int s = (int)blockIdx.x % S;
  if (cl >= ncl) return;
  const int t = threadIdx.x;
  const int lane = t & (TR_WAVE - 1);
  const int wv = t / TR_WAVE;
  const int ct = t - TR_WAVE;  // streaming-thread index (negative in wave 0)
  constexpr int64_t PS = (int64_t)CL_TC * CH * 4;
  const int64_t p0 = (int64_t)s * PS;
  const int64_t plen = P - p0 < PS ? P - p0 : PS;  // floats of this member's slice (% 4 == 0)
  float* red = reinterpret_cast<float*>(lds_b + CL_TC * CH);  // [2][CL_NW] wave partials
  float* tot = red + 2 * CL_NW;                               // [2] cluster dot per row parity

  if (wv > 0) {
    const float4* B4 = reinterpret_cast<const float4*>(B + p0);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = ct + c * CL_TC;
      lds_b[idx] = (int64_t)idx * 4 < plen ? B4[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();

  const int64_t r0 = (int64_t)cl * rows_per_cl;
  const int64_t r1 = r0 + rows_per_cl < N ? r0 + rows_per_cl : N;
  const int64_t nr = r1 - r0;  // identical for every member of the cluster
  const float bias = *bias_p;
  const uint32_t slice_bytes = (uint32_t)(plen * 4);
  const int voff = (ct < 0 ? 0 : ct) * 16;
  const char* Xb = reinterpret_cast<const char*>(X) + p0 * 4;

  float4 g[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) g[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  double sse = 0.0, rsum = 0.0;
  bool dead = false;
  const int spin_limit = (int)err[1];  // bounded poll (see header)

  auto row_of = [&](int64_t i) -> int64_t { return reverse ? (r1 - 1 - i) : (r0 + i); };
  auto load = [&](float4(&x)[CH], int64_t i) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(Xb + row_of(i) * xld * 4), (short)0, (int)slice_bytes, 0x00020000);
#pragma unroll
    for (int c = 0; c < CH; ++c) {  // beyond the slice the range check returns zeros
      const tr_f4 v = __builtin_bit_cast(tr_f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, c * CL_TC * 16, 2));
      x[c] = make_float4(v.x, v.y, v.z, v.w);
    }
  };

  float4 xn[CH];
  if (wv > 0 && nr > 0) load(xn, 0);
#pragma unroll 1
  for (int64_t i = 0; i < nr; ++i) {
    const int par = (int)(i & 1);
    float4 xc[CH];
    if (wv > 0) {
#pragma unroll
      for (int c = 0; c < CH; ++c) xc[c] = xn[c];
      load(xn, (i + 1 < nr) ? i + 1 : nr - 1);  // row i+1 in flight during the exchange of row i
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < CH; ++c) d = tr_dot4(xc[c], lds_b[ct + c * CL_TC], d);
      d = tr_wave_allreduce(d);
      if (lane == 0) red[par * CL_NW + wv] = d;
    }
    cl_barrier();
    if (wv == 0) {
      float part = 0.f;
#pragma unroll
      for (int k = 1; k < CL_NW; ++k) part += red[par * CL_NW + k];
      const uint32_t tag = tag0 + (uint32_t)i;
      unsigned long long* slot = gran + ((int64_t)cl * 2 + par) * S;
      if (lane == 0)
        __hip_atomic_store(slot + s, ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(part),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      float v = lane == s ? part : 0.f;
      if (!dead && spin_limit == 0) {  // test knob (TR_CLUSTER_SPIN_LIMIT=0): every exchange fails
        dead = true;
        if (lane == 0) atomicOr(err, 1u);
      }
      if (!dead) {
        for (int spins = 0;; ++spins) {
          bool ok = true;
          if (lane < S && lane != s) {
            const unsigned long long x = __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(x >> 32) == tag;
            v = __uint_as_float((uint32_t)x);
          }
          if (__all(ok)) break;
          if (spins >= spin_limit) {
            dead = true;
            if (lane == 0) atomicOr(err, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      float dot = 0.f;  // slice order: the same bits in every member
      for (int k = 0; k < S; ++k) dot += __shfl(v, k, TR_WAVE);
      if (dead) dot = __builtin_nanf("");
      if (lane == 0) tot[par] = dot;
    }
    cl_barrier();
    if (wv > 0) {
      const float dot = tot[par];
      const float e = dot + bias - y[row_of(i)];
      const float r = e * scale;
#pragma unroll
      for (int c = 0; c < CH; ++c) tr_axpy4(r, xc[c], g[c]);
      if (ct == 0) {
        sse += (double)e * (double)e;
        rsum += (double)r;
      }
    }
  }

  if (wv > 0) {
    float4* gp = reinterpret_cast<float4*>(gpart + (int64_t)cl * P + p0);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = ct + c * CL_TC;
      if ((int64_t)idx * 4 < plen) gp[idx] = g[c];
    }
    if (ct == 0 && s == 0) {
      dpart[2 * cl + 0] = sse;
      dpart[2 * cl + 1] = rsum;
    }
  }
}

// ---- host side ---------------------------------------------------------------------------
#define TR_CLUSTER_LIST(X) X(8) X(10) X(12) X(13) X(14) X(15) X(16)

template <int CH>
static hipError_t cluster_launch_t(int S, int ncl, const float* X, int64_t N, int64_t P, int64_t xld,
                                   const float* B, const float* bias, const float* y, float scale, float* gpart,
                                   double* dpart, int64_t rpc, int reverse, uint32_t tag0,
                                   unsigned long long* gran, uint32_t* err, const int32_t* stop, hipStream_t st) {
  hipLaunchKernelGGL((k_linear_cluster<CH>), dim3((unsigned)(S * ncl)), dim3(CL_T), linear_cluster_lds(CH), st, X, N,
                     P, xld, B, bias, y, scale, gpart, dpart, S, ncl, rpc, reverse, tag0, gran, err, stop);
  return hipGetLastError();
}

typedef hipError_t (*cluster_fn_t)(int, int, const float*, int64_t, int64_t, int64_t, const float*, const float*,
                                   const float*, float, float*, double*, int64_t, int, uint32_t,
                                   unsigned long long*, uint32_t*, const int32_t*, hipStream_t);
struct ClusterEntry {
  int CH;
  const void* kernel;
  cluster_fn_t launch;
};
#define TR_CLUSTER_ENTRY(CC) {CC, reinterpret_cast<const void*>(&k_linear_cluster<CC>), &cluster_launch_t<CC>},
static const ClusterEntry kCluster[] = {TR_CLUSTER_LIST(TR_CLUSTER_ENTRY)};

static const ClusterEntry* find_cluster(int CH) {
  for (const ClusterEntry& e : kCluster)
    if (e.CH == CH) return &e;
  return nullptr;
}

int linear_cluster_num_ch(void) { return (int)(sizeof(kCluster) / sizeof(kCluster[0])); }
int linear_cluster_ch(int k) { return kCluster[k].CH; }
int64_t linear_cluster_slice(int CH) { return (int64_t)CL_TC * CH * 4; }
size_t linear_cluster_lds(int CH) { return (size_t)linear_cluster_slice(CH) * 4 + (2 * CL_NW + 4) * 4; }

hipError_t prepare_linear_cluster(int CH, int* wg_per_cu) {
  *wg_per_cu = 0;
  const ClusterEntry* e = find_cluster(CH);
  if (e == nullptr) return hipErrorInvalidValue;
  const size_t lds = linear_cluster_lds(CH);
  hipError_t err = hipFuncSetAttribute(e->kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  hipFuncAttributes attr;
  err = hipFuncGetAttributes(&attr, e->kernel);
  if (err != hipSuccess) return err;
  if (attr.localSizeBytes > 0) return hipSuccess;  // spills: reject
  int nb = 0;
  err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, e->kernel, CL_T, lds);
  if (err != hipSuccess) return err;
  *wg_per_cu = nb;
  return hipSuccess;
}

hipError_t launch_linear_cluster(int CH, int S, int ncl, const float* X, int64_t N, int64_t P, int64_t xld,
                                 const float* B, const float* bias, const float* y, float scale, float* gpart,
                                 double* dpart, int64_t rows_per_cl, int reverse, uint32_t tag0,
                                 unsigned long long* gran, uint32_t* err, const int32_t* stop, hipStream_t st) {
  const ClusterEntry* e = find_cluster(CH);
  if (e == nullptr || S < 1 || S > TR_WAVE || ncl < 1) return hipErrorInvalidValue;
  // the slices must cover P exactly once and every member must own a non-empty slice
  const int64_t PS = linear_cluster_slice(CH);
  if ((int64_t)(S - 1) * PS >= P || (int64_t)S * PS < P || P % 4 != 0 || xld % 4 != 0) return hipErrorInvalidValue;
  return e->launch(S, ncl, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_cl, reverse, tag0, gran, err,
                   stop, st);
}

}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_cluster() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_linear_cluster<15>));
}
}  // namespace tr
