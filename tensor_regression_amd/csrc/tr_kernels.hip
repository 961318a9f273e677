// tr_kernels.hip — gfx950 (MI355X / CDNA4) kernels for the CP tensor-regression hot path.
//
// Reference op sequence replaced (one fit_Adam iteration, standard_tensor_regression.py:458-470,
// multinomial_tensor_regression.py:453-465):
//
//   non_neg_fn            -> k_prep_factors       softplus / softplus' of flagged factors
//   cp_to_tensor          -> k_build_dense        B = (Phi_0 * w) @ KR(Phi_1..)^T, factor columns in LDS
//   inner + loss + backward (the two aten::mm that are ~96 % of the reference's time):
//       linear, P fits a CU -> k_linear_fused    ONE pass over X: y_hat, residual, G = X^T r
//       otherwise           -> k_rows + k_cols   two passes (forward rows, column reduction)
//   (partials)            -> k_reduce_slabs       fixed-order slab sum (deterministic, no atomics)
//   cp_to_tensor backward -> k_mttkrp             dPhi_f = G_(f) . KR(others) * w, chained through softplus'
//   L2_penalty + Adam     -> k_update             (tr_update.hip)
//
// Every reduction is a fixed-order tree (wave butterfly, then LDS in wave order, then slabs
// in index order) so a run is bitwise reproducible; no float atomics anywhere.

#include <cstdlib>

#include "tr_common.h"
#include "tr_kernels.h"

#include <cstring>

namespace tr {

// ------------------------------------------------------------------------------------------
// X stream load policy: X is read once per pass (>> the 256 MiB Infinity Cache), so its loads
// are non-temporal: 6.80 vs 6.32 TB/s with the default policy on the single-pass kernel, 6.82 vs
// 6.06 TB/s on a grid-stride read probe (tools/hbm_probe.hip).
// ------------------------------------------------------------------------------------------
#define TR_X_AUX 2  // buffer-load cache-policy bits (2 = nt)
__device__ __forceinline__ float4 ldx(const float4* p) {
  const tr_f4 v = __builtin_nontemporal_load(reinterpret_cast<const tr_f4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float ldx(const float* p) { return __builtin_nontemporal_load(p); }

// ==========================================================================================
// X range statistics (tr_x_range), for the plan's choice of its split kernels' X form: over the
// rows of workgroup b (one wave per row: rows 4 b + w, 4 b + w + 4 nblocks, ...) max |x|, min x,
// and the smallest mean x^2 of a row that is not all zero
// ==========================================================================================
__global__ __launch_bounds__(256) void k_x_range(const float* __restrict__ X, int64_t N, int64_t P, int64_t xld,
                                                 double* __restrict__ out) {
  __shared__ float smax[4], smin[4];
  __shared__ double sms[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float m = 0.f, mn = __builtin_huge_valf();
  double rms_min = __builtin_huge_val();
  for (int64_t n = 4 * (int64_t)blockIdx.x + w; n < N; n += 4 * (int64_t)gridDim.x) {
    const float* row = X + n * xld;
    double ps = 0.0;
    for (int64_t e = lane; e < P; e += 64) {
      const float v = ldx(row + e);
      m = (v != v) ? v : fmaxf(m, fabsf(v));  // a NaN is reported, not dropped by fmaxf
      mn = fminf(mn, v);
      ps += (double)v * (double)v;
    }
    for (int o = 32; o > 0; o >>= 1) ps += __shfl_xor(ps, o, 64);
    if (ps > 0.0) rms_min = fmin(rms_min, ps / (double)P);
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float a = __shfl_xor(m, o, 64);
    m = (m != m || a != a) ? __builtin_nanf("") : fmaxf(m, a);
    mn = fminf(mn, __shfl_xor(mn, o, 64));
  }
  if (lane == 0) {
    smax[w] = m;
    smin[w] = mn;
    sms[w] = rms_min;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = smax[0], b = smin[0];
    double c = sms[0];
    for (int k = 1; k < 4; ++k) {
      a = (a != a || smax[k] != smax[k]) ? __builtin_nanf("") : fmaxf(a, smax[k]);
      b = fminf(b, smin[k]);
      c = fmin(c, sms[k]);
    }
    out[blockIdx.x] = (double)a;
    out[gridDim.x + blockIdx.x] = c;
    out[2 * gridDim.x + blockIdx.x] = (double)b;
  }
}

hipError_t launch_x_range(const float* X, int64_t N, int64_t P, int64_t xld, double* out, int nblocks, hipStream_t st) {
  if (nblocks < 1 || nblocks > 1024 || N < 0 || P < 1 || xld < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_x_range, dim3(nblocks), dim3(256), 0, st, X, N, P, xld, out);
  return hipGetLastError();
}

// ==========================================================================================
// K1a: factor preparation  (non_neg_fn, standard…py:53-85; multinomial…py:116-146)
// ==========================================================================================
__global__ __launch_bounds__(256) void k_prep_factors(FactorSet fs, const float* __restrict__ params,
                                                      float beta, float thr, float* __restrict__ phi,
                                                      float* __restrict__ dphi,
                                                      const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= fs.nfelem) return;
  int f = 0;
#pragma unroll
  for (int g = 1; g < TR_MAXF; ++g)
    if (g < fs.nf && e >= fs.off[g]) f = g;
  const float a = params[e];
  if (fs.nonneg[f]) {
    phi[e] = tr_softplus(a, beta, thr);
    dphi[e] = tr_softplus_grad(a, beta, thr);
  } else {
    phi[e] = a;
    dphi[e] = 1.0f;
  }
}

// ==========================================================================================
// K1b: dense coefficient tensor (tensorly cp_to_tensor, called at standard…py:124,
// multinomial…py:182), fused with non_neg_fn: every workgroup stages the raw factors in LDS and
// applies softplus there (sum_f I_f * R floats); workgroup 0 also publishes Phi and softplus'
// for the gradient kernels.  Factor sets too large for LDS fall back to k_prep_factors + global.
// ==========================================================================================
__device__ __forceinline__ int tr_factor_of(const FactorSet& fs, int64_t e) {
  int f = 0;
#pragma unroll
  for (int g = 1; g < TR_MAXF; ++g)
    if (g < fs.nf && e >= fs.off[g]) f = g;
  return f;
}

__global__ __launch_bounds__(256) void k_build_dense(FactorSet fs, const float* __restrict__ params,
                                                     float beta, float thr, float* __restrict__ phi,
                                                     float* __restrict__ dphi, const float* __restrict__ w,
                                                     float* __restrict__ dense, int use_lds,
                                                     const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float sphi[];
  if (stop != nullptr && *stop != 0) return;
  const float* F = phi;
  if (use_lds) {
    const bool publish = blockIdx.x == 0;
    unsigned nnmask = 0;  // factors under softplus
#pragma unroll
    for (int g = 0; g < TR_MAXF; ++g)
      if (g < fs.nf && fs.nonneg[g]) nnmask |= 1u << g;
    auto stage = [&](int64_t k, float a) {
      float v = a, d = 1.0f;
      if ((nnmask >> tr_factor_of(fs, k)) & 1u) {
        v = tr_softplus(a, beta, thr);
        d = tr_softplus_grad(a, beta, thr);
      }
      sphi[k] = v;
      if (publish) {
        phi[k] = v;
        dphi[k] = d;
      }
    };
    // four elements per trip with their loads in flight together: the factors are read from a
    // cold L2 right after the update, one round trip per element would dominate the launch
    const int64_t B = blockDim.x;
    int64_t k = threadIdx.x;
    for (; k + 3 * B < fs.nfelem; k += 4 * B) {
      const float a0 = params[k], a1 = params[k + B], a2 = params[k + 2 * B], a3 = params[k + 3 * B];
      stage(k, a0);
      stage(k + B, a1);
      stage(k + 2 * B, a2);
      stage(k + 3 * B, a3);
    }
    for (; k < fs.nfelem; k += B) stage(k, params[k]);
    __syncthreads();
    F = sphi;
  }
  const int R = fs.rank;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < fs.total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t idx[TR_MAXF];
    int64_t pos = 0;
    if (fs.total < (int64_t(1) << 31)) {  // 32-bit index arithmetic (every config)
      const uint32_t e32 = (uint32_t)e;
#pragma unroll
      for (int f = 0; f < TR_MAXF; ++f) {
        if (f < fs.nf) {
          idx[f] = (e32 / (uint32_t)fs.rstride[f]) % (uint32_t)fs.dim[f];
          pos += idx[f] * fs.stride[f];
        }
      }
    } else {
#pragma unroll
      for (int f = 0; f < TR_MAXF; ++f) {
        if (f < fs.nf) {
          idx[f] = (e / fs.rstride[f]) % fs.dim[f];
          pos += idx[f] * fs.stride[f];
        }
      }
    }
    float s = 0.0f;
    if (fs.nf == 1) {
      // cp_to_tensor single-factor branch: sum(weights * factors[0], dim=1)
      const float* a0 = F + fs.off[0] + idx[0] * R;
      for (int r = 0; r < R; ++r) s += w[r] * a0[r];
    } else {
      // (Phi_0 * w) @ KR(Phi_1, ..., Phi_{F-1})^T, KR folded left (first matrix slowest)
      for (int r = 0; r < R; ++r) {
        const float a = F[fs.off[0] + idx[0] * R + r] * w[r];
        float k = F[fs.off[1] + idx[1] * R + r];
        for (int f = 2; f < fs.nf; ++f) k *= F[fs.off[f] + idx[f] * R + r];
        s = fmaf(a, k, s);
      }
    }
    dense[pos] = s;
  }
}

// ==========================================================================================
// K2 (linear, single pass): fused forward + MSE residual + X^T r for one WG-owned row range.
//
// One workgroup of T threads owns a contiguous row range; the whole P-wide row is split
// across its T threads as CH float4 per thread (P == 4*T*CH).  B (P floats) sits in LDS,
// the partial gradient G_wg (P floats) in registers, and X rows stream through two register
// buffers (row i+1 is in flight while row i is reduced) — X is read from HBM exactly once
// per iteration, where the reference's autograd reads it twice (mm forward + MmBackward0).
//
// Per row:  dot = <X_n, B> (lane FMAs -> wave butterfly -> LDS across waves, fixed order)
//           y_hat = dot + bias; e = y_hat - y_n; r = e * (2/N)   (MSELoss mean backward)
//           G_wg += r * X_n;  sse += e^2; rsum += r               (bias grad = sum r)
// ==========================================================================================
template <int T, int CH>
__global__ __launch_bounds__(T) void k_linear_fused(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t xld, const float* __restrict__ B,
    const float* __restrict__ bias_p, const float* __restrict__ y, float scale,
    float* __restrict__ gpart, double* __restrict__ dpart, float* __restrict__ yhat,
    int64_t rows_per_wg, int reverse, const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float4 lds_b[];
  if (stop != nullptr && *stop != 0) return;
  constexpr int NW = T / TR_WAVE;
  const int t = threadIdx.x;
  const int lane = t & (TR_WAVE - 1);
  const int wv = t / TR_WAVE;
  float* red = reinterpret_cast<float*>(lds_b + T * CH);  // [2][NW]

  // P may fall short of 4 T CH (a padded row) and need not be a multiple of 4: the floats past P take
  // zero B and read zero X (the row descriptor's range is checked per dword; rows start 4-B aligned,
  // which a dwordx4 buffer load takes), and the partial slab is written with a stride of P rounded up
  // to 4 floats (its floats past P hold zero)
  const float4* B4 = reinterpret_cast<const float4*>(B);
  const int64_t P4 = P / 4, Pq = (P + 3) / 4;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t q = t + c * T;
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < P4) {
      b = B4[q];
    } else if (q < Pq) {  // the last, partial quad
      const int64_t e = 4 * q;
      b.x = B[e];
      if (e + 1 < P) b.y = B[e + 1];
      if (e + 2 < P) b.z = B[e + 2];
    }
    lds_b[q] = b;
  }
  __syncthreads();

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r1 = r0 + rows_per_wg < N ? r0 + rows_per_wg : N;
  const int64_t nr = r1 - r0;
  const float bias = *bias_p;
  // rows are addressed through a per-row buffer descriptor (SGPRs): one 32-bit voffset per
  // lane instead of CH 64-bit addresses keeps the row buffers + G partial inside 128 VGPRs.
  const uint32_t row_bytes = (uint32_t)(P * 4);
  const int voff = t * 16;
  const char* Xb = reinterpret_cast<const char*>(X);

  float4 g[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) g[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  double sse = 0.0, rsum = 0.0;

  auto row_of = [&](int64_t i) -> int64_t { return reverse ? (r1 - 1 - i) : (r0 + i); };
  auto load = [&](float4(&x)[CH], int64_t i) {
    const char* base = Xb + row_of(i) * xld * 4;  // row stride xld floats (>= or < P: windowed views)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(base), (short)0, (int)row_bytes, 0x00020000);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const tr_f4 v = __builtin_bit_cast(tr_f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, c * T * 16, TR_X_AUX));
      x[c] = make_float4(v.x, v.y, v.z, v.w);
    }
  };
  auto process = [&](const float4(&x)[CH], int64_t i, int par) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) s = tr_dot4(x[c], lds_b[t + c * T], s);
    s = tr_wave_allreduce(s);
    if (lane == 0) red[par * NW + wv] = s;
    __syncthreads();
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) dot += red[par * NW + k];
    const int64_t row = row_of(i);
    const float yh = dot + bias;
    const float e = yh - y[row];
    const float r = e * scale;
#pragma unroll
    for (int c = 0; c < CH; ++c) tr_axpy4(r, x[c], g[c]);
    if (t == 0) {
      sse += (double)e * (double)e;
      rsum += (double)r;
    }
  };

  if (nr > 0) {
    float4 xn[CH];
    load(xn, 0);
#pragma unroll 1
    for (int64_t i = 0; i < nr; ++i) {
      float4 xc[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) xc[c] = xn[c];
      load(xn, (i + 1 < nr) ? i + 1 : nr - 1);  // row i+1 in flight while row i is reduced
      process(xc, i, (int)(i & 1));
    }
  }

  float4* gp = reinterpret_cast<float4*>(gpart + (int64_t)blockIdx.x * (4 * Pq)) + t;
#pragma unroll
  for (int c = 0; c < CH; ++c)
    if (t + c * T < Pq) gp[c * T] = g[c];
  if (t == 0) {
    dpart[2 * blockIdx.x + 0] = sse;
    dpart[2 * blockIdx.x + 1] = rsum;
  }
}

// ==========================================================================================
// K2p (linear, single pass, short rows P <= 128): k_linear_fused puts one row on at least one
// wave (4 T CH >= 256 floats), so a 16-float row leaves 15 of 16 lanes idle and the pass runs at
// 9 % of HBM.  Here a wave holds G = 64 / PQ rows at once: lane l takes quad q = l % PQ of row
// l / PQ (PQ = ceil(P / 4) rounded up to a power of two), so one 16-B load per lane covers G
// consecutive rows (G P floats, contiguous when xld == P).  The dot is a segmented xor-butterfly
// over the PQ lanes of a row (ds_swizzle, inside a 32-lane half); every lane of the segment
// gets the same sum, forms r and accumulates r X_n into its own quad of G.  At the end the G
// segments' quads are summed (xor PQ .. 32), then the 4 waves in LDS in fixed order: the partial
// slab per workgroup is the one k_linear_fused writes (stride 4 ceil(P / 4), zero past P), so
// k_reduce_slabs finishes it unchanged.  U blocks of G rows are in flight per wave.
//   Row range per workgroup as k_linear_fused (rows_per_wg, reverse: blocks taken backwards);
//   a block's buffer descriptor starts at its first row and ends at the last row's float P, so
//   rows past the range and floats past P of the last row read zero; floats past P of the other
//   rows (the next row's data) are zeroed in registers.
// ==========================================================================================
template <int PQ, int U>
__global__ __launch_bounds__(256) void k_linear_packed(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t xld, const float* __restrict__ B,
    const float* __restrict__ bias_p, const float* __restrict__ y, float scale,
    float* __restrict__ gpart, double* __restrict__ dpart, int64_t rows_per_wg, int reverse,
    const int32_t* __restrict__ stop) {
  constexpr int G = TR_WAVE / PQ;  // rows per block
  constexpr int NW = 4;
  static_assert(PQ >= 1 && PQ <= 32 && (PQ & (PQ - 1)) == 0, "PQ: a power of two <= 32");
  __shared__ float4 sg[NW][PQ];
  __shared__ double sd[NW][2];
  if (stop != nullptr && *stop != 0) return;
  const int t = threadIdx.x;
  const int lane = t & (TR_WAVE - 1);
  const int wv = t / TR_WAVE;
  const int q = lane % PQ;
  const int seg = lane / PQ;
  const int64_t Pq = (P + 3) / 4;
  // this lane's B quad and the mask of its floats below P
  const int e0 = 4 * q;
  const bool m0 = e0 < P, m1 = e0 + 1 < P, m2 = e0 + 2 < P, m3 = e0 + 3 < P;
  float4 b = make_float4(m0 ? B[e0] : 0.f, m1 ? B[e0 + 1] : 0.f, m2 ? B[e0 + 2] : 0.f, m3 ? B[e0 + 3] : 0.f);
  const float bias = bias_p != nullptr ? *bias_p : 0.f;

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r1 = r0 + rows_per_wg < N ? r0 + rows_per_wg : N;
  const int64_t nr = r1 > r0 ? r1 - r0 : 0;
  const int64_t nb = (nr + G - 1) / G;
  const int voff = (int)((int64_t)seg * xld * 4 + 16 * q);
  const char* Xb = reinterpret_cast<const char*>(X);

  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  double sse = 0.0, rsum = 0.0;
#pragma unroll 1
  for (int64_t k0 = (int64_t)wv * U; k0 < nb; k0 += (int64_t)NW * U) {
    float4 x[U];
    int64_t fr[U];
    int rin[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = k0 + u;
      const int64_t kb = reverse ? nb - 1 - k : k;
      fr[u] = r0 + kb * G;
      const int64_t left = r1 - fr[u];
      rin[u] = k < nb ? (int)(left < G ? left : G) : 0;
      const int nrec = rin[u] > 0 ? (int)((int64_t)(rin[u] - 1) * xld * 4 + P * 4) : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char*>(Xb + (k < nb ? fr[u] : 0) * xld * 4), (short)0, nrec, 0x00020000);
      const tr_f4 v = __builtin_bit_cast(tr_f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, TR_X_AUX));
      x[u] = make_float4(m0 ? v.x : 0.f, m1 ? v.y : 0.f, m2 ? v.z : 0.f, m3 ? v.w : 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s = tr_dot4(x[u], b, 0.f);
      if (PQ >= 32) s += tr_swz_xor<0x401F>(s);
      if (PQ >= 16) s += tr_swz_xor<0x201F>(s);
      if (PQ >= 8) s += tr_swz_xor<0x101F>(s);
      if (PQ >= 4) s += tr_swz_xor<0x081F>(s);
      if (PQ >= 2) s += tr_swz_xor<0x041F>(s);
      const bool valid = seg < rin[u];
      const float e = valid ? s + bias - y[fr[u] + seg] : 0.f;
      const float r = e * scale;
      tr_axpy4(r, x[u], g);
      if (q == 0) {
        sse += (double)e * (double)e;
        rsum += (double)r;
      }
    }
  }
  // the G segments' quads, then the waves in fixed order
#pragma unroll
  for (int o = PQ; o < TR_WAVE; o <<= 1) {
    g.x += __shfl_xor(g.x, o, TR_WAVE);
    g.y += __shfl_xor(g.y, o, TR_WAVE);
    g.z += __shfl_xor(g.z, o, TR_WAVE);
    g.w += __shfl_xor(g.w, o, TR_WAVE);
  }
  sse = tr_wave_allreduce_d(sse);
  rsum = tr_wave_allreduce_d(rsum);
  if (seg == 0) sg[wv][q] = g;
  if (lane == 0) {
    sd[wv][0] = sse;
    sd[wv][1] = rsum;
  }
  __syncthreads();
  if (t < PQ && t < Pq) {
    float4 a = sg[0][t];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float4 c = sg[w][t];
      a.x += c.x;
      a.y += c.y;
      a.z += c.z;
      a.w += c.w;
    }
    reinterpret_cast<float4*>(gpart + (int64_t)blockIdx.x * (4 * Pq))[t] = a;
  }
  if (t == 0) {
    dpart[2 * blockIdx.x + 0] = sd[0][0] + sd[1][0] + sd[2][0] + sd[3][0];
    dpart[2 * blockIdx.x + 1] = sd[0][1] + sd[1][1] + sd[2][1] + sd[3][1];
  }
}

// ==========================================================================================
// K2' two-pass forward: Z[n, c] = <X_n, Bt_c>  (+ fused epilogue per MODE)
//   MODE_LIN_TRAIN : r[n] = (z + bias - y) * scale; per-wave (sse, sum r)
//   MODE_LIN_PRED  : out[n] = z + bias
//   MODE_MNL_TRAIN : S = softmax(z); CE on S (double softmax, multinomial…py:448-450);
//                    dZ[n, :] written; per-wave weighted NLL partial
//   MODE_MNL_PRED  : out[n, :] = softmax(z)
// One wave owns RB consecutive rows; lanes stride the row in W-float vectors; the C class
// columns of B come from L2 (B <= a few hundred KiB stays resident in every XCD's L2).
// ==========================================================================================
template <int W> struct VecT;
template <> struct VecT<4> {
  using T = float4;
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ float dot(const T a, const T b, float acc) { return tr_dot4(a, b, acc); }
  static __device__ __forceinline__ void axpy(float s, const T x, T& acc) { tr_axpy4(s, x, acc); }
  static __device__ __forceinline__ float hsum(const T a) { return (a.x + a.y) + (a.z + a.w); }
  static __device__ __forceinline__ T add(const T a, const T b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
};
template <> struct VecT<1> {
  using T = float;
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ float dot(const T a, const T b, float acc) { return fmaf(a, b, acc); }
  static __device__ __forceinline__ void axpy(float s, const T x, T& acc) { acc = fmaf(s, x, acc); }
  static __device__ __forceinline__ float hsum(const T a) { return a; }
  static __device__ __forceinline__ T add(const T a, const T b) { return a + b; }
};

template <int C, int RB, int MODE, int W>
__global__ __launch_bounds__(256) void k_rows(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t xld, const float* __restrict__ Bt,
    const float* __restrict__ bias_p, const void* __restrict__ target,
    const float* __restrict__ class_w, float scale, float* __restrict__ out,
    double* __restrict__ dpart, float* __restrict__ yhat, const int32_t* __restrict__ stop, int64_t ldo) {
  using V = VecT<W>;
  using VT = typename V::T;
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x / TR_WAVE) + (threadIdx.x / TR_WAVE);
  const int64_t row0 = gw * RB;
  if (row0 >= N) {
    if (MODE == MODE_LIN_TRAIN || MODE == MODE_MNL_TRAIN) {
      if (lane == 0) {
        dpart[2 * gw] = 0.0;
        dpart[2 * gw + 1] = 0.0;
      }
    }
    return;
  }
  const int64_t PW = P / W;
  const VT* Xv = reinterpret_cast<const VT*>(X);
  const VT* Bv = reinterpret_cast<const VT*>(Bt);
  const VT* xr[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int64_t row = (row0 + r < N) ? row0 + r : N - 1;
    xr[r] = Xv + row * (xld / W);
  }
  float acc[RB][C];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[r][c] = 0.f;

  int64_t q = lane;
  for (; q + TR_WAVE < PW; q += 2 * TR_WAVE) {
    VT x0[RB], x1[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      x0[r] = ldx(xr[r] + q);
      x1[r] = ldx(xr[r] + q + TR_WAVE);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const VT b0 = Bv[c * PW + q];
      const VT b1 = Bv[c * PW + q + TR_WAVE];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        acc[r][c] = V::dot(x0[r], b0, acc[r][c]);
        acc[r][c] = V::dot(x1[r], b1, acc[r][c]);
      }
    }
  }
  if (q < PW) {
    VT x0[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) x0[r] = ldx(xr[r] + q);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const VT b0 = Bv[c * PW + q];
#pragma unroll
      for (int r = 0; r < RB; ++r) acc[r][c] = V::dot(x0[r], b0, acc[r][c]);
    }
  }
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[r][c] = tr_wave_allreduce(acc[r][c]);

  if (MODE == MODE_MNL_LOGITS) {  // one class tile of the logits, row stride ldo
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int64_t row = row0 + r;
      if (row < N)
#pragma unroll
        for (int c = 0; c < C; ++c)
          if (lane == c) out[row * ldo + c] = acc[r][c];
    }
  } else if (MODE == MODE_LIN_TRAIN || MODE == MODE_LIN_PRED) {
    const float bias = *bias_p;
    const float* y = reinterpret_cast<const float*>(target);
    double sse = 0.0, rsum = 0.0;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int64_t row = row0 + r;
      if (row < N) {
        const float yh = acc[r][0] + bias;
        if (MODE == MODE_LIN_PRED) {
          if (lane == r) out[row] = yh;
        } else {
          const float e = yh - y[row];
          const float rr = e * scale;
          if (lane == r) {
            out[row] = rr;
            if (yhat != nullptr) yhat[row] = yh;
          }
          sse += (double)e * (double)e;
          rsum += (double)rr;
        }
      }
    }
    if (MODE == MODE_LIN_TRAIN && lane == 0) {
      dpart[2 * gw] = sse;
      dpart[2 * gw + 1] = rsum;
    }
  } else {
    const int64_t* lab = reinterpret_cast<const int64_t*>(target);
    double lsum = 0.0;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int64_t row = row0 + r;
      if (row < N) {
        // S = softmax(z)
        float mx = acc[r][0];
#pragma unroll
        for (int c = 1; c < C; ++c) mx = fmaxf(mx, acc[r][c]);
        float S[C];
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          S[c] = expf(acc[r][c] - mx);
          sum += S[c];
        }
        const float inv = 1.0f / sum;
#pragma unroll
        for (int c = 0; c < C; ++c) S[c] = S[c] * inv;
        if (MODE == MODE_MNL_PRED) {
#pragma unroll
          for (int c = 0; c < C; ++c)
            if (lane == c) out[row * C + c] = S[c];
        } else {
          // CrossEntropyLoss(weight) applied to the probabilities S (double softmax):
          // log Q = S - m2 - log(sum exp(S - m2))
          float m2 = S[0];
#pragma unroll
          for (int c = 1; c < C; ++c) m2 = fmaxf(m2, S[c]);
          float Q[C];
          float s2 = 0.f;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            Q[c] = expf(S[c] - m2);
            s2 += Q[c];
          }
          const float lse = logf(s2);
          const float inv2 = 1.0f / s2;
          const int64_t yl = lab[row];
          const float cw = class_w[yl];
          float logq_y = 0.f;
#pragma unroll
          for (int c = 0; c < C; ++c)
            if (c == yl) logq_y = (S[c] - m2) - lse;
          lsum += (double)cw * (double)(-logq_y);
          // dL/dS = (Q - onehot) * cw / W ; dL/dZ = S * (dS - <dS, S>)
          const float gsc = cw * scale;
          float dS[C];
          float dot = 0.f;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            dS[c] = (Q[c] * inv2 - (c == yl ? 1.0f : 0.0f)) * gsc;
            dot = fmaf(dS[c], S[c], dot);
          }
#pragma unroll
          for (int c = 0; c < C; ++c)
            if (lane == c) out[row * C + c] = S[c] * (dS[c] - dot);
        }
      }
    }
    if (MODE == MODE_MNL_TRAIN && lane == 0) {
      dpart[2 * gw] = lsum;
      dpart[2 * gw + 1] = 0.0;
    }
  }
}

// ==========================================================================================
// K2m: multinomial forward on the matrix cores.  Z (rows x C) = X (rows x P) . B (P x C) with
// v_mfma_f32_16x16x4_f32 (exact fp32, C padded to 16 lanes), fused double-softmax CE / dZ
// epilogue.  A wave owns RT tiles of 16 rows; per 32-deep k step each lane loads two float4 of
// X (its row, 8 consecutive features: 4 lanes cover a full 128-B line) and two float4 of the
// class-major Bt (shared by the RT row tiles), then issues 8*RT MFMAs.  Lane l supplies
// A[i=l&15][k=l>>4] and B[k=l>>4][j=l&15]; MFMA m of a step uses feature k0 + 8*(l>>4) + m on
// both operands, so the k order is permuted consistently.  Accumulator layout: class = l&15,
// row = 4*(l>>4) + reg.  Class reductions are 16-lane swizzle butterflies (deterministic).
// ==========================================================================================
template <int PATTERN>
__device__ __forceinline__ float tr_swz(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), PATTERN));
}
__device__ __forceinline__ float tr_sum16(float v) {
  v += tr_swz<0x201F>(v);  // xor 8
  v += tr_swz<0x101F>(v);  // xor 4
  v += tr_swz<0x081F>(v);  // xor 2
  v += tr_swz<0x041F>(v);  // xor 1
  return v;
}
__device__ __forceinline__ float tr_max16(float v) {
  v = fmaxf(v, tr_swz<0x201F>(v));
  v = fmaxf(v, tr_swz<0x101F>(v));
  v = fmaxf(v, tr_swz<0x081F>(v));
  v = fmaxf(v, tr_swz<0x041F>(v));
  return v;
}

typedef float tr_f32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int RT>
__global__ __launch_bounds__(256) void k_rows_mfma(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t xld, const float* __restrict__ Bt, int C,
    const int64_t* __restrict__ lab, const float* __restrict__ class_w, float scale,
    float* __restrict__ out, double* __restrict__ dpart, const int32_t* __restrict__ stop, int64_t ldo) {
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x / TR_WAVE) + (threadIdx.x / TR_WAVE);
  const int64_t row0 = gw * (16 * RT);
  if (MODE == MODE_MNL_LOGITS) {  // class tile blockIdx.y: Bt / out are offset by the host
    Bt += (int64_t)blockIdx.y * 16 * P;
    out += (int64_t)blockIdx.y * 16;
    C = C - 16 * (int)blockIdx.y < 16 ? C - 16 * (int)blockIdx.y : 16;
  }
  const int i = lane & 15;  // A row in tile / class column
  const int g = lane >> 4;  // k group
  if (row0 >= N) {
    if (MODE == MODE_MNL_TRAIN && lane == 0) {
      dpart[2 * gw] = 0.0;
      dpart[2 * gw + 1] = 0.0;
    }
    return;
  }
  const float4* xr[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    int64_t r = row0 + rt * 16 + i;
    r = r < N ? r : N - 1;
    xr[rt] = reinterpret_cast<const float4*>(X + r * xld + 8 * g);
  }
  const bool cls_ok = i < C;
  // Bt is padded to 16 class rows (rows >= C are zero): unconditional loads, no per-lane branches
  const float4* br = reinterpret_cast<const float4*>(Bt + (int64_t)i * P + 8 * g);
  // Blocked summation: 8 independent accumulator chains per row tile (MFMA m of a step feeds
  // chain m), folded by a fixed tree into a running total every 16 steps (512 features).  One
  // chain over all P/4 MFMAs (round 2) left Z 6.5e-5 from exact at P = 8192, |Z| = 58
  // (mnl_duo_t), 2x the probability error of the reference's own blocked fp32 GEMM; this order
  // is 6.9e-6 (emulated).  Independent chains also keep back-to-back MFMAs independent.
  tr_f32x4 ac[RT][8], acc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    acc[rt] = tr_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 8; ++m) ac[rt][m] = tr_f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto fold = [&]() {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      acc[rt] += ((ac[rt][0] + ac[rt][1]) + (ac[rt][2] + ac[rt][3])) + ((ac[rt][4] + ac[rt][5]) + (ac[rt][6] + ac[rt][7]));
#pragma unroll
      for (int m = 0; m < 8; ++m) ac[rt][m] = tr_f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  const int nsteps = (int)(P / 32);
  auto step = [&](const float4(&xa)[RT], const float4(&xb)[RT], const float4 ba, const float4 bb) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      ac[rt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[rt].x, ba.x, ac[rt][0], 0, 0, 0);
      ac[rt][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[rt].y, ba.y, ac[rt][1], 0, 0, 0);
      ac[rt][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[rt].z, ba.z, ac[rt][2], 0, 0, 0);
      ac[rt][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[rt].w, ba.w, ac[rt][3], 0, 0, 0);
      ac[rt][4] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[rt].x, bb.x, ac[rt][4], 0, 0, 0);
      ac[rt][5] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[rt].y, bb.y, ac[rt][5], 0, 0, 0);
      ac[rt][6] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[rt].z, bb.z, ac[rt][6], 0, 0, 0);
      ac[rt][7] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[rt].w, bb.w, ac[rt][7], 0, 0, 0);
    }
  };
  int st = 0;
  for (; st + 1 < nsteps; st += 2) {  // two k steps of loads in flight before the MFMAs
    float4 xa0[RT], xb0[RT], xa1[RT], xb1[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      xa0[rt] = xr[rt][8 * st];  // default policy: each 128-B line is read by two
      xb0[rt] = xr[rt][8 * st + 1];  // consecutive steps' loads (nt measured 14 % slower)
      xa1[rt] = xr[rt][8 * st + 8];
      xb1[rt] = xr[rt][8 * st + 9];
    }
    const float4 ba0 = br[8 * st], bb0 = br[8 * st + 1];
    const float4 ba1 = br[8 * st + 8], bb1 = br[8 * st + 9];
    __builtin_amdgcn_sched_barrier(0);  // keep all 4*RT+4 loads of the two steps in flight together
    step(xa0, xb0, ba0, bb0);
    step(xa1, xb1, ba1, bb1);
    if (((st + 2) & 15) == 0) fold();
  }
  if (st < nsteps) {
    float4 xa0[RT], xb0[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      xa0[rt] = xr[rt][8 * st];
      xb0[rt] = xr[rt][8 * st + 1];
    }
    const float4 ba0 = br[8 * st], bb0 = br[8 * st + 1];
    step(xa0, xb0, ba0, bb0);
  }
  fold();
  const float NEG = -__builtin_huge_valf();
  double lsum = 0.0;
  if (MODE == MODE_MNL_LOGITS) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int64_t row = row0 + rt * 16 + 4 * g + reg;
        if (cls_ok && row < N) out[row * ldo + i] = acc[rt][reg];
      }
    return;
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int64_t row = row0 + rt * 16 + 4 * g + reg;
      const float z = cls_ok ? acc[rt][reg] : NEG;
      const float mx = tr_max16(z);
      const float ez = cls_ok ? expf(z - mx) : 0.f;
      const float sum = tr_sum16(ez);
      const float S = ez * (1.0f / sum);
      if (MODE == MODE_MNL_PRED) {
        if (cls_ok && row < N) out[row * ldo + i] = S;
        continue;
      }
      // CrossEntropyLoss(weight) on the probabilities S (double softmax)
      const float m2 = tr_max16(cls_ok ? S : NEG);
      const float q = cls_ok ? expf(S - m2) : 0.f;
      const float s2 = tr_sum16(q);
      const float lse = logf(s2);
      const bool valid = row < N;
      const int64_t yl = valid ? lab[row] : -1;
      const float cw = valid ? class_w[yl] : 0.f;
      const bool is_y = cls_ok && (int64_t)i == yl;
      if (is_y) lsum += (double)cw * (double)(-((S - m2) - lse));
      const float dS = cls_ok ? (q * (1.0f / s2) - (is_y ? 1.0f : 0.0f)) * (cw * scale) : 0.f;
      const float dot = tr_sum16(dS * S);
      if (cls_ok && valid) out[row * ldo + i] = S * (dS - dot);
    }
  }
  if (MODE == MODE_MNL_TRAIN) {
    lsum = tr_wave_allreduce_d(lsum);
    if (lane == 0) {
      dpart[2 * gw] = lsum;
      dpart[2 * gw + 1] = 0.0;
    }
  }
}

// ==========================================================================================
// K2w: wide-class epilogue (C > 16).  One wave per row (grid-stride over rows), the C logits
// across lanes in chunks of 64: S = softmax(Z) (multinomial…py:187), then CrossEntropyLoss(weight)
// on the probabilities (the double softmax, :448-456) and dZ = S (dS - <dS, S>), written over Z.
// Fixed-order reductions (per-lane strided sums, then the wave butterfly): deterministic.
// ==========================================================================================
template <int MODE>
__global__ __launch_bounds__(256) void k_softmax_rows(float* __restrict__ Z, int64_t N, int C,
                                                      const int64_t* __restrict__ lab,
                                                      const float* __restrict__ class_w, float scale,
                                                      float* __restrict__ out, double* __restrict__ dpart,
                                                      const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x / TR_WAVE) + (threadIdx.x / TR_WAVE);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / TR_WAVE);
  const float NEG = -__builtin_huge_valf();
  double lsum = 0.0;
  for (int64_t row = gw; row < N; row += nw) {
    float* z = Z + row * C;
    float mx = NEG;
    for (int c = lane; c < C; c += TR_WAVE) mx = fmaxf(mx, z[c]);
    mx = tr_wave_allreduce_max(mx);
    float sum = 0.f;
    for (int c = lane; c < C; c += TR_WAVE) sum += expf(z[c] - mx);
    sum = tr_wave_allreduce(sum);
    const float inv = 1.0f / sum;
    if (MODE == MODE_MNL_PRED) {
      for (int c = lane; c < C; c += TR_WAVE) out[row * C + c] = expf(z[c] - mx) * inv;
      continue;
    }
    float m2 = NEG;
    for (int c = lane; c < C; c += TR_WAVE) m2 = fmaxf(m2, expf(z[c] - mx) * inv);
    m2 = tr_wave_allreduce_max(m2);
    float s2 = 0.f;
    for (int c = lane; c < C; c += TR_WAVE) s2 += expf(expf(z[c] - mx) * inv - m2);
    s2 = tr_wave_allreduce(s2);
    const float lse = logf(s2), inv2 = 1.0f / s2;
    const int64_t yl = lab[row];
    const float cw = class_w[yl];
    const float gsc = cw * scale;
    float dot = 0.f;
    for (int c = lane; c < C; c += TR_WAVE) {
      const float S = expf(z[c] - mx) * inv;
      const float dS = (expf(S - m2) * inv2 - (c == yl ? 1.0f : 0.0f)) * gsc;
      dot = fmaf(dS, S, dot);
      if (c == yl) lsum += (double)cw * (double)(-((S - m2) - lse));
    }
    dot = tr_wave_allreduce(dot);
    for (int c = lane; c < C; c += TR_WAVE) {
      const float S = expf(z[c] - mx) * inv;
      const float dS = (expf(S - m2) * inv2 - (c == yl ? 1.0f : 0.0f)) * gsc;
      z[c] = S * (dS - dot);
    }
  }
  if (MODE == MODE_MNL_TRAIN) {
    lsum = tr_wave_allreduce_d(lsum);
    if (lane == 0) {
      dpart[2 * gw] = lsum;
      dpart[2 * gw + 1] = 0.0;
    }
  }
}

// ==========================================================================================
// K3 two-pass backward: partial column reduction  Gpart[k][c][p] = sum_{n in chunk k} V[n,c] X[n,p]
// (the reference's MmBackward0 X^T . dL/dZ).  Workgroup (stripe s, chunk k): 256 threads,
// each owns CW vectors of columns; the per-row weights V[n, 0..C-1] are wave-uniform scalar
// loads.  Chunks are walked last-first when `reverse` is set so the rows the forward pass
// streamed last (still in the Infinity Cache) are read first.
// ==========================================================================================
template <int C, int CW, int W>
__global__ __launch_bounds__(256) void k_cols(const float* __restrict__ X, int64_t N, int64_t P, int64_t xld,
                                              const float* __restrict__ Vw, int64_t rows_per_chunk,
                                              float* __restrict__ gpart, int reverse,
                                              const int32_t* __restrict__ stop, int64_t ldv, int64_t slab_stride) {
  using V = VecT<W>;
  using VT = typename V::T;
  if (stop != nullptr && *stop != 0) return;
  const int t = threadIdx.x;
  const int64_t PW = P / W;
  const int64_t LDW = xld / W;  // row stride in vectors
  const int64_t k = reverse ? (int64_t)(gridDim.y - 1 - blockIdx.y) : (int64_t)blockIdx.y;
  const int64_t n0 = k * rows_per_chunk;
  const int64_t n1 = n0 + rows_per_chunk < N ? n0 + rows_per_chunk : N;
  int64_t col[CW];
  bool ok[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) {
    const int64_t qq = (int64_t)blockIdx.x * (256 * CW) + j * 256 + t;
    ok[j] = qq < PW;
    col[j] = ok[j] ? qq : PW - 1;
  }
  VT acc[CW][C];
#pragma unroll
  for (int j = 0; j < CW; ++j)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[j][c] = V::zero();

  const VT* Xv = reinterpret_cast<const VT*>(X);
  constexpr int U = (CW * C <= 8) ? 8 : 4;
  int64_t n = n0;
  for (; n + U <= n1; n += U) {
    VT x[U][CW];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < CW; ++j) x[u][j] = ldx(Xv + (n + u) * LDW + col[j]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float v = Vw[(n + u) * ldv + c];
#pragma unroll
        for (int j = 0; j < CW; ++j) V::axpy(v, x[u][j], acc[j][c]);
      }
    }
  }
  for (; n < n1; ++n) {
    VT x[CW];
#pragma unroll
    for (int j = 0; j < CW; ++j) x[j] = ldx(Xv + n * LDW + col[j]);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float v = Vw[n * ldv + c];
#pragma unroll
      for (int j = 0; j < CW; ++j) V::axpy(v, x[j], acc[j][c]);
    }
  }
  VT* gp = reinterpret_cast<VT*>(gpart + k * slab_stride);
#pragma unroll
  for (int j = 0; j < CW; ++j)
    if (ok[j])
#pragma unroll
      for (int c = 0; c < C; ++c) gp[c * PW + col[j]] = acc[j][c];
}

// ==========================================================================================
// K4: fixed-order slab reduction  out[col] = sum_k part[k][col]  (+ scalar partials)
// Summation order (fixed, the same for both layouts below): for q = 0..15 and j = 0..3,
// a_j(q) = sum over rounds t of slab q + 16 j + 64 t (rounds while q + 64 t + 48 < nslabs; the
// remaining slabs q + 64 T + 16 m go into a_0(q)); s_q = (a_0 + a_1) + (a_2 + a_3); out =
// s_0 + s_1 + ... + s_15 left to right.  Workgroup = 16 waves (q = wave).
//   WIDE   (64 vector columns per workgroup): lane = column, the thread forms a_0..a_3 (4 loads
//          in flight); for many columns (enough workgroups to fill the chip).
//   NARROW (16 vector columns per workgroup): lane (c = lane & 15, j = lane >> 4) forms a_j(q)
//          alone, its loads issued four rounds ahead of the in-order adds; for few columns and
//          many slabs (config 3: 512 slabs of 1.6 K floats), where WIDE ran 7 workgroups
//          through 8 dependent load rounds.
// Both write bitwise-identical sums.  Block 0 also reduces the per-wave/per-WG fp64 scalar
// partials (loss, bias gradient) and writes them into the gradient arena.
// ==========================================================================================
template <int W, bool NARROW>
__global__ __launch_bounds__(1024) void k_reduce_slabs(const float* __restrict__ part, int64_t nslabs,
                                                       int64_t ncols, float* __restrict__ out,
                                                       const double* __restrict__ dpart, int64_t nd,
                                                       double loss_scale, float* __restrict__ loss_slot,
                                                       float* __restrict__ bias_slot,
                                                       const float* __restrict__ chain_dphi,
                                                       float* __restrict__ chain_out, int64_t nchain,
                                                       const uint32_t* __restrict__ err,
                                                       const int32_t* __restrict__ stop) {
  using V = VecT<W>;
  using VT = typename V::T;
  constexpr int NWV = 16, NP = 64;
  constexpr int CPW = NARROW ? 16 : TR_WAVE;  // vector columns per workgroup
  __shared__ VT sred[NWV * TR_WAVE];          // NARROW: [4 q + j][c]; WIDE: [q][lane]
  __shared__ double dred[2][NWV];
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int q = threadIdx.x / TR_WAVE;
  const int c = lane & (CPW - 1), j = NARROW ? lane >> 4 : 0;
  const int64_t NCW = ncols / W;
  const int64_t colv = (int64_t)blockIdx.x * CPW + c;
  const VT* pv = reinterpret_cast<const VT*>(part);
  const int64_t T = nslabs > q + 48 ? (nslabs - q - 48 + NP - 1) / NP : 0;  // full rounds of wave q
  const int64_t st = (int64_t)NP * NCW;
  if (NARROW) {
    VT a = V::zero();
    if (colv < NCW) {
      const VT* src = pv + (int64_t)(q + 16 * j) * NCW + colv;
      int64_t t = 0;
      for (; t + 4 <= T; t += 4) {
        const VT u0 = src[t * st], u1 = src[(t + 1) * st], u2 = src[(t + 2) * st], u3 = src[(t + 3) * st];
        a = V::add(a, u0);
        a = V::add(a, u1);
        a = V::add(a, u2);
        a = V::add(a, u3);
      }
      for (; t < T; ++t) a = V::add(a, src[t * st]);
      if (j == 0)
        for (int64_t k = q + NP * T; k < nslabs; k += NWV) a = V::add(a, pv[k * NCW + colv]);
    }
    sred[(4 * q + j) * CPW + c] = a;
  } else if (colv < NCW) {
    VT a0 = V::zero(), a1 = V::zero(), a2 = V::zero(), a3 = V::zero();
    const VT* src = pv + (int64_t)q * NCW + colv;
    for (int64_t t = 0; t < T; ++t) {
      const VT u0 = src[t * st];
      const VT u1 = src[t * st + 16 * NCW];
      const VT u2 = src[t * st + 32 * NCW];
      const VT u3 = src[t * st + 48 * NCW];
      a0 = V::add(a0, u0);
      a1 = V::add(a1, u1);
      a2 = V::add(a2, u2);
      a3 = V::add(a3, u3);
    }
    for (int64_t k = q + NP * T; k < nslabs; k += NWV) a0 = V::add(a0, pv[k * NCW + colv]);
    sred[q * TR_WAVE + lane] = V::add(V::add(a0, a1), V::add(a2, a3));
  }
  __syncthreads();
  if (q == 0 && j == 0 && colv < NCW) {
    VT s = V::zero();
#pragma unroll
    for (int qq = 0; qq < NWV; ++qq) {
      const VT sq = NARROW ? V::add(V::add(sred[(4 * qq) * CPW + c], sred[(4 * qq + 1) * CPW + c]),
                                    V::add(sred[(4 * qq + 2) * CPW + c], sred[(4 * qq + 3) * CPW + c]))
                           : sred[qq * TR_WAVE + lane];
      s = qq == 0 ? sq : V::add(s, sq);
    }
    reinterpret_cast<VT*>(out)[colv] = s;
    if (chain_out != nullptr) {  // softplus chain of arena-layout slabs (k_spec_chain) fused
      const float* sv = reinterpret_cast<const float*>(&s);
#pragma unroll
      for (int cc = 0; cc < W; ++cc) {
        const int64_t e = colv * W + cc;
        if (e < nchain) chain_out[e] = sv[cc] * chain_dphi[e];
      }
    }
  }
  if (blockIdx.x == 0 && dpart != nullptr) {
    double s0 = 0.0, s1 = 0.0;
    for (int64_t i = threadIdx.x; i < nd; i += blockDim.x) {
      s0 += dpart[2 * i];
      s1 += dpart[2 * i + 1];
    }
    s0 = tr_wave_allreduce_d(s0);
    s1 = tr_wave_allreduce_d(s1);
    if (lane == 0) {
      dred[0][q] = s0;
      dred[1][q] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double l = 0.0, b = 0.0;
      for (int w = 0; w < NWV; ++w) {
        l += dred[0][w];
        b += dred[1][w];
      }
      *loss_slot = (float)(l * loss_scale);
      if (bias_slot != nullptr) *bias_slot = (float)b;
    }
  }
  // device status slot (after the loss slot): nonzero iff a kernel of this pass failed
  if (blockIdx.x == 0 && threadIdx.x == 0 && loss_slot != nullptr)
    loss_slot[1] = (err != nullptr && err[0] != 0u) ? 1.0f : 0.0f;
}

// ==========================================================================================
// K5: MTTKRP + softplus chain: grad[A_f][i, r] = dphi * w_r * sum_{e: i_f(e)=i} G[e] prod_{g!=f} Phi_g[i_g(e), r]
// (the autograd of cp_to_tensor + non_neg_fn, standard…py:462).  One workgroup per factor row.
// The NO "other" modes are walked with a division-free mixed-radix counter whose fastest digit
// is the mode with the smallest dense stride (most contiguous G reads); U gathers of G are
// issued before they are consumed (G is L2-resident, so the loop is latency-, not
// bandwidth-bound); factor columns sit in LDS; fixed-order block reduction over rank columns.
// ==========================================================================================
template <int RMAX, int NO, bool USE_LDS>
__global__ __launch_bounds__(256) void k_mttkrp(FactorSet fs, const float* __restrict__ phi,
                                                const float* __restrict__ dphi,
                                                const float* __restrict__ w,
                                                const float* __restrict__ G, float* __restrict__ out,
                                                const int32_t* __restrict__ stop) {
  constexpr int U = RMAX >= 64 ? 4 : 8;
  constexpr int NOD = NO > 0 ? NO : 1;
  extern __shared__ __attribute__((aligned(16))) float sphi[];
  __shared__ float red[4][RMAX];
  __shared__ float sw[RMAX];
  if (stop != nullptr && *stop != 0) return;
  const int R = fs.rank;
  const int nf = fs.nf;
  // rank tile of this workgroup: columns [rt0, rt0 + Rt) (grid.y tiles a rank beyond RMAX)
  const int rt0 = (int)blockIdx.y * RMAX;
  const int Rt = R - rt0 < RMAX ? R - rt0 : RMAX;
  int b = blockIdx.x;
  int f = 0;
  while (f < nf - 1 && b >= (int)fs.dim[f]) {
    b -= (int)fs.dim[f];
    ++f;
  }
  const int i = b;
  // The factors are staged in LDS with an odd row stride S (lanes walking consecutive rows hit
  // distinct banks; stride R = 8 / 16 put 8 / 16 lanes on one bank), and USE_LDS is a template
  // parameter so that the reads compile to ds_read rather than generic flat loads.
  const int S = USE_LDS ? (R | 1) : R;
  const float* F = phi;
  if constexpr (USE_LDS) {
    for (int k = threadIdx.x; k < (int)fs.nfelem; k += blockDim.x) {
      const int g = tr_factor_of(fs, k);
      int rows_before = 0;
      for (int h = 0; h < g; ++h) rows_before += (int)fs.dim[h];
      const int within = k - (int)fs.off[g];
      sphi[(rows_before + within / R) * S + within % R] = phi[k];
    }
    F = sphi;
  }
  if (threadIdx.x < RMAX) sw[threadIdx.x] = (int)threadIdx.x < Rt ? w[rt0 + threadIdx.x] : 0.f;
  __syncthreads();

  // other modes ordered by decreasing dense stride (digit NO-1 = most contiguous), host-sorted
  int od[NOD], ostr[NOD], ooff[NOD];
#pragma unroll
  for (int k = 0; k < NOD; ++k) {
    if (k < NO) {
      const int g = fs.others[f][k];
      od[k] = (int)fs.dim[g];
      ostr[k] = (int)fs.stride[g];
      if (USE_LDS) {
        int rows_before = 0;
        for (int h = 0; h < g; ++h) rows_before += (int)fs.dim[h];
        ooff[k] = rows_before * S;
      } else {
        ooff[k] = (int)fs.off[g];
      }
    } else {
      od[k] = 1;
      ostr[k] = 0;
      ooff[k] = 0;
    }
  }
  const int nother = (int)(fs.total / fs.dim[f]);
  const int base = i * (int)fs.stride[f];
  // per-thread digit state of j = threadIdx.x, and the stride 256 in the same radix
  int idx[NOD], sd[NOD];
  {
    int rem = threadIdx.x, rs = blockDim.x;
#pragma unroll
    for (int k = NOD - 1; k >= 0; --k) {
      idx[k] = rem % od[k];
      rem /= od[k];
      sd[k] = rs % od[k];
      rs /= od[k];
    }
  }
  auto advance = [&]() {
    int carry = 0;
#pragma unroll
    for (int k = NOD - 1; k >= 0; --k) {
      int d = idx[k] + sd[k] + carry;
      carry = 0;
      while (d >= od[k]) {
        d -= od[k];
        ++carry;
      }
      idx[k] = d;
    }
  };
  float acc[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) acc[r] = 0.f;
  for (int j0 = threadIdx.x; j0 < nother; j0 += U * (int)blockDim.x) {
    float gv[U];
    int frow[U][NOD];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = j0 + u * (int)blockDim.x < nother;
      int pos = base;
#pragma unroll
      for (int k = 0; k < NOD; ++k) {
        pos += idx[k] * ostr[k];
        frow[u][k] = ooff[k] + idx[k] * S + rt0;
      }
      gv[u] = ok ? G[pos] : 0.f;
      advance();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < RMAX; ++r) {
        if (r < Rt) {
          float prod = sw[r];
#pragma unroll
          for (int k = 0; k < NO; ++k) prod *= F[frow[u][k] + r];
          acc[r] = fmaf(gv[u], prod, acc[r]);
        }
      }
    }
  }
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int q = threadIdx.x / TR_WAVE;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    if (r < Rt) {
      const float v = tr_wave_allreduce(acc[r]);
      if (lane == 0) red[q][r] = v;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < Rt) {
    const int r = threadIdx.x;
    const float s2 = ((red[0][r] + red[1][r]) + red[2][r]) + red[3][r];
    const int64_t e = fs.off[f] + (int64_t)i * R + rt0 + r;
    out[e] = s2 * dphi[e];
  }
}

}  // namespace tr

// ==========================================================================================
// Host-side launch helpers (template dispatch)
// ==========================================================================================
namespace tr {

static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch_prep_factors(const FactorSet& fs, const float* params, float beta, float thr,
                               float* phi, float* dphi, const int32_t* stop, hipStream_t st) {
  hipLaunchKernelGGL(k_prep_factors, dim3(cdiv(fs.nfelem, 256)), dim3(256), 0, st, fs, params, beta,
                     thr, phi, dphi, stop);
  return hipGetLastError();
}

static const int64_t kLdsFactorLimit = 12288;  // floats of factor columns staged in LDS (48 KiB)

hipError_t launch_build_dense(const FactorSet& fs, const float* params, float beta, float thr, float* phi,
                              float* dphi, const float* w, float* dense, const int32_t* stop, hipStream_t st) {
  const int use_lds = fs.nfelem <= kLdsFactorLimit;
  if (!use_lds) {
    hipError_t e = launch_prep_factors(fs, params, beta, thr, phi, dphi, stop, st);
    if (e != hipSuccess) return e;
  }
  int64_t blocks = cdiv(fs.total, 256);
  if (blocks > 1024) blocks = 1024;
  const size_t lds = use_lds ? (size_t)fs.nfelem * sizeof(float) : 0;
  hipLaunchKernelGGL(k_build_dense, dim3((unsigned)blocks), dim3(256), lds, st, fs, params, beta, thr, phi, dphi,
                     w, dense, use_lds, stop);
  return hipGetLastError();
}

// ---- fused linear --------------------------------------------------------------------------
// Instantiated (T, CH) pairs: every P = 4*T*CH whose B fits LDS (P <= 40704 floats) and whose
// registers fit (T = 512 spills above CH = 16, T = 1024 at CH = 8: prepare_linear_fused rejects
// it); any other P runs the next pair up, padded (choose_fused in tr_api.hip; <= 25 % padding).
#define TR_FUSED_LIST(X) \
  X(64, 1) X(64, 2) X(64, 3) X(64, 4) X(64, 5) X(64, 6) X(64, 7) X(64, 8) X(64, 12) X(64, 16)           \
  X(128, 1) X(128, 2) X(128, 3) X(128, 4) X(128, 5) X(128, 6) X(128, 7) X(128, 8) X(128, 12) X(128, 16) \
  X(256, 1) X(256, 2) X(256, 3) X(256, 4) X(256, 5) X(256, 6) X(256, 7) X(256, 8) X(256, 12) X(256, 16) \
  X(512, 1) X(512, 2) X(512, 3) X(512, 4) X(512, 5) X(512, 6) X(512, 7) X(512, 8) X(512, 9) X(512, 10)  \
  X(512, 11) X(512, 12) X(512, 13) X(512, 14) X(512, 15) X(512, 16)                                     \
  X(1024, 1) X(1024, 2) X(1024, 3) X(1024, 4) X(1024, 5) X(1024, 6) X(1024, 7) X(1024, 8)

template <int T, int CH>
static hipError_t fused_launch_t(int grid, const float* X, int64_t N, int64_t P, int64_t xld, const float* B,
                                 const float* bias, const float* y, float scale, float* gpart,
                                 double* dpart, float* yhat, int64_t rpw, int reverse,
                                 const int32_t* stop, hipStream_t st) {
  const size_t lds = (size_t)T * CH * 4 * sizeof(float) + 2 * (T / TR_WAVE) * sizeof(float);  // B padded to 4 T CH
  if (P > 4 * (int64_t)T * CH) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_linear_fused<T, CH>), dim3(grid), dim3(T), lds, st, X, N, P, xld, B, bias, y,
                     scale, gpart, dpart, yhat, rpw, reverse, stop);
  return hipGetLastError();
}

typedef hipError_t (*fused_fn_t)(int, const float*, int64_t, int64_t, int64_t, const float*, const float*,
                                 const float*, float, float*, double*, float*, int64_t, int,
                                 const int32_t*, hipStream_t);
struct FusedEntry {
  int T, CH;
  const void* kernel;
  fused_fn_t launch;
};
#define TR_FUSED_ENTRY(TT, CC) \
  {TT, CC, reinterpret_cast<const void*>(&k_linear_fused<TT, CC>), &fused_launch_t<TT, CC>},
static const FusedEntry kFused[] = {TR_FUSED_LIST(TR_FUSED_ENTRY)};
static const int kNumFused = sizeof(kFused) / sizeof(kFused[0]);

static const FusedEntry* find_fused(int T, int CH) {
  for (int i = 0; i < kNumFused; ++i)
    if (kFused[i].T == T && kFused[i].CH == CH) return &kFused[i];
  return nullptr;
}

bool linear_fused_supported(int T, int CH) { return find_fused(T, CH) != nullptr; }

hipError_t launch_linear_fused(int T, int CH, int grid, const float* X, int64_t N, int64_t P, int64_t xld,
                               const float* B, const float* bias, const float* y, float scale,
                               float* gpart, double* dpart, float* yhat, int64_t rows_per_wg,
                               int reverse, const int32_t* stop, hipStream_t st) {
  const FusedEntry* e = find_fused(T, CH);
  if (e == nullptr) return hipErrorInvalidValue;
  return e->launch(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, yhat, rows_per_wg, reverse, stop, st);
}

// Sets the dynamic-LDS limit and reports spill-free occupancy (workgroups per CU; 0 = unusable).
hipError_t prepare_linear_fused(int T, int CH, size_t lds_bytes, int* wg_per_cu) {
  *wg_per_cu = 0;
  const FusedEntry* e = find_fused(T, CH);
  if (e == nullptr) return hipErrorInvalidValue;
  hipError_t err = hipFuncSetAttribute(e->kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  if (err != hipSuccess) return err;
  hipFuncAttributes attr;
  err = hipFuncGetAttributes(&attr, e->kernel);
  if (err != hipSuccess) return err;
  if (attr.localSizeBytes > 0) return hipSuccess;  // spills: reject
  int nb = 0;
  err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, e->kernel, T, lds_bytes);
  if (err != hipSuccess) return err;
  *wg_per_cu = nb;
  return hipSuccess;
}

// ---- single pass, short rows ---------------------------------------------------------------
// U = 4 blocks in flight per wave (2: 0-10 points lower, 8: 4-11 lower; DESIGN.md k_linear_packed)
template <int PQ>
static hipError_t packed_launch_t(int grid, const float* X, int64_t N, int64_t P, int64_t xld, const float* B,
                                  const float* bias, const float* y, float scale, float* gpart, double* dpart,
                                  int64_t rpw, int reverse, const int32_t* stop, hipStream_t st) {
  if (P < 1 || P > 4 * PQ) return hipErrorInvalidValue;
  if ((int64_t)(TR_WAVE / PQ) * xld * 4 + P * 4 > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_linear_packed<PQ, 4>), dim3(grid), dim3(256), 0, st, X, N, P, xld, B, bias, y, scale, gpart,
                     dpart, rpw, reverse, stop);
  return hipGetLastError();
}
template <int PQ>
static const void* packed_kernel_t() {
  return reinterpret_cast<const void*>(&k_linear_packed<PQ, 4>);
}
static const void* packed_kernel(int PQ) {
  switch (PQ) {
    case 1: return packed_kernel_t<1>();
    case 2: return packed_kernel_t<2>();
    case 4: return packed_kernel_t<4>();
    case 8: return packed_kernel_t<8>();
    case 16: return packed_kernel_t<16>();
    case 32: return packed_kernel_t<32>();
  }
  return nullptr;
}
int linear_packed_pq(int64_t P) {
  if (P < 1 || P > 128) return 0;
  int pq = 1;
  while (4 * pq < P) pq *= 2;
  return pq;
}
hipError_t launch_linear_packed(int PQ, int grid, const float* X, int64_t N, int64_t P, int64_t xld, const float* B,
                                const float* bias, const float* y, float scale, float* gpart, double* dpart,
                                int64_t rows_per_wg, int reverse, const int32_t* stop, hipStream_t st) {
  switch (PQ) {
    case 1: return packed_launch_t<1>(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_wg, reverse, stop, st);
    case 2: return packed_launch_t<2>(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_wg, reverse, stop, st);
    case 4: return packed_launch_t<4>(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_wg, reverse, stop, st);
    case 8: return packed_launch_t<8>(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_wg, reverse, stop, st);
    case 16: return packed_launch_t<16>(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_wg, reverse, stop, st);
    case 32: return packed_launch_t<32>(grid, X, N, P, xld, B, bias, y, scale, gpart, dpart, rows_per_wg, reverse, stop, st);
  }
  return hipErrorInvalidValue;
}
// spill-free occupancy of the short-row pass (workgroups of 256 per CU; 0 = unusable)
hipError_t prepare_linear_packed(int PQ, int* wg_per_cu) {
  *wg_per_cu = 0;
  const void* k = packed_kernel(PQ);
  if (k == nullptr) return hipErrorInvalidValue;
  hipFuncAttributes attr;
  hipError_t err = hipFuncGetAttributes(&attr, k);
  if (err != hipSuccess) return err;
  if (attr.localSizeBytes > 0) return hipSuccess;
  int nb = 0;
  err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0);
  if (err != hipSuccess) return err;
  *wg_per_cu = nb;
  return hipSuccess;
}

// ---- two-pass forward rows -----------------------------------------------------------------
int rows_rb(int C) { return C == 1 ? 8 : 4; }
int cols_cw(int C) { return C == 1 ? 4 : (C == 2 ? 2 : 1); }
bool rows_supported(int C) { return C >= 1 && C <= 16; }
int64_t rows_num_waves(int C, int64_t N) { return (N + rows_rb(C) - 1) / rows_rb(C); }

template <int C, int MODE, int W>
static hipError_t rows_launch_t(const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt, const float* bias,
                                const void* target, const float* class_w, float scale, float* out,
                                double* dpart, float* yhat, const int32_t* stop, hipStream_t st) {
  constexpr int RB = (C == 1) ? 8 : 4;
  const int64_t waves = (N + RB - 1) / RB;
  const unsigned grid = cdiv(waves, 4);
  hipLaunchKernelGGL((k_rows<C, RB, MODE, W>), dim3(grid), dim3(256), 0, st, X, N, P, xld, Bt, bias, target,
                     class_w, scale, out, dpart, yhat, stop, (int64_t)C);
  return hipGetLastError();
}

template <int C>
static hipError_t rows_launch_c(int mode, int W, const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt,
                                const float* bias, const void* target, const float* class_w, float scale,
                                float* out, double* dpart, float* yhat, const int32_t* stop,
                                hipStream_t st) {
#define TR_ROWS(MODE, WW) \
  rows_launch_t<C, MODE, WW>(X, N, P, xld, Bt, bias, target, class_w, scale, out, dpart, yhat, stop, st)
  if (C == 1 && mode == MODE_LIN_TRAIN) return W == 4 ? TR_ROWS(MODE_LIN_TRAIN, 4) : TR_ROWS(MODE_LIN_TRAIN, 1);
  if (C == 1 && mode == MODE_LIN_PRED) return W == 4 ? TR_ROWS(MODE_LIN_PRED, 4) : TR_ROWS(MODE_LIN_PRED, 1);
  if (mode == MODE_MNL_TRAIN) return W == 4 ? TR_ROWS(MODE_MNL_TRAIN, 4) : TR_ROWS(MODE_MNL_TRAIN, 1);
  if (mode == MODE_MNL_PRED) return W == 4 ? TR_ROWS(MODE_MNL_PRED, 4) : TR_ROWS(MODE_MNL_PRED, 1);
#undef TR_ROWS
  return hipErrorInvalidValue;
}

#define TR_C_CASES(CALL) \
  switch (C) {           \
    case 1: return CALL(1);   case 2: return CALL(2);   case 3: return CALL(3);   case 4: return CALL(4);   \
    case 5: return CALL(5);   case 6: return CALL(6);   case 7: return CALL(7);   case 8: return CALL(8);   \
    case 9: return CALL(9);   case 10: return CALL(10); case 11: return CALL(11); case 12: return CALL(12); \
    case 13: return CALL(13); case 14: return CALL(14); case 15: return CALL(15); case 16: return CALL(16); \
    default: break;      \
  }

hipError_t launch_rows(int C, int mode, int W, const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt,
                       const float* bias, const void* target, const float* class_w, float scale,
                       float* out, double* dpart, float* yhat, const int32_t* stop, hipStream_t st) {
#define TR_CALL_ROWS(CC) \
  rows_launch_c<CC>(mode, W, X, N, P, xld, Bt, bias, target, class_w, scale, out, dpart, yhat, stop, st)
  TR_C_CASES(TR_CALL_ROWS)
#undef TR_CALL_ROWS
  return hipErrorInvalidValue;
}

// ---- multinomial forward on MFMA ------------------------------------------------------------
// row tiles of 16 per wave by row width: one for rows of
// <= 256 floats (more waves for short rows: (16, 16) 0.690 -> 0.590 ms), four from 4096 ((64, 64)
// 0.454 -> 0.394 ms, (128, 64) 0.376 -> 0.366 ms), else two (profiles/r05_mnl_rows_rt.txt)
static int mfma_rt(int64_t P) {
  return P <= 256 ? 1 : (P >= 4096 ? 4 : 2);
}
bool rows_mfma_supported(int C, int64_t P) { return C >= 1 && C <= 16 && P % 32 == 0; }
int64_t rows_mfma_num_waves(int64_t N, int64_t P) { return (N + 16 * mfma_rt(P) - 1) / (16 * mfma_rt(P)); }
template <int RT>
static void rows_mfma_go(int mode, unsigned grid, const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt,
                         int C, const int64_t* lab, const float* class_w, float scale, float* out, double* dpart,
                         const int32_t* stop, hipStream_t st) {
  if (mode == MODE_MNL_TRAIN)
    hipLaunchKernelGGL((k_rows_mfma<MODE_MNL_TRAIN, RT>), dim3(grid), dim3(256), 0, st, X, N, P, xld, Bt, C, lab,
                       class_w, scale, out, dpart, stop, (int64_t)C);
  else
    hipLaunchKernelGGL((k_rows_mfma<MODE_MNL_PRED, RT>), dim3(grid), dim3(256), 0, st, X, N, P, xld, Bt, C, lab,
                       class_w, scale, out, dpart, stop, (int64_t)C);
}

hipError_t launch_rows_mfma(int mode, const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt, int C,
                            const int64_t* lab, const float* class_w, float scale, float* out, double* dpart,
                            const int32_t* stop, hipStream_t st) {
  const int64_t waves = rows_mfma_num_waves(N, P);
  const unsigned grid = cdiv(waves, 4);
  if (mode != MODE_MNL_TRAIN && mode != MODE_MNL_PRED) return hipErrorInvalidValue;
  if (mfma_rt(P) == 1)
    rows_mfma_go<1>(mode, grid, X, N, P, xld, Bt, C, lab, class_w, scale, out, dpart, stop, st);
  else if (mfma_rt(P) == 4)
    rows_mfma_go<4>(mode, grid, X, N, P, xld, Bt, C, lab, class_w, scale, out, dpart, stop, st);
  else
    rows_mfma_go<2>(mode, grid, X, N, P, xld, Bt, C, lab, class_w, scale, out, dpart, stop, st);
  return hipGetLastError();
}

// ---- two-pass backward columns -------------------------------------------------------------
template <int C, int W>
static hipError_t cols_launch_t(int64_t nstripes, int64_t nchunks, const float* X, int64_t N, int64_t P, int64_t xld,
                                const float* V, int64_t rpc, float* gpart, int reverse,
                                const int32_t* stop, hipStream_t st, int64_t ldv = C, int64_t slab_stride = -1) {
  constexpr int CW = (C == 1) ? 4 : (C == 2 ? 2 : 1);
  hipLaunchKernelGGL((k_cols<C, CW, W>), dim3((unsigned)nstripes, (unsigned)nchunks), dim3(256), 0, st,
                     X, N, P, xld, V, rpc, gpart, reverse, stop, ldv, slab_stride < 0 ? (int64_t)C * P : slab_stride);
  return hipGetLastError();
}

hipError_t launch_cols(int C, int W, int64_t nstripes, int64_t nchunks, const float* X, int64_t N,
                       int64_t P, int64_t xld, const float* V, int64_t rows_per_chunk, float* gpart, int reverse,
                       const int32_t* stop, hipStream_t st) {
#define TR_CALL_COLS(CC)                                                                           \
  (W == 4 ? cols_launch_t<CC, 4>(nstripes, nchunks, X, N, P, xld, V, rows_per_chunk, gpart, reverse, stop, st) \
          : cols_launch_t<CC, 1>(nstripes, nchunks, X, N, P, xld, V, rows_per_chunk, gpart, reverse, stop, st))
  TR_C_CASES(TR_CALL_COLS)
#undef TR_CALL_COLS
  return hipErrorInvalidValue;
}

// ---- wide-class multinomial path (C > 16) ------------------------------------------------------
int wide_class_tile(void) { return 16; }

template <int CT, int W>
static hipError_t logits_tile_t(const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt, float* Z,
                                int64_t ldo, const int32_t* stop, hipStream_t st) {
  const int64_t waves = (N + 3) / 4;
  hipLaunchKernelGGL((k_rows<CT, 4, MODE_MNL_LOGITS, W>), dim3(cdiv(waves, 4)), dim3(256), 0, st, X, N, P, xld, Bt,
                     nullptr, nullptr, nullptr, 0.f, Z, nullptr, nullptr, stop, ldo);
  return hipGetLastError();
}

hipError_t launch_mnl_logits(int C, int mfma, int W, const float* X, int64_t N, int64_t P, int64_t xld,
                             const float* Bt, float* Z, const int32_t* stop, hipStream_t st) {
  const int ntiles = (C + 15) / 16;
  if (mfma) {  // every class tile in one launch (grid.y); Bt padded to 16 * ntiles class rows
    if (P % 32 != 0) return hipErrorInvalidValue;
    const int64_t waves = (N + 31) / 32;  // two row tiles per wave
    hipLaunchKernelGGL((k_rows_mfma<MODE_MNL_LOGITS, 2>), dim3(cdiv(waves, 4), (unsigned)ntiles), dim3(256), 0,
                       st, X, N, P, xld, Bt, C, nullptr, nullptr, 0.f, Z, nullptr, stop, (int64_t)C);
    return hipGetLastError();
  }
  for (int t = 0; t < ntiles; ++t) {
    const int CT = C - 16 * t < 16 ? C - 16 * t : 16;
    const float* Bt_t = Bt + (int64_t)16 * t * P;
    float* Z_t = Z + 16 * t;
    hipError_t e = hipErrorInvalidValue;
#define TR_CALL_LOGITS(CC) \
  (W == 4 ? logits_tile_t<CC, 4>(X, N, P, xld, Bt_t, Z_t, C, stop, st) : logits_tile_t<CC, 1>(X, N, P, xld, Bt_t, Z_t, C, stop, st))
    switch (CT) {
      case 1: e = TR_CALL_LOGITS(1); break;   case 2: e = TR_CALL_LOGITS(2); break;
      case 3: e = TR_CALL_LOGITS(3); break;   case 4: e = TR_CALL_LOGITS(4); break;
      case 5: e = TR_CALL_LOGITS(5); break;   case 6: e = TR_CALL_LOGITS(6); break;
      case 7: e = TR_CALL_LOGITS(7); break;   case 8: e = TR_CALL_LOGITS(8); break;
      case 9: e = TR_CALL_LOGITS(9); break;   case 10: e = TR_CALL_LOGITS(10); break;
      case 11: e = TR_CALL_LOGITS(11); break; case 12: e = TR_CALL_LOGITS(12); break;
      case 13: e = TR_CALL_LOGITS(13); break; case 14: e = TR_CALL_LOGITS(14); break;
      case 15: e = TR_CALL_LOGITS(15); break; default: e = TR_CALL_LOGITS(16); break;
    }
#undef TR_CALL_LOGITS
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

static const int64_t kSoftmaxWaves = 4096;
int64_t softmax_rows_num_waves(int64_t N) { return N < kSoftmaxWaves ? (N > 0 ? N : 1) : kSoftmaxWaves; }

hipError_t launch_softmax_rows(int mode, int C, float* Z, int64_t N, const int64_t* lab, const float* class_w,
                               float scale, float* out, double* dpart, const int32_t* stop, hipStream_t st) {
  const int64_t waves = softmax_rows_num_waves(N);
  const unsigned grid = cdiv(waves, 4);  // 4 waves per workgroup; dpart holds 4 * grid entries
  if (mode == MODE_MNL_TRAIN)
    hipLaunchKernelGGL(k_softmax_rows<MODE_MNL_TRAIN>, dim3(grid), dim3(256), 0, st, Z, N, C, lab, class_w, scale,
                       out, dpart, stop);
  else if (mode == MODE_MNL_PRED)
    hipLaunchKernelGGL(k_softmax_rows<MODE_MNL_PRED>, dim3(grid), dim3(256), 0, st, Z, N, C, lab, class_w, scale,
                       out, dpart, stop);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_cols_wide(int C, int W, int64_t nstripes, int64_t nchunks, const float* X, int64_t N, int64_t P,
                            int64_t xld, const float* V, int64_t rows_per_chunk, float* gpart, int reverse,
                            const int32_t* stop, hipStream_t st) {
  // class tiles of 16: X is read once per tile; the slabs keep the (class, feature) layout of C
  for (int t = 0; t * 16 < C; ++t) {
    const int CT = C - 16 * t < 16 ? C - 16 * t : 16;
    const float* Vt = V + 16 * t;
    float* gt = gpart + (int64_t)16 * t * P;
    const int64_t ss = (int64_t)C * P;
    hipError_t e = hipErrorInvalidValue;
#define TR_CALL_COLSW(CC)                                                                                   \
  (W == 4 ? cols_launch_t<CC, 4>(nstripes, nchunks, X, N, P, xld, Vt, rows_per_chunk, gt, reverse, stop, st, C, ss) \
          : cols_launch_t<CC, 1>(nstripes, nchunks, X, N, P, xld, Vt, rows_per_chunk, gt, reverse, stop, st, C, ss))
    switch (CT) {
      case 1: e = TR_CALL_COLSW(1); break;   case 2: e = TR_CALL_COLSW(2); break;
      case 3: e = TR_CALL_COLSW(3); break;   case 4: e = TR_CALL_COLSW(4); break;
      case 5: e = TR_CALL_COLSW(5); break;   case 6: e = TR_CALL_COLSW(6); break;
      case 7: e = TR_CALL_COLSW(7); break;   case 8: e = TR_CALL_COLSW(8); break;
      case 9: e = TR_CALL_COLSW(9); break;   case 10: e = TR_CALL_COLSW(10); break;
      case 11: e = TR_CALL_COLSW(11); break; case 12: e = TR_CALL_COLSW(12); break;
      case 13: e = TR_CALL_COLSW(13); break; case 14: e = TR_CALL_COLSW(14); break;
      case 15: e = TR_CALL_COLSW(15); break; default: e = TR_CALL_COLSW(16); break;
    }
#undef TR_CALL_COLSW
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---- slab reduction --------------------------------------------------------------------------
hipError_t launch_reduce_slabs(int W, const float* part, int64_t nslabs, int64_t ncols, float* out,
                               const double* dpart, int64_t nd, double loss_scale, float* loss_slot,
                               float* bias_slot, const int32_t* stop, hipStream_t st, const float* chain_dphi,
                               float* chain_out, int64_t nchain, const uint32_t* err) {
  // NARROW when the wide layout would leave most CUs idle (fewer than 128 workgroups)
  const bool narrow = cdiv(ncols / W, TR_WAVE) < 128;
  const unsigned grid = cdiv(ncols / W, narrow ? 16 : TR_WAVE);
#define TR_RED(WW, NN)                                                                                      \
  hipLaunchKernelGGL((k_reduce_slabs<WW, NN>), dim3(grid), dim3(1024), 0, st, part, nslabs, ncols, out, dpart, \
                     nd, loss_scale, loss_slot, bias_slot, chain_dphi, chain_out, nchain, err, stop)
  if (W == 4) {
    if (narrow)
      TR_RED(4, true);
    else
      TR_RED(4, false);
  } else if (narrow) {
    TR_RED(1, true);
  } else {
    TR_RED(1, false);
  }
#undef TR_RED
  return hipGetLastError();
}

// ---- MTTKRP -----------------------------------------------------------------------------------
template <int RMAX>
static hipError_t mttkrp_launch_r(const FactorSet& fs, const float* phi, const float* dphi, const float* w,
                                  const float* G, float* grad, int use_lds, const int32_t* stop, hipStream_t st,
                                  dim3 grid, size_t lds) {
  const dim3 block(256);
#define TR_MTT(NO)                                                                                      \
  if (use_lds)                                                                                          \
    hipLaunchKernelGGL((k_mttkrp<RMAX, NO, true>), grid, block, lds, st, fs, phi, dphi, w, G, grad, stop); \
  else                                                                                                  \
    hipLaunchKernelGGL((k_mttkrp<RMAX, NO, false>), grid, block, lds, st, fs, phi, dphi, w, G, grad, stop)
  switch (fs.nf - 1) {
    case 0: TR_MTT(0); break;
    case 1: TR_MTT(1); break;
    case 2: TR_MTT(2); break;
    case 3: TR_MTT(3); break;
    case 4: TR_MTT(4); break;
    case 5: TR_MTT(5); break;
    case 6: TR_MTT(6); break;
    default: TR_MTT(7); break;
  }
#undef TR_MTT
  return hipGetLastError();
}

hipError_t launch_mttkrp(const FactorSet& fs, const float* phi, const float* dphi, const float* w,
                         const float* G, float* grad, const int32_t* stop, hipStream_t st, float* part,
                         int64_t part_cap) {
  if (mttkrp2_supported(fs)) return launch_mttkrp2(fs, phi, dphi, w, G, grad, stop, st);
  const char* m3e = std::getenv("TR_MTTKRP3");  // 0: the general k_mttkrp for three factors too
  const bool m3 = m3e == nullptr || m3e[0] != '0';
  if (m3 && part != nullptr && mttkrp3_supported(fs, part_cap))
    return launch_mttkrp3(fs, phi, dphi, w, G, grad, part, part_cap, stop, st);
  int64_t rows = 0;
  for (int f = 0; f < fs.nf; ++f) rows += fs.dim[f];
  const int64_t padded = rows * (fs.rank | 1);  // odd LDS row stride (k_mttkrp)
  const int use_lds = padded <= kLdsFactorLimit;
  const size_t lds = use_lds ? (size_t)padded * sizeof(float) : 0;
  const dim3 grid((unsigned)rows, (unsigned)((fs.rank + 63) / 64));  // rank tiles of 64 beyond rank 64
  if (fs.rank <= 8) return mttkrp_launch_r<8>(fs, phi, dphi, w, G, grad, use_lds, stop, st, grid, lds);
  if (fs.rank <= 16) return mttkrp_launch_r<16>(fs, phi, dphi, w, G, grad, use_lds, stop, st, grid, lds);
  if (fs.rank <= 32) return mttkrp_launch_r<32>(fs, phi, dphi, w, G, grad, use_lds, stop, st, grid, lds);
  return mttkrp_launch_r<64>(fs, phi, dphi, w, G, grad, use_lds, stop, st, grid, lds);
}

}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_kernels() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_build_dense));
}
}  // namespace tr
