// tr_fp64.hip — the linear CP model in float64 (CP_linear_regression(..., dtype=torch.float64),
// standard_tensor_regression.py:206; the reference's own KAT-1, demo_TensorRegression.ipynb, is an
// fp64 LBFGS fit).  Same pipeline as the fp32 two-pass path, in double on the VALU (gfx950 has
// no f64 MFMA path worth the operand shuffles for a GEMV; X streams at HBM rate either way):
//
//   k64_prep    softplus / softplus' of flagged factors (non_neg_fn, :53-85), bias copied
//   k64_dense   B = (Phi_0 * w) @ KR(Phi_1..)^T (tensorly cp_to_tensor, called at :124)
//   k64_rows    y_hat_n = <X_n, B> + bias, residual r_n = 2 (y_hat_n - y_n) / N (MSELoss mean
//               backward), per-wave (sse, sum r) partials; predict mode writes y_hat
//   k64_cols    G partial slabs: Gpart[k][p] = sum_{n in chunk k} r_n X[n, p]  (X^T r, the
//               reference's MmBackward0)
//   k64_reduce  slabs summed in index order; block 0: data loss and bias gradient
//   k64_mttkrp  dPhi_f[i, r] = dphi * w_r sum_j G[i, j] prod_{g != f} Phi_g[., r]  (cp_to_tensor
//               backward), chained through softplus'
//   k64_update  L2_penalty (:180-196) gradient + torch.optim.Adam / AMSGrad (torch 2.10
//               _single_tensor_adam, fp64 tensors: python-float scalars stay double) + the
//               loss record and plateau test, or the LBFGS closure's total gradient / loss
// Every reduction is a fixed-order tree: bitwise reproducible.
#include <hip/hip_runtime.h>

#include <cstring>

#include "tr_common.h"
#include "tr_fp64.h"

namespace tr {

__device__ __forceinline__ double d_softplus(double a, double beta, double thr) {
  const double ab = a * beta;
  return ab > thr ? a : log1p(exp(ab)) / beta;
}
__device__ __forceinline__ double d_softplus_grad(double a, double beta, double thr) {
  const double ab = a * beta;
  if (ab > thr) return 1.0;
  const double z = exp(ab);
  return z / (z + 1.0);
}
__device__ __forceinline__ double d_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int d_factor_of(const FactorSet& fs, int64_t e) {
  int f = 0;
#pragma unroll
  for (int g = 1; g < TR_MAXF; ++g)
    if (g < fs.nf && e >= fs.off[g]) f = g;
  return f;
}

__global__ __launch_bounds__(256) void k64_prep(FactorSet fs, const double* __restrict__ params, double beta,
                                                double thr, double* __restrict__ phi, double* __restrict__ dphi,
                                                const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < fs.nfelem; e += (int64_t)gridDim.x * blockDim.x) {
    const double a = params[e];
    if (fs.nonneg[d_factor_of(fs, e)]) {
      phi[e] = d_softplus(a, beta, thr);
      dphi[e] = d_softplus_grad(a, beta, thr);
    } else {
      phi[e] = a;
      dphi[e] = 1.0;
    }
  }
}

__global__ __launch_bounds__(256) void k64_dense(FactorSet fs, const double* __restrict__ F,
                                                 const double* __restrict__ w, double* __restrict__ dense,
                                                 const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int R = fs.rank;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < fs.total; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t idx[TR_MAXF];
    int64_t pos = 0;
#pragma unroll
    for (int f = 0; f < TR_MAXF; ++f)
      if (f < fs.nf) {
        idx[f] = (e / fs.rstride[f]) % fs.dim[f];
        pos += idx[f] * fs.stride[f];
      }
    double s = 0.0;
    if (fs.nf == 1) {
      for (int r = 0; r < R; ++r) s += w[r] * F[fs.off[0] + idx[0] * R + r];
    } else {
      for (int r = 0; r < R; ++r) {
        const double a = F[fs.off[0] + idx[0] * R + r] * w[r];
        double k = F[fs.off[1] + idx[1] * R + r];
        for (int f = 2; f < fs.nf; ++f) k *= F[fs.off[f] + idx[f] * R + r];
        s = fma(a, k, s);
      }
    }
    dense[pos] = s;
  }
}

// one wave per row; PRED: out[n] = y_hat; TRAIN: out[n] = r_n, dpart[wave] = (sse, sum r)
template <int PRED>
__global__ __launch_bounds__(256) void k64_rows(const double* __restrict__ X, int64_t N, int64_t P, int64_t xld,
                                                const double* __restrict__ B, const double* __restrict__ bias_p,
                                                const double* __restrict__ y, double scale, double* __restrict__ out,
                                                double* __restrict__ yhat, double* __restrict__ dpart,
                                                const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const double bias = *bias_p;
  double sse = 0.0, rsum = 0.0;
  for (int64_t n = gw; n < N; n += nw) {
    const double* xr = X + n * xld;
    double a0 = 0.0, a1 = 0.0;
    int64_t p = lane;
    for (; p + 64 < P; p += 128) {
      a0 = fma(xr[p], B[p], a0);
      a1 = fma(xr[p + 64], B[p + 64], a1);
    }
    if (p < P) a0 = fma(xr[p], B[p], a0);
    const double yh = d_wave_sum(a0 + a1) + bias;
    if (PRED) {
      if (lane == 0) out[n] = yh;
      continue;
    }
    const double e = yh - y[n];
    const double rr = e * scale;
    if (lane == 0) {
      out[n] = rr;
      if (yhat != nullptr) yhat[n] = yh;
    }
    sse += e * e;
    rsum += rr;
  }
  if (!PRED && lane == 0) {
    dpart[2 * gw] = sse;
    dpart[2 * gw + 1] = rsum;
  }
}

// Gpart[k][p] = sum_{n in chunk k} r[n] X[n, p]: thread per column, chunk = blockIdx.y
__global__ __launch_bounds__(256) void k64_cols(const double* __restrict__ X, int64_t N, int64_t P, int64_t xld,
                                                const double* __restrict__ r, int64_t rows_per_chunk,
                                                double* __restrict__ gpart, const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t k = blockIdx.y;
  const int64_t n0 = k * rows_per_chunk;
  const int64_t n1 = n0 + rows_per_chunk < N ? n0 + rows_per_chunk : N;
  if (p >= P) return;
  double a0 = 0.0, a1 = 0.0;
  int64_t n = n0;
  for (; n + 1 < n1; n += 2) {
    a0 = fma(r[n], X[n * xld + p], a0);
    a1 = fma(r[n + 1], X[(n + 1) * xld + p], a1);
  }
  if (n < n1) a0 = fma(r[n], X[n * xld + p], a0);
  gpart[k * P + p] = a0 + a1;
}

__global__ __launch_bounds__(256) void k64_reduce(const double* __restrict__ part, int64_t nslabs, int64_t P,
                                                  double* __restrict__ G, const double* __restrict__ dpart,
                                                  int64_t nd, double loss_scale, double* __restrict__ loss_slot,
                                                  double* __restrict__ bias_slot, const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p < P) {
    double s = 0.0;
    for (int64_t k = 0; k < nslabs; ++k) s += part[k * P + p];
    G[p] = s;
  }
  if (blockIdx.x == 0) {
    __shared__ double red[2][4];
    double s0 = 0.0, s1 = 0.0;
    for (int64_t i = threadIdx.x; i < nd; i += 256) {
      s0 += dpart[2 * i];
      s1 += dpart[2 * i + 1];
    }
    s0 = d_wave_sum(s0);
    s1 = d_wave_sum(s1);
    const int q = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][q] = s0;
      red[1][q] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      *loss_slot = (((red[0][0] + red[0][1]) + red[0][2]) + red[0][3]) * loss_scale;
      loss_slot[1] = 0.0;  // device status slot (the fp64 pass has no failure mode)
      if (bias_slot != nullptr) *bias_slot = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
  }
}

// one workgroup per (factor row i, rank tile of 32); threads walk the other modes' index j
__global__ __launch_bounds__(256) void k64_mttkrp(FactorSet fs, const double* __restrict__ phi,
                                                  const double* __restrict__ dphi, const double* __restrict__ w,
                                                  const double* __restrict__ G, double* __restrict__ out,
                                                  const int32_t* __restrict__ stop) {
  constexpr int RT = 32;
  __shared__ double red[4][RT];
  if (stop != nullptr && *stop != 0) return;
  const int R = fs.rank, nf = fs.nf;
  int b = blockIdx.x, f = 0;
  while (f < nf - 1 && b >= (int)fs.dim[f]) {
    b -= (int)fs.dim[f];
    ++f;
  }
  const int i = b;
  const int r0 = blockIdx.y * RT;
  const int Rt = R - r0 < RT ? R - r0 : RT;
  const int64_t nother = fs.total / fs.dim[f];
  double acc[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r] = 0.0;
  for (int64_t j = threadIdx.x; j < nother; j += 256) {
    // decode j over the other modes in row-major order of their dims (the dense layout minus f)
    int64_t rem = j, pos = (int64_t)i * fs.stride[f];
    int64_t row[TR_MAXF];
    for (int g = nf - 1; g >= 0; --g) {
      if (g == f) continue;
      const int64_t ig = rem % fs.dim[g];
      rem /= fs.dim[g];
      row[g] = ig;
      pos += ig * fs.stride[g];
    }
    const double gv = G[pos];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      if (r < Rt) {
        double prod = w[r0 + r];
        for (int g = 0; g < nf; ++g)
          if (g != f) prod *= phi[fs.off[g] + row[g] * R + r0 + r];
        acc[r] = fma(gv, prod, acc[r]);
      }
    }
  }
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    if (r < Rt) {
      const double v = d_wave_sum(acc[r]);
      if (lane == 0) red[q][r] = v;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < Rt) {
    const int r = threadIdx.x;
    const int64_t e = fs.off[f] + (int64_t)i * R + r0 + r;
    out[e] = (((red[0][r] + red[1][r]) + red[2][r]) + red[3][r]) * dphi[e];
  }
}

__global__ __launch_bounds__(1024) void k64_update(FactorSet fs, int n_bias, double* __restrict__ params,
                                                   const double* __restrict__ grad, Update64 ua,
                                                   double* __restrict__ m, double* __restrict__ v,
                                                   double* __restrict__ vmax, double* __restrict__ grad_total_out,
                                                   double* __restrict__ loss_out, double* __restrict__ loss_hist,
                                                   int32_t* __restrict__ stop) {
  __shared__ double wsum[TR_MAXF * 16];
  __shared__ double norms[TR_MAXF];
  if (stop != nullptr && *stop != 0) return;
  const int t = threadIdx.x, lane = t & 63, q = t >> 6, NWV = blockDim.x >> 6;
  const int64_t nfe = fs.nfelem, np = nfe + n_bias;
  if (ua.mode == 0 && stop != nullptr && grad[np + 1] != 0.0) {
    if (t == 0) *stop = TR_STOP_DEVICE_ERROR - (int32_t)ua.iter;
    return;
  }
  {
    double accn[TR_MAXF];
#pragma unroll
    for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.0;
    for (int64_t k = t; k < nfe; k += blockDim.x) {
      const double a = params[k];
      const int f = d_factor_of(fs, k);
#pragma unroll
      for (int g = 0; g < TR_MAXF; ++g)
        if (g == f) accn[g] = fma(a, a, accn[g]);
    }
#pragma unroll
    for (int f = 0; f < TR_MAXF; ++f)
      if (f < fs.nf) {
        const double s = d_wave_sum(accn[f]);
        if (lane == 0) wsum[f * 16 + q] = s;
      }
    __syncthreads();
    if (t < fs.nf) {
      double tot = 0.0;
      for (int k = 0; k < NWV; ++k) tot += wsum[t * 16 + k];
      norms[t] = sqrt(tot);
    }
    __syncthreads();
  }
  const double lam = ua.lambda_l2;
  for (int64_t e = t; e < np; e += blockDim.x) {
    double g = grad[e];
    double p = params[e];
    if (e < nfe) g = g + (lam / (2.0 * norms[d_factor_of(fs, e)])) * (2.0 * p);
    if (ua.mode == 1) {
      grad_total_out[e] = g;
      continue;
    }
    if (ua.weight_decay != 0.0) g = fma(p, ua.weight_decay, g);
    double mm = m[e];
    mm = fma(ua.one_minus_b1, g - mm, mm);
    double vv = v[e] * ua.beta2;
    vv = vv + ua.one_minus_b2 * g * g;
    double den_src = vv;
    if (ua.amsgrad) {
      const double vm = fmax(vmax[e], vv);
      vmax[e] = vm;
      den_src = vm;
    }
    const double denom = sqrt(den_src) / ua.bc2_sqrt + ua.eps;
    p = p + (-ua.step_size) * (mm / denom);
    m[e] = mm;
    v[e] = vv;
    params[e] = p;
  }
  if (t == 0) {
    double l2 = 0.0;
    for (int f = 0; f < fs.nf; ++f) l2 = l2 + norms[f];
    const double total = grad[np] + lam * l2;
    if (loss_out != nullptr) *loss_out = total;
    if (ua.mode == 0 && loss_hist != nullptr) loss_hist[ua.hist_base + ua.iter] = total;
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static inline unsigned cdiv64(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch64_prep_dense(const FactorSet& fs, const double* params, double beta, double thr, double* phi,
                               double* dphi, const double* w, double* dense, const int32_t* stop, hipStream_t st) {
  unsigned b1 = cdiv64(fs.nfelem, 256);
  if (b1 > 256) b1 = 256;
  hipLaunchKernelGGL(k64_prep, dim3(b1), dim3(256), 0, st, fs, params, beta, thr, phi, dphi, stop);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  unsigned b2 = cdiv64(fs.total, 256);
  if (b2 > 2048) b2 = 2048;
  hipLaunchKernelGGL(k64_dense, dim3(b2), dim3(256), 0, st, fs, phi, w, dense, stop);
  return hipGetLastError();
}

int64_t rows64_num_waves(int64_t N) { return N < 4096 ? (N > 0 ? (N + 3) / 4 * 4 : 4) : 4096; }

hipError_t launch64_rows(int pred, const double* X, int64_t N, int64_t P, int64_t xld, const double* B,
                         const double* bias, const double* y, double scale, double* out, double* yhat, double* dpart,
                         const int32_t* stop, hipStream_t st) {
  const unsigned grid = (unsigned)(rows64_num_waves(N) / 4);
  if (pred)
    hipLaunchKernelGGL(k64_rows<1>, dim3(grid), dim3(256), 0, st, X, N, P, xld, B, bias, y, scale, out, yhat, dpart,
                       stop);
  else
    hipLaunchKernelGGL(k64_rows<0>, dim3(grid), dim3(256), 0, st, X, N, P, xld, B, bias, y, scale, out, yhat, dpart,
                       stop);
  return hipGetLastError();
}

hipError_t launch64_cols(const double* X, int64_t N, int64_t P, int64_t xld, const double* r, int64_t nchunks,
                         double* gpart, const int32_t* stop, hipStream_t st) {
  const int64_t rpc = (N + nchunks - 1) / nchunks;
  const int64_t nk = (N + rpc - 1) / rpc;
  hipLaunchKernelGGL(k64_cols, dim3(cdiv64(P, 256), (unsigned)nk), dim3(256), 0, st, X, N, P, xld, r, rpc, gpart,
                     stop);
  return hipGetLastError();
}

hipError_t launch64_reduce(const double* part, int64_t nslabs, int64_t P, double* G, const double* dpart, int64_t nd,
                           double loss_scale, double* loss_slot, double* bias_slot, const int32_t* stop,
                           hipStream_t st) {
  hipLaunchKernelGGL(k64_reduce, dim3(cdiv64(P, 256)), dim3(256), 0, st, part, nslabs, P, G, dpart, nd, loss_scale,
                     loss_slot, bias_slot, stop);
  return hipGetLastError();
}

hipError_t launch64_mttkrp(const FactorSet& fs, const double* phi, const double* dphi, const double* w,
                           const double* G, double* grad, const int32_t* stop, hipStream_t st) {
  int64_t rows = 0;
  for (int f = 0; f < fs.nf; ++f) rows += fs.dim[f];
  hipLaunchKernelGGL(k64_mttkrp, dim3((unsigned)rows, (unsigned)((fs.rank + 31) / 32)), dim3(256), 0, st, fs, phi,
                     dphi, w, G, grad, stop);
  return hipGetLastError();
}

hipError_t launch64_update(const FactorSet& fs, int n_bias, double* params, const double* grad, const Update64& ua,
                           double* m, double* v, double* vmax, double* grad_total_out, double* loss_out,
                           double* loss_hist, int32_t* stop, hipStream_t st) {
  hipLaunchKernelGGL(k64_update, dim3(1), dim3(1024), 0, st, fs, n_bias, params, grad, ua, m, v, vmax, grad_total_out,
                     loss_out, loss_hist, stop);
  return hipGetLastError();
}

}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_fp64() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k64_prep));
}
}  // namespace tr
