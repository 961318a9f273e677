// tr_update.hip — the L2 term + Adam/AMSGrad step of fit_Adam, the loss record and the
// plateau test (k_update, k_converge; one launch each per iteration).
//
//   L2_penalty (standard…py:180-196): sum_k sqrt(sum(A_k^2)) over RAW factors (not squared)
//   d/dA [lambda*sqrt(sum A^2)] = (lambda / (2 ||A||)) * (2 A)     (Sqrt/Pow backward)
//   torch/optim/adam.py _single_tensor_adam (torch 2.10), non-capturable branch.
//   numpy's pairwise summation is restated for np.sum(np.abs(np.diff(...))) (k_converge).
//
// One 1024-thread workgroup: the norms are a dependency of every element, and several
// workgroups could not overwrite a factor before all had read it.  The step is a few thousand
// elements (config 2: 3073, config 5: 8242) and runs right after a pass that streamed GBs, from
// cold caches, so what it costs is memory round trips and instruction-cache misses, not
// bandwidth or arithmetic.  Measured variants (tools/update_bench.hip, after a 1 GiB flush;
// c2 / c3 / c5 parameter counts): the element-by-element loop with a per-element factor search
// and L2 division 8.1 / 6.7 / 16.5 us; all loads of a thread issued up front in fully unrolled
// code 7.7 / 6.2 / 15.4 us (the code no longer fits the instruction cache it starts cold in);
// this kernel 5.6 / 5.2 / 10.9 us: compact rolled loops with two elements per trip (both loads
// in flight), the factor's norm accumulator selected without a branch and its L2 coefficient
// lambda / (2 ||A_f||) computed once.  Thread t sums the factor elements k = t (mod 1024) in
// increasing k, then the wave butterfly and the wave-order LDS sum: the norms, and the whole
// step, are bitwise those of the element-by-element loop.
#include <cstring>

#include "tr_common.h"
#include "tr_kernels.h"

namespace tr {

#ifndef TR_UPD_PROFILE
#define TR_UPD_PROFILE 0  // tools/update_bench.hip only: wall-clock stamps of the phases of k_update
#endif
#if TR_UPD_PROFILE
__device__ long long g_upd_prof[64][8];
__device__ int g_upd_launch;
#define UPD_MARK(i) \
  if (threadIdx.x == 0) g_upd_prof[g_upd_launch & 63][i] = wall_clock64()
#else
#define UPD_MARK(i)
#endif

namespace {
constexpr int UPD_T = 1024;  // threads of the one workgroup (the norm order above assumes it)
constexpr int UPD_TRIP = 2;  // elements per thread per loop trip (loads in flight together; 4: no better)

__device__ __forceinline__ int factor_of(const FactorSet& fs, int64_t e) {
  int f = 0;
#pragma unroll
  for (int g = 1; g < TR_MAXF; ++g)
    if (g < fs.nf && e >= fs.off[g]) f = g;
  return f;
}
}

__device__ double np_pairwise_sum_absdiff(const double* h, int64_t n) {
  // sum_{j<n} |h[j+1] - h[j]| in numpy's pairwise order (PW_BLOCKSIZE 128, 8 accumulators),
  // iterative over the recursion tree (left-first), n <= 2^20.
  double total = 0.0;
  // explicit stack of (start, len, depth-combine) — emulate recursion with partial sums
  struct Frame { int64_t s, n; int state; double left; };
  Frame st[48];
  int sp = 0;
  st[sp++] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp > 0) {
    Frame& fr = st[sp - 1];
    if (fr.n <= 128 && fr.state == 0) {
      const int64_t s = fr.s, m = fr.n;
      double res;
      if (m < 8) {
        res = -0.0;
        for (int64_t i = 0; i < m; ++i) res += fabs(h[s + i + 1] - h[s + i]);
      } else {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = fabs(h[s + j + 1] - h[s + j]);
        int64_t i = 8;
        for (; i < m - (m % 8); i += 8)
          for (int j = 0; j < 8; ++j) r[j] += fabs(h[s + i + j + 1] - h[s + i + j]);
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < m; ++i) res += fabs(h[s + i + 1] - h[s + i]);
      }
      ret = res;
      --sp;
      continue;
    }
    int64_t n2 = fr.n / 2;
    n2 -= n2 % 8;
    if (fr.state == 0) {
      fr.state = 1;
      st[sp++] = {fr.s, n2, 0, 0.0};
    } else if (fr.state == 1) {
      fr.left = ret;
      fr.state = 2;
      const int64_t s = fr.s + n2, m = fr.n - n2;
      st[sp++] = {s, m, 0, 0.0};
    } else {
      ret = fr.left + ret;
      --sp;
    }
  }
  total = ret;
  return total;
}


__global__ __launch_bounds__(UPD_T) void k_update(FactorSet fs, int n_bias,
                                                  float* __restrict__ params, const float* __restrict__ grad,
                                                  UpdateArgs ua, float* __restrict__ m, float* __restrict__ v,
                                                  float* __restrict__ vmax, float* __restrict__ grad_total_out,
                                                  float* __restrict__ loss_out, double* __restrict__ loss_hist,
                                                  int32_t* __restrict__ stop, PrepArgs pa) {
#pragma clang fp contract(off)
  __shared__ float wsum[TR_MAXF * 16];
  __shared__ float norms[TR_MAXF];
  __shared__ float coef[TR_MAXF];
  UPD_MARK(0);
  const int t = threadIdx.x;
  const int lane = t & (TR_WAVE - 1);
  const int q = t / TR_WAVE;
  constexpr int NWV = UPD_T / TR_WAVE;
  constexpr int64_t B = UPD_T;
  const int64_t nfe = fs.nfelem;
  const int64_t np = nfe + n_bias;  // bias entries after the factors (linear 1, spectral n_out)
  // the flag and the status slot are loaded first and branched on after the norms
  const bool checked = ua.mode == 0 && stop != nullptr;
  const int32_t stop0 = stop != nullptr ? *stop : 0;
  const float status = checked ? grad[np + 1] : 0.f;
  // ||A_f||_F of every factor (raw parameters): per-thread sums in increasing k, the factor's
  // accumulator selected without a branch, then the wave butterfly and the wave-order LDS sum
  float accn[TR_MAXF];
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) accn[f] = 0.f;
  auto acc = [&](int64_t k, float a) {
    const int f = factor_of(fs, k);
#pragma unroll
    for (int g = 0; g < TR_MAXF; ++g) accn[g] = g == f ? fmaf(a, a, accn[g]) : accn[g];
  };
  int64_t k = t;
  for (; k + (UPD_TRIP - 1) * B < nfe; k += UPD_TRIP * B) {
    float a[UPD_TRIP];
#pragma unroll
    for (int u = 0; u < UPD_TRIP; ++u) a[u] = params[k + u * B];
#pragma unroll
    for (int u = 0; u < UPD_TRIP; ++u) acc(k + u * B, a[u]);
  }
  for (; k < nfe; k += B) acc(k, params[k]);
#pragma unroll
  for (int f = 0; f < TR_MAXF; ++f) {
    if (f < fs.nf) {
      const float r = tr_wave_allreduce(accn[f]);
      if (lane == 0) wsum[f * 16 + q] = r;
    }
  }
  UPD_MARK(1);
  __syncthreads();
  if (t < fs.nf) {
    float tot = 0.f;
    for (int w = 0; w < NWV; ++w) tot += wsum[t * 16 + w];
    norms[t] = sqrtf(tot);
    coef[t] = ua.lambda_l2 / (2.0f * norms[t]);  // d/dA lambda ||A|| = (lambda / (2 ||A||)) * (2 A)
  }
  __syncthreads();
  UPD_MARK(2);
  if (stop0 != 0) return;
  // a failed pass (status slot set, summed over shards by the all-reduce): stop the fit before
  // the step so the parameters and the Adam state stay those of the last good iteration
  if (checked && status != 0.0f) {
    if (t == 0) *stop = TR_STOP_DEVICE_ERROR - (int32_t)ua.iter;
    return;
  }
  unsigned nnmask = 0;  // factors under softplus (the next iteration's phi / dphi)
#pragma unroll
  for (int g = 0; g < TR_MAXF; ++g)
    if (g < fs.nf && fs.nonneg[g]) nnmask |= 1u << g;
  const bool adam = ua.mode != 1;
  const bool ams = adam && ua.amsgrad;
  auto step = [&](int64_t e, float g, float p, float mm, float vv, float vm) {
    const int f = factor_of(fs, e);
    g = e < nfe ? g + coef[f] * (2.0f * p) : g;
    if (!adam) {
      grad_total_out[e] = g;
      return;
    }
    g = ua.weight_decay != 0.0f ? fmaf(p, ua.weight_decay, g) : g;  // grad.add(param, alpha=wd)
    mm = fmaf(ua.one_minus_b1, g - mm, mm);                          // exp_avg.lerp_(grad, 1 - b1)
    vv = vv * ua.beta2;                                              // exp_avg_sq.mul_(b2)
    vv = vv + ua.one_minus_b2 * g * g;                               //   .addcmul_(g, g, 1 - b2)
    vm = fmaxf(vm, vv);
    if (ams) vmax[e] = vm;
    const float denom = sqrtf(ams ? vm : vv) / ua.bc2_sqrt + ua.eps;
    p = p + (-ua.step_size) * (mm / denom);                          // addcdiv_(m, denom, -step_size)
    m[e] = mm;
    v[e] = vv;
    params[e] = p;
    if (pa.mode > 0 && e < nfe) {  // the next iteration's phi / dphi (k_prep_factors' arithmetic)
      const bool soft = (nnmask >> f) & 1u;
      pa.phi[e] = soft ? tr_softplus(p, pa.beta, pa.thr) : p;
      pa.dphi[e] = soft ? tr_softplus_grad(p, pa.beta, pa.thr) : 1.0f;
    }
  };
  // UPD_TRIP elements per trip: their loads are in flight before any is consumed
  int64_t e = t;
  for (; e + (UPD_TRIP - 1) * B < np; e += UPD_TRIP * B) {
    float g[UPD_TRIP], p[UPD_TRIP], mo[UPD_TRIP], vo[UPD_TRIP], xo[UPD_TRIP];
#pragma unroll
    for (int u = 0; u < UPD_TRIP; ++u) {
      const int64_t eu = e + u * B;
      g[u] = grad[eu];
      p[u] = params[eu];
      mo[u] = adam ? m[eu] : 0.f;
      vo[u] = adam ? v[eu] : 0.f;
      xo[u] = ams ? vmax[eu] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UPD_TRIP; ++u) step(e + u * B, g[u], p[u], mo[u], vo[u], xo[u]);
  }
  for (; e < np; e += B) step(e, grad[e], params[e], adam ? m[e] : 0.f, adam ? v[e] : 0.f, ams ? vmax[e] : 0.f);
  UPD_MARK(3);
  if (t == 0) {
    float l2 = 0.f;
    for (int f = 0; f < fs.nf; ++f) l2 = l2 + norms[f];
    const float total = grad[np] + ua.lambda_l2 * l2;
    if (loss_out != nullptr) *loss_out = total;
    if (ua.mode == 0 && loss_hist != nullptr) loss_hist[ua.hist_base + ua.iter] = (double)total;
    // spectral…py:738-741: `elif np.isnan(loss_running[-1])` only while ii <= patience;
    // a negative flag = stopped without convergence, |flag| iterations run
    if (ua.mode == 0 && ua.nan_stop && stop != nullptr && ua.iter <= ua.patience && __builtin_isnan(total))
      *stop = -(int32_t)(ua.iter + 1);
  }
  UPD_MARK(4);
#if TR_UPD_PROFILE
  __syncthreads();
  UPD_MARK(5);
  if (t == 0) g_upd_launch = g_upd_launch + 1;
#endif
}

// Plateau test of fit_Adam (standard…py:467-470): one wave, launched only when it can fire.
__global__ __launch_bounds__(64) void k_converge(const double* __restrict__ loss_hist, int64_t hist_base,
                                                 int64_t iter, int64_t patience, double tol,
                                                 int32_t* __restrict__ stop) {
  if (*stop != 0 || threadIdx.x != 0) return;
  const int64_t s = iter - patience;             // loss_running[ii - patience:]
  const int64_t cnt = hist_base + iter - s;      // number of diffs in the slice
  const double d = np_pairwise_sum_absdiff(loss_hist + s, cnt);
  if (d < tol) *stop = (int32_t)(iter + 1);  // iterations completed (loss_running length)
}

hipError_t launch_converge(const double* loss_hist, int64_t hist_base, int64_t iter, int64_t patience, double tol,
                           int32_t* stop, hipStream_t st) {
  hipLaunchKernelGGL(k_converge, dim3(1), dim3(64), 0, st, loss_hist, hist_base, iter, patience, tol, stop);
  return hipGetLastError();
}

// ==========================================================================================
// MTTKRP of a two-factor model (config 2: rows 256 + 128, rank 8), one wave per factor row:
//   grad[A_f][i, r] = dphi * sum_j G[i_f = i, i_g = j] * (w_r * Phi_g[j, r])      (g = 1 - f)
// k_mttkrp's general form (any number of factors, tr_kernels.hip) stages every factor in LDS in
// every one of its 256-thread workgroups and walks a mixed-radix index; with one other factor
// the wave reads its rows of Phi_g straight from L2 (two 16-B loads per row at rank 8).  Same
// per-element product (w_r * Phi) and fma as k_mttkrp; the sum over j is a 64-lane butterfly.
// ==========================================================================================
template <int RMAX>
__global__ __launch_bounds__(64) void k_mttkrp2(FactorSet fs, const float* __restrict__ phi,
                                                const float* __restrict__ dphi, const float* __restrict__ w,
                                                const float* __restrict__ G, float* __restrict__ out,
                                                const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int R = fs.rank;
  const int lane = threadIdx.x;
  const bool f1 = (int64_t)blockIdx.x >= fs.dim[0];
  const int f = f1 ? 1 : 0, g = 1 - f;
  const int64_t i = f1 ? (int64_t)blockIdx.x - fs.dim[0] : (int64_t)blockIdx.x;
  const int64_t dg = fs.dim[g];
  const float* __restrict__ Fg = phi + fs.off[g];
  const float* __restrict__ Gi = G + i * fs.stride[f];
  const int64_t sg = fs.stride[g];
  float wr[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) wr[r] = r < R ? w[r] : 0.f;
  float acc[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) acc[r] = 0.f;
  // four rows per trip, all loads in flight first (config 2: one or two trips per lane)
  constexpr int J = 4;
  for (int64_t j0 = lane; j0 < dg; j0 += J * TR_WAVE) {
    float gv[J], fr[J][RMAX];
#pragma unroll
    for (int u = 0; u < J; ++u) {
      const int64_t j = j0 + u * TR_WAVE;
      const int64_t jc = j < dg ? j : dg - 1;
      gv[u] = Gi[jc * sg];
#pragma unroll
      for (int r = 0; r < RMAX; ++r) fr[u][r] = r < R ? Fg[jc * R + r] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < J; ++u)
      if (j0 + u * TR_WAVE < dg)
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
          if (r < R) acc[r] = fmaf(gv[u], wr[r] * fr[u][r], acc[r]);
  }
  float res = 0.f;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    if (r < R) {
      const float s = tr_wave_allreduce(acc[r]);
      if (lane == r) res = s;
    }
  }
  if (lane < R) {
    const int64_t e = fs.off[f] + i * R + lane;
    out[e] = res * dphi[e];
  }
}

bool mttkrp2_supported(const FactorSet& fs) { return fs.nf == 2 && fs.rank >= 1 && fs.rank <= 16; }

hipError_t launch_mttkrp2(const FactorSet& fs, const float* phi, const float* dphi, const float* w, const float* G,
                          float* grad, const int32_t* stop, hipStream_t st) {
  if (!mttkrp2_supported(fs)) return hipErrorInvalidValue;
  const unsigned rows = (unsigned)(fs.dim[0] + fs.dim[1]);
  if (fs.rank <= 8)
    hipLaunchKernelGGL(k_mttkrp2<8>, dim3(rows), dim3(TR_WAVE), 0, st, fs, phi, dphi, w, G, grad, stop);
  else
    hipLaunchKernelGGL(k_mttkrp2<16>, dim3(rows), dim3(TR_WAVE), 0, st, fs, phi, dphi, w, G, grad, stop);
  return hipGetLastError();
}


// ==========================================================================================
// MTTKRP of a three-factor model as two small GEMM stages (config 4: dims 64 x 64 x 32, rank 16;
// the autograd of cp_to_tensor, standard…py:123-130).  Modes by dense stride: s (slowest), m,
// q (stride 1), G = the dense gradient, a_f = w (.) Phi_f rows:
//   dA_s[i, r] = w_r sum_j a_m[j, r] H[i, j, r]        H[i, j, r] = sum_k G[i, j, k] Phi_q[k, r]
//   dA_m[j, r] = w_r sum_i Phi_s[i, r] H[i, j, r]
//   dA_q[k, r] = w_r sum_{i, j} G[i, j, k] Phi_s[i, r] Phi_m[j, r]
// k_mttkrp3_part: one workgroup per (i, block of JB rows j): its G block (JB x I_q floats,
// contiguous) is read once, coalesced, into LDS; H_block = G_block . Phi_q (a (JB x I_q) x
// (I_q x R) GEMM) and G_block^T . (Phi_m (.) Phi_s[i]) (an (I_q x JB) x (JB x R) GEMM) give its
// partials of all three gradients.  k_mttkrp3_sum adds the partials in a fixed order and applies
// the softplus chain.  (k_mttkrp, tr_kernels.hip, walks each factor row's slice of G: the
// stride-1 mode's rows read G at a 128-B stride, every line of G once per row: 24.5 us at c4.)
// ==========================================================================================
namespace {
constexpr int M3_T = 256;
constexpr int M3_TILE = 4096;  // floats of G per workgroup at most
constexpr int M3_FQR = 8192;   // I_q * R floats of Phi_q in LDS at most
}  // namespace

struct Mttkrp3Geom {
  int fs_, fm, fq;  // factor index of the slow / middle / fast mode
  int Is, Im, Iq, JB, NJ, R, slab;
};

static bool mttkrp3_geom(const FactorSet& fs, Mttkrp3Geom* g) {
  if (fs.nf != 3 || fs.rank < 1 || fs.rank > 16) return false;
  int ord[3] = {0, 1, 2};
  for (int a = 0; a < 3; ++a)
    for (int b = a + 1; b < 3; ++b)
      if (fs.stride[ord[b]] > fs.stride[ord[a]]) {
        const int t = ord[a];
        ord[a] = ord[b];
        ord[b] = t;
      }
  // a dense row-major layout under the permutation (stride-1 fast mode, no gaps)
  if (fs.stride[ord[2]] != 1 || fs.stride[ord[1]] != fs.dim[ord[2]] ||
      fs.stride[ord[0]] != fs.dim[ord[1]] * fs.dim[ord[2]])
    return false;
  g->fs_ = ord[0];
  g->fm = ord[1];
  g->fq = ord[2];
  g->Is = (int)fs.dim[ord[0]];
  g->Im = (int)fs.dim[ord[1]];
  g->Iq = (int)fs.dim[ord[2]];
  g->R = fs.rank;
  if (g->Iq > M3_TILE || (int64_t)g->Iq * g->R > M3_FQR) return false;
  g->JB = M3_TILE / g->Iq;
  if (g->JB > g->Im) g->JB = g->Im;
  if (g->JB > 32) g->JB = 32;  // c4: 2 blocks per row i, 128 workgroups
  g->NJ = (g->Im + g->JB - 1) / g->JB;
  g->slab = g->R * (1 + g->JB + g->Iq);
  return true;
}

__global__ __launch_bounds__(M3_T) void k_mttkrp3_part(FactorSet fs, Mttkrp3Geom g, const float* __restrict__ phi,
                                                       const float* __restrict__ G, float* __restrict__ part,
                                                       const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  __shared__ __attribute__((aligned(16))) float sG[M3_TILE];
  __shared__ float sQ[M3_FQR];    // Phi_q [k][r]
  __shared__ float sM[64 * 16];   // Phi_m rows of the block [j][r]
  __shared__ float sH[64 * 16];   // H[j][r]
  const int t = threadIdx.x, R = g.R, Iq = g.Iq;
  const int i = blockIdx.x / g.NJ, jb = blockIdx.x - i * g.NJ;
  const int j0 = jb * g.JB, nj = g.Im - j0 < g.JB ? g.Im - j0 : g.JB;
  const float* __restrict__ Ps = phi + fs.off[g.fs_];
  const float* __restrict__ Pm = phi + fs.off[g.fm];
  const float* __restrict__ Pq = phi + fs.off[g.fq];
  // every global read of the workgroup at once: the block's G rows (nj * Iq contiguous floats),
  // Phi_q, the block's Phi_m rows; this thread's Phi_s[i][r] (the rank r of its outputs below is
  // t % R for every e = t + 256 c when R divides 256, else re-read per output)
  const float* __restrict__ Gb = G + ((int64_t)i * g.Im + j0) * Iq;
  const int ng = nj * Iq;
  if ((((uintptr_t)Gb) & 15) == 0 && (ng & 3) == 0) {
    for (int e = 4 * t; e < ng; e += 4 * M3_T)
      *reinterpret_cast<float4*>(sG + e) = *reinterpret_cast<const float4*>(Gb + e);
  } else {
    for (int e = t; e < ng; e += M3_T) sG[e] = Gb[e];
  }
  for (int e = t; e < Iq * R; e += M3_T) sQ[e] = Pq[e];
  for (int e = t; e < nj * R; e += M3_T) sM[e] = Pm[(int64_t)j0 * R + e];
  __syncthreads();
  float* slab = part + (int64_t)blockIdx.x * g.slab;
  // slab: [ s-partial (R) | m-partials (JB x R) | q-partials (Iq x R) ]
  // H[j][r] = sum_k G[j][k] Phi_q[k][r] (nj x R); its m partial H Phi_s[i, r]
  for (int e = t; e < nj * R; e += M3_T) {
    const int j = e / R, r = e - j * R;
    const float* gr = sG + j * Iq;
    float h = 0.f;
    for (int k = 0; k < Iq; ++k) h = fmaf(gr[k], sQ[k * R + r], h);
    sH[e] = h;
    slab[R + e] = h * Ps[(int64_t)i * R + r];
  }
  // q partial[k][r] = sum_j G[j][k] Phi_m[j][r] Phi_s[i][r]
  for (int e = t; e < Iq * R; e += M3_T) {
    const int k = e / R, r = e - k * R;
    float a = 0.f;
    for (int j = 0; j < nj; ++j) a = fmaf(sG[j * Iq + k], sM[j * R + r], a);
    slab[R + g.JB * R + e] = a * Ps[(int64_t)i * R + r];
  }
  __syncthreads();
  if (t < R) {  // s partial: sum_j H[j][r] Phi_m[j][r]
    float a = 0.f;
    for (int j = 0; j < nj; ++j) a = fmaf(sH[j * R + t], sM[j * R + t], a);
    slab[t] = a;
  }
}

// sum of the values b = q, q + 4, q + 8, ... (< n) at a stride: four interleaved running sums,
// all loads of a trip in flight together
__device__ __forceinline__ float m3_sum_q(const float* __restrict__ p, int64_t stride, int n, int q) {
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int b = q;
  for (; b + 12 < n; b += 16) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[(int64_t)(b + 4 * u) * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += v[u];
  }
  for (int u = 0; b < n; b += 4, ++u) a[u & 3] += p[(int64_t)b * stride];
  return (a[0] + a[2]) + (a[1] + a[3]);
}

// 64 outputs per workgroup, each summed by four waves (wave q: partials q, q + 4, ...) and the four
// quarter sums added in a fixed order (a single running sum over config 4's 128 block partials
// doubled the fast factor's distance from fp64 against k_mttkrp's per-row butterfly; one thread
// per output left 16 dependent L2 round trips on the critical path)
__global__ __launch_bounds__(M3_T) void k_mttkrp3_sum(FactorSet fs, Mttkrp3Geom g, const float* __restrict__ dphi,
                                                      const float* __restrict__ w, const float* __restrict__ part,
                                                      float* __restrict__ out, const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  __shared__ float red[4][64];
  const int R = g.R;
  const int ol = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + ol;
  const int64_t ns = (int64_t)g.Is * R, nm = (int64_t)g.Im * R, nq = (int64_t)g.Iq * R;
  const bool ok = e < ns + nm + nq;
  float acc = 0.f;
  int f = 0;
  int64_t row = 0;
  int r = 0;
  if (!ok) {
  } else if (e < ns) {  // dA_s[i][r]: the NJ blocks of row i
    f = g.fs_;
    row = e / R;
    r = (int)(e - row * R);
    acc = m3_sum_q(part + row * g.NJ * g.slab + r, g.slab, g.NJ, q);
  } else if (e < ns + nm) {  // dA_m[j][r]: every i of j's block
    f = g.fm;
    const int64_t x = e - ns;
    row = x / R;
    r = (int)(x - row * R);
    const int jb = (int)(row / g.JB), jj = (int)(row - (int64_t)jb * g.JB);
    acc = m3_sum_q(part + (int64_t)jb * g.slab + R + jj * R + r, (int64_t)g.NJ * g.slab, g.Is, q);
  } else {  // dA_q[k][r]: every block
    f = g.fq;
    const int64_t x = e - ns - nm;
    row = x / R;
    r = (int)(x - row * R);
    acc = m3_sum_q(part + R + (int64_t)g.JB * R + x, g.slab, g.Is * g.NJ, q);
  }
  red[q][ol] = acc;
  __syncthreads();
  if (q == 0 && ok) {
    const float s = (red[0][ol] + red[1][ol]) + (red[2][ol] + red[3][ol]);
    const int64_t o = fs.off[f] + row * R + r;
    out[o] = s * w[r] * dphi[o];
  }
}

bool mttkrp3_supported(const FactorSet& fs, int64_t part_cap) {
  Mttkrp3Geom g;
  if (!mttkrp3_geom(fs, &g)) return false;
  return (int64_t)g.Is * g.NJ * g.slab <= part_cap;
}

hipError_t launch_mttkrp3(const FactorSet& fs, const float* phi, const float* dphi, const float* w, const float* G,
                          float* grad, float* part, int64_t part_cap, const int32_t* stop, hipStream_t st) {
  Mttkrp3Geom g;
  if (!mttkrp3_geom(fs, &g) || (int64_t)g.Is * g.NJ * g.slab > part_cap) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_mttkrp3_part, dim3((unsigned)(g.Is * g.NJ)), dim3(M3_T), 0, st, fs, g, phi, G, part, stop);
  const int64_t nout = (int64_t)(g.Is + g.Im + g.Iq) * g.R;
  hipLaunchKernelGGL(k_mttkrp3_sum, dim3((unsigned)((nout + 63) / 64)), dim3(M3_T), 0, st, fs, g, dphi, w, part,
                     grad, stop);
  return hipGetLastError();
}

bool update_prepare_mode_ok(const FactorSet& fs, int mode) {
  // mode 1: phi / dphi of the new factors, elementwise.  (Building dense B in the update too was
  // measured slower than the separate multi-workgroup k_build_dense: one CU took 17 us for
  // config 2's 32768 x 8 products.)
  (void)fs;
  return mode <= 1;
}

hipError_t launch_update(const FactorSet& fs, int n_bias, float* params, const float* grad,
                         const UpdateArgs& ua, float* m, float* v, float* vmax, float* grad_total_out,
                         float* loss_out, double* loss_hist, int32_t* stop, hipStream_t st, const PrepArgs* pa) {
  PrepArgs p0;
  std::memset(&p0, 0, sizeof(p0));
  const PrepArgs& pp = pa != nullptr && ua.mode == 0 ? *pa : p0;
  if (!update_prepare_mode_ok(fs, pp.mode)) return hipErrorInvalidValue;
  if (fs.nf < 1 || fs.nf > TR_MAXF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_update, dim3(1), dim3(UPD_T), 0, st, fs, n_bias, params, grad, ua, m, v, vmax,
                     grad_total_out, loss_out, loss_hist, stop, pp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ua.mode == 0 && loss_hist != nullptr && stop != nullptr && ua.iter > ua.patience && ua.tol > 0.0) {
    hipLaunchKernelGGL(k_converge, dim3(1), dim3(64), 0, st, loss_hist, ua.hist_base, ua.iter, ua.patience,
                       ua.tol, stop);
    e = hipGetLastError();
  }
  return e;
}

}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_update() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_update));
}
}  // namespace tr
