// tr_spectral_gen.hip — the spectral model for shapes beyond the fused kernel's envelope
// (X.shape[1] or X.shape[2] > 256, K = rank_normal + rank_spectral*(n_complex_dim+1) > 32,
// n_out > 256, or one sample + scratch beyond a CU's LDS).  Same math as tr_spectral.hip
// (spectral_tensor_regression.py: lin_model :118-165 + stepwise_spectral_model :339-390 for the
// fit, spectral_model :168-220 for predict, stepwise_latents_model :284-336), staged through HBM:
//
//   k_specg_fwd   T_n (D x Kp) = X_n^T Phi0 for every sample  (v_mfma_f32_16x16x4_f32, operands
//                 straight from global memory: X rows as 64-B segments, Phi0 L1/L2-resident)
//   k_specg_epi   per sample, T_n in LDS: column sums (Z, V; predict: U), y_hat, residual, loss,
//                 dZ / dV, dT_n written over T_n, and the small-factor gradients (A1, C1, A2, C2,
//                 bias) accumulated per workgroup in LDS -> one arena-layout slab per chunk
//   k_specg_bwd   dPhi0 (W x Kp) += X_n dT_n over a chunk of samples (MFMA; X rows read as
//                 float4 feeding four k steps) -> the A0 / C0 entries of the same slabs
//
// X crosses HBM twice per iteration (k_specg_fwd, k_specg_bwd) plus T / dT (D*Kp per sample):
// the fallback trades the fused kernel's single pass for an unbounded sample shape.  For Kp <= 64
// (round 6) the forward and backward run k_specg_fwd4 / k_specg_bwd4: 16-B buffer loads at fixed
// per-lane offsets, the k tile count compiled in (no conditional operand loads), batched loads
// issued a batch ahead (1.7x the round-1 kernels at (512, 129); TR_SPECG_SCALAR=1 keeps those).  Slabs are
// summed in index order by k_reduce_slabs (+ softplus chain): bitwise reproducible.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "tr_common.h"
#include "tr_spectral.h"

namespace tr {

typedef float sg_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ sg_f32x4 sg_mfma(float a, float b, sg_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// forward: T[n][d][k] = sum_w X[n][w][d] Phi0[w][k].  Workgroup (d group of 64, sample chunk):
// wave v owns d tile 4*blockIdx.x + v and every k tile.  MFMA C[i=d][j=k]: lane (j, q) of a k step
// supplies A = X[w0 + q][d0 + (lane & 15)] and B = Phi0[w0 + q][k0 + j].
// ------------------------------------------------------------------------------------------
template <int KTM>
__global__ __launch_bounds__(256) void k_specg_fwd(const float* __restrict__ X, int64_t N, int64_t xld, SpecGeom g,
                                                   const float* __restrict__ Phi0, float* __restrict__ T,
                                                   int64_t rows_per_blk, const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int W = g.W, D = g.D, K = g.K, KP = g.gKP, KT = KP / 16;
  const int dt = blockIdx.x * 4 + wv;
  const int i = lane & 15, q = lane >> 4;
  const int d = dt * 16 + i;
  const bool dok = d < D;
  const int64_t n0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t n1 = n0 + rows_per_blk < N ? n0 + rows_per_blk : N;
  if (dt * 16 >= D) return;
  for (int64_t n = n0; n < n1; ++n) {
    const float* xs = X + n * xld;
    sg_f32x4 acc[KTM];
#pragma unroll
    for (int t = 0; t < KTM; ++t) acc[t] = sg_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int w0 = 0; w0 < W; w0 += 16) {
      float a[4], b[4][KTM];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int w = w0 + 4 * s + q;
        const bool wok = w < W;
        a[s] = (wok && dok) ? xs[(int64_t)w * D + d] : 0.f;
#pragma unroll
        for (int t = 0; t < KTM; ++t) {
          const int k = t * 16 + i;
          b[s][t] = (t < KT && wok && k < K) ? Phi0[(int64_t)w * K + k] : 0.f;
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < KTM; ++t)
          if (t < KT) acc[t] = sg_mfma(a[s], b[s][t], acc[t]);
    }
    // C[i = d row][j = k col]: lane (j, q) reg r holds row 4q + r of the tile, column j
    float* tn = T + n * (int64_t)D * KP;
#pragma unroll
    for (int t = 0; t < KTM; ++t)
      if (t < KT)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int dd = dt * 16 + 4 * q + r;
          if (dd < D) tn[(int64_t)dd * KP + t * 16 + i] = acc[t][r];
        }
  }
}

// ------------------------------------------------------------------------------------------
// forward, vectorised (round 6; K <= 64): T^T = Phi0^T X_n on v_mfma_f32_16x16x4_f32 with the d
// columns as N.  Wave wv of d group blockIdx.x owns d in [256 dg + 64 wv, +64); per 4 w rows, lane
// (i, q) reads X[w0 + q][d0 + 4i .. 4i + 3] as ONE 16-B buffer load (any D: 4-B aligned dwordx4s
// read exactly, tools/buf_range_probe.hip; rows past W come back zero from the sample's buffer
// range, and a quad straddling D reads the next row's first values, masked here) and MFMA m of the
// four takes component m: A = Phi0[w0 + q][k0 + i], B = X[w0 + q][d0 + 4i + m], so C[k][i] of MFMA m
// is T[d0 + 4i + m][k] -- lane (i, q) holds four consecutive k of one d: one 16-B store.  (The
// scalar form above reads 4 B per lane and instruction: 26 % of HBM at (512, 129).)
// ------------------------------------------------------------------------------------------
template <int KTM>
__global__ __launch_bounds__(64) void k_specg_fwd4(const float* __restrict__ X, int64_t N, int64_t xld, SpecGeom g,
                                                    const float* __restrict__ Phi0, float* __restrict__ T,
                                                    int64_t rows_per_blk, const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  // (one wave per workgroup: d group blockIdx.x of 64 columns, sample block blockIdx.y)
  const int lane = threadIdx.x & 63;
  const int W = g.W, D = g.D, K = g.K, KP = g.gKP;  // (KP == 16 KTM: the launch's choice)
  const int i = lane & 15, q = lane >> 4;
  const int d0 = blockIdx.x * 64;
  const int db = d0 + 4 * i;  // this lane's quad of d
  bool mok[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) mok[m] = db + m < D;
  const int64_t n0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t n1 = n0 + rows_per_blk < N ? n0 + rows_per_blk : N;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Phi0, (short)0, (int)((int64_t)W * K * 4), 0x00020000);
  for (int64_t n = n0; n < n1; ++n) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)(X + n * xld), (short)0, (int)((int64_t)W * D * 4), 0x00020000);
    sg_f32x4 acc[KTM][4];
#pragma unroll
    for (int t = 0; t < KTM; ++t)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[t][m] = sg_f32x4{0.f, 0.f, 0.f, 0.f};
    // SG_U steps of 4 rows per batch, the next batch's loads issued before this batch's MFMAs: one
    // load in flight per wave left the loop waiting on memory latency (1.09 ms at (512, 129))
    constexpr int SG_U = 4;
    const int xvo = 4 * (q * D + db), pvo = 4 * (q * K + i);
    bool kok[KTM];  // column k = 16 t + i of Phi0 exists (past K: the next row's values, masked)
#pragma unroll
    for (int t = 0; t < KTM; ++t) kok[t] = 16 * t + i < K;
    sg_f32x4 xb[2][SG_U];
    float ab[2][SG_U][KTM];
    // (per-lane offsets fixed, the row in the scalar offset: no per-element address registers; rows
    // past W read zeros from both buffers' ranges, columns k >= K of Phi0 are masked)
    auto load_batch = [&](int w0, int buf) {
#pragma unroll
      for (int u = 0; u < SG_U; ++u) {
        const int wr = w0 + 4 * u;
        xb[buf][u] = __builtin_bit_cast(sg_f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, xvo, 4 * wr * D, 0));
#pragma unroll
        for (int t = 0; t < KTM; ++t)  // (loaded unconditionally, masked by a select: a conditional
          // load compiles to a branch with a vmcnt(0) wait inside it, which serialised the loop)
          ab[buf][u][t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, pvo, 4 * (wr * K + 16 * t), 0));
      }
    };
    auto compute = [&](int buf) {  // (called with a literal: the buffer index is compile-time)
#pragma unroll
      for (int u = 0; u < SG_U; ++u)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          if (d0 + m >= D) continue;  // (uniform: no lane's column d0 + 4 i + m exists; D = 129's tail)
          const float b = mok[m] ? xb[buf][u][m] : 0.f;
#pragma unroll
          for (int t = 0; t < KTM; ++t) acc[t][m] = sg_mfma(kok[t] ? ab[buf][u][t] : 0.f, b, acc[t][m]);
        }
    };
    const int nbat = (W + 4 * SG_U - 1) / (4 * SG_U);
    load_batch(0, 0);
    for (int bt = 0; bt < nbat; bt += 2) {
      if (bt + 1 < nbat) load_batch((bt + 1) * 4 * SG_U, 1);
      compute(0);
      if (bt + 1 < nbat) {
        if (bt + 2 < nbat) load_batch((bt + 2) * 4 * SG_U, 0);
        compute(1);
      }
    }
    float* tn = T + n * (int64_t)D * KP;
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (mok[m])
#pragma unroll
        for (int t = 0; t < KTM; ++t) *reinterpret_cast<sg_f32x4*>(tn + (int64_t)(db + m) * KP + t * 16 + 4 * q) = acc[t][m];
  }
}

// ------------------------------------------------------------------------------------------
// epilogue, one workgroup per sample chunk.  LDS: T_n [D][KP+1], the factor images, the
// small-factor gradient accumulators (owner-computes: no two threads add into one item).
// ------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void k_specg_epi(int64_t N, SpecGeom g, const float* __restrict__ phi,
                                                   const float* __restrict__ wts, const float* __restrict__ y,
                                                   float scale, float* __restrict__ T, float* __restrict__ slab,
                                                   int64_t slab_stride, double* __restrict__ dpart,
                                                   float* __restrict__ out, int64_t rows_per_blk,
                                                   const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (stop != nullptr && *stop != 0) return;
  constexpr int NT = 256;
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const int D = g.D, K = g.K, KP = g.gKP, Rn = g.Rn, Rs = g.Rs, Cc = g.Cc, NO = g.NO;
  const int R2 = Rn + Rs;
  const int TS = KP + 1;
  float* sT = lds;                        // [D][TS]
  float* sPA1 = sT + D * TS;              // [D][Rn]   phi(A1)
  float* sPC1 = sPA1 + D * Rn;            // [D][Rs]   phi(C1)
  float* sPA2 = sPC1 + D * Rs;            // [NO][Rn]  w_r phi(A2)  (predict / fit)
  float* sPC2 = sPA2 + NO * Rn;           // [NO][Rs]  phi(C2) (fit) or w_{Rn+r} phi(C2) (predict)
  float* sB = sPC2 + NO * Rs;             // [NO]
  float* sW = sB + NO;                    // [R2]
  float* sZV = sW + R2;                   // [KP]  Z | V   (predict: Z | U over all K columns)
  float* sDZ = sZV + KP;                  // [R2]
  float* sRv = sDZ + R2;                  // [NO]
  float* sAcc = sRv + NO;                 // [D*R2 | NO*R2 | NO]  dA1,dC1 (d-major [d][j]) | dA2,dC2 [o][j] | bias
  const int nacc = (D + NO) * R2 + NO;
  for (int e = t; e < D * Rn; e += NT) sPA1[e] = phi[g.offA1 + e];
  for (int e = t; e < D * Rs; e += NT) sPC1[e] = phi[g.offC1 + e];
  if (MODE != SPEC_LATENT) {
    for (int e = t; e < NO * Rn; e += NT) sPA2[e] = wts[e % Rn] * phi[g.offA2 + e];
    for (int e = t; e < NO * Rs; e += NT)
      sPC2[e] = MODE == SPEC_PRED ? wts[Rn + e % Rs] * phi[g.offC2 + e] : phi[g.offC2 + e];
    for (int e = t; e < NO; e += NT) sB[e] = phi[g.offB + e];
    for (int e = t; e < R2; e += NT) sW[e] = wts[e];
  }
  for (int e = t; e < nacc; e += NT) sAcc[e] = 0.f;
  double lsum = 0.0;
  const int64_t n0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t n1 = n0 + rows_per_blk < N ? n0 + rows_per_blk : N;
  const int nred = MODE == SPEC_TRAIN ? R2 : (MODE == SPEC_PRED ? K : Rn);
  for (int64_t n = n0; n < n1; ++n) {
    float* tn = T + n * (int64_t)D * KP;
    __syncthreads();
    for (int e = t; e < D * KP; e += NT) {
      const int dd = e / KP, k = e - dd * KP;
      sT[dd * TS + k] = tn[e];
    }
    __syncthreads();
    // column sums: one wave per value j, lanes over d, fixed-order wave reduction
    for (int j = wv; j < nred; j += 4) {
      float v = 0.f;
      if (MODE == SPEC_TRAIN && j >= Rn) {
        const int r = j - Rn, c0 = Rn + r * Cc;
        for (int dd = lane; dd < D; dd += 64) {
          float ss = 0.f;
          for (int c = 0; c < Cc; ++c) {
            const float x = sT[dd * TS + c0 + c];
            ss = fmaf(x, x, ss);
          }
          v = fmaf(sqrtf(ss), sPC1[dd * Rs + r], v);
        }
      } else {
        for (int dd = lane; dd < D; dd += 64) {
          const float ph = j < Rn ? sPA1[dd * Rn + j] : sPC1[dd * Rs + (j - Rn) / Cc];
          v = fmaf(sT[dd * TS + j], ph, v);
        }
      }
      v = tr_wave_allreduce(v);
      if (lane == 0) sZV[j] = v;
    }
    __syncthreads();
    if (MODE == SPEC_LATENT) {
      for (int r = t; r < Rn; r += NT) out[n * Rn + r] = sZV[r];
      continue;
    }
    if (MODE == SPEC_PRED) {
      for (int o = t; o < NO; o += NT) {
        float res = 0.f;
        const float b = sB[o];
        if (Rn > 0) {
          float yl = 0.f;
          for (int r = 0; r < Rn; ++r) yl = fmaf(sPA2[o * Rn + r], sZV[r], yl);
          res = yl + b;
        }
        if (Rs > 0) {
          float ss = 0.f;
          for (int c = 0; c < Cc; ++c) {
            float yc = 0.f;
            for (int r = 0; r < Rs; ++r) yc = fmaf(sPC2[o * Rs + r], sZV[Rn + r * Cc + c], yc);
            ss = fmaf(yc, yc, ss);
          }
          res = res + (sqrtf(ss) + b);
        }
        out[n * NO + o] = res;
      }
      continue;
    }
    // fit: y_hat, residual (bias added by both terms, quirk Q10), loss, small-factor gradients
    const float bm = (float)((Rn > 0) + (Rs > 0));
    for (int o = t; o < NO; o += NT) {
      const float b = sB[o];
      float yl = 0.f, ys = 0.f;
      for (int r = 0; r < Rn; ++r) yl = fmaf(sPA2[o * Rn + r], sZV[r], yl);
      for (int r = 0; r < Rs; ++r) ys = fmaf(sPC2[o * Rs + r], sZV[Rn + r], ys);
      const float yh = (Rn > 0 ? yl + b : 0.f) + (Rs > 0 ? ys + b : 0.f);
      const float e = yh - y[n * NO + o];
      const float rv = e * scale;
      sRv[o] = rv;
      sAcc[(D + NO) * R2 + o] += bm * rv;
      lsum += (double)e * (double)e;
      if (out != nullptr) out[n * NO + o] = yh;
    }
    __syncthreads();
    for (int e2 = t; e2 < NO * R2; e2 += NT) {
      const int o = e2 / R2, r = e2 - o * R2;
      const float rv = sRv[o];
      sAcc[D * R2 + e2] += r < Rn ? sW[r] * rv * sZV[r] : rv * sZV[r];
    }
    for (int j = t; j < R2; j += NT) {
      float dz = 0.f;
      if (j < Rn)
        for (int o = 0; o < NO; ++o) dz = fmaf(sRv[o], sPA2[o * Rn + j], dz);  // sPA2 = w_r phi(A2)
      else
        for (int o = 0; o < NO; ++o) dz = fmaf(sRv[o], sPC2[o * Rs + (j - Rn)], dz);
      sDZ[j] = dz;
    }
    __syncthreads();
    // dT_n and the A1 / C1 gradients, item (d, j); dT goes to global over T_n (pad columns 0)
    for (int e = t; e < D * R2; e += NT) {
      const int dd = e / R2, j = e - dd * R2;
      const float dz = sDZ[j];
      const float* tr = sT + dd * TS;
      float* to = tn + (int64_t)dd * KP;
      if (j < Rn) {
        sAcc[e] += dz * tr[j];
        to[j] = dz * sPA1[dd * Rn + j];
      } else {
        const int r = j - Rn, c0 = Rn + r * Cc;
        float ss = 0.f;
        for (int c = 0; c < Cc; ++c) ss = fmaf(tr[c0 + c], tr[c0 + c], ss);
        const float mg = sqrtf(ss);
        sAcc[e] += dz * mg;
        const float qq = mg > 0.f ? dz * sPC1[dd * Rs + r] / mg : 0.f;  // torch's norm backward (0 at 0)
        for (int c = 0; c < Cc; ++c) to[c0 + c] = qq * tr[c0 + c];
      }
    }
  }
  if (MODE != SPEC_TRAIN) return;
  __syncthreads();
  float* sl = slab + (int64_t)blockIdx.x * slab_stride;
  for (int e = t; e < D * R2; e += NT) {
    const int dd = e / R2, j = e - dd * R2;
    if (j < Rn)
      sl[g.offA1 + (int64_t)dd * Rn + j] = sAcc[e];
    else
      sl[g.offC1 + (int64_t)dd * Rs + (j - Rn)] = sAcc[e];
  }
  for (int e = t; e < NO * R2; e += NT) {
    const int o = e / R2, j = e - o * R2;
    if (j < Rn)
      sl[g.offA2 + (int64_t)o * Rn + j] = sAcc[D * R2 + e];
    else
      sl[g.offC2 + (int64_t)o * Rs + (j - Rn)] = sAcc[D * R2 + e];
  }
  for (int o = t; o < NO; o += NT) sl[g.offB + o] = sAcc[(D + NO) * R2 + o];
  // loss partial: fixed-order block reduction
  __shared__ double dred[4];
  const double ls = tr_wave_allreduce_d(lsum);
  if (lane == 0) dred[wv] = ls;
  __syncthreads();
  if (t == 0) {
    dpart[2 * blockIdx.x] = ((dred[0] + dred[1]) + dred[2]) + dred[3];
    dpart[2 * blockIdx.x + 1] = 0.0;
  }
}

// ------------------------------------------------------------------------------------------
// backward: dPhi0[w][k] = sum_n sum_d X[n][w][d] dT[n][d][k] over the chunk of samples of this
// workgroup (grid.y), w tile 4*blockIdx.x + wave.  MFMA C[i=w][j=k]; per 16 d: lane (i, q) loads
// X[w0 + i][d0 + 4q .. +3] (one float4 when VEC) and MFMA m of the four uses component m with
// B = dT[d0 + 4q + m][k0 + j] — a consistent permutation of the k (= d) order.
// ------------------------------------------------------------------------------------------
template <int KTM, int VEC>
__global__ __launch_bounds__(256) void k_specg_bwd(const float* __restrict__ X, int64_t N, int64_t xld, SpecGeom g,
                                                   const float* __restrict__ T, float* __restrict__ slab,
                                                   int64_t slab_stride, int64_t rows_per_blk,
                                                   const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int W = g.W, D = g.D, K = g.K, KP = g.gKP, KT = KP / 16, Rn = g.Rn, Rs = g.Rs, Cc = g.Cc;
  const int wt = blockIdx.x * 4 + wv;
  const int i = lane & 15, q = lane >> 4;
  const int w = wt * 16 + i;
  const bool wok = w < W;
  const int64_t n0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t n1 = n0 + rows_per_blk < N ? n0 + rows_per_blk : N;
  sg_f32x4 acc[KTM];
#pragma unroll
  for (int tt = 0; tt < KTM; ++tt) acc[tt] = sg_f32x4{0.f, 0.f, 0.f, 0.f};
  if (wt * 16 < W) {
    for (int64_t n = n0; n < n1; ++n) {
      const float* xr = X + n * xld + (int64_t)(wok ? w : 0) * D;
      const float* tn = T + n * (int64_t)D * KP;
      for (int d0 = 0; d0 < D; d0 += 16) {
        const int db = d0 + 4 * q;
        float a[4];
        if (VEC && db + 3 < D) {
          const float4 v = *reinterpret_cast<const float4*>(xr + db);
          a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m) a[m] = db + m < D ? xr[db + m] : 0.f;
        }
        if (!wok) a[0] = a[1] = a[2] = a[3] = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int dd = db + m;
#pragma unroll
          for (int tt = 0; tt < KTM; ++tt)
            if (tt < KT) {
              const float b = dd < D ? tn[(int64_t)dd * KP + tt * 16 + i] : 0.f;
              acc[tt] = sg_mfma(a[m], b, acc[tt]);
            }
        }
      }
    }
  }
  if (wt * 16 >= W) return;
  // lane (j, q) reg r holds dPhi0[w = wt*16 + 4q + r][k = tt*16 + j] -> arena (phi space) A0 / C0
  float* sl = slab + (int64_t)blockIdx.y * slab_stride;
#pragma unroll
  for (int tt = 0; tt < KTM; ++tt)
    if (tt < KT)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ww = wt * 16 + 4 * q + r, k = tt * 16 + i;
        if (ww < W && k < K) {
          const int64_t dst = k < Rn ? g.offA0 + (int64_t)ww * Rn + k : g.offC0 + (int64_t)ww * Rs * Cc + (k - Rn);
          sl[dst] = acc[tt][r];
        }
      }
}

// backward, batched (round 6): k_specg_bwd's MFMA layout, every operand by buffer load at a fixed
// per-lane offset with the d step in the scalar offset (X: one 16-B load per lane and step, any D;
// dT: the sample's D x KP image, rows past D read zero), SG_UB steps per batch and the next batch's
// loads issued before this batch's MFMAs.
template <int KTM>
__global__ __launch_bounds__(256) void k_specg_bwd4(const float* __restrict__ X, int64_t N, int64_t xld, SpecGeom g,
                                                    const float* __restrict__ T, float* __restrict__ slab,
                                                    int64_t slab_stride, int64_t rows_per_blk,
                                                    const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  // two 16-row w tiles per wave (each dT operand feeds both): wave wv of w group blockIdx.x owns
  // rows [128 blockIdx.x + 32 wv, +32)
  constexpr int SG_UB = 4, NWT = 2;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int W = g.W, D = g.D, K = g.K, KP = g.gKP, Rn = g.Rn, Rs = g.Rs, Cc = g.Cc;  // (KP == 16 KTM)
  const int w00 = blockIdx.x * 128 + wv * 32;
  const int i = lane & 15, q = lane >> 4;
  const int64_t n0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t n1 = n0 + rows_per_blk < N ? n0 + rows_per_blk : N;
  sg_f32x4 acc[NWT][KTM];
#pragma unroll
  for (int h = 0; h < NWT; ++h)
#pragma unroll
    for (int tt = 0; tt < KTM; ++tt) acc[h][tt] = sg_f32x4{0.f, 0.f, 0.f, 0.f};
  int xvo[NWT];  // rows past W: out of range, zero
#pragma unroll
  for (int h = 0; h < NWT; ++h) {
    const int w = w00 + 16 * h + i;
    xvo[h] = w < W ? 4 * (w * D + 4 * q) : 0x40000000;
  }
  const int tvo = 4 * (4 * q * KP + i);
  const int nds = (D + 15) / 16;
  if (w00 < W) {
    for (int64_t n = n0; n < n1; ++n) {
      const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(uintptr_t)(X + n * xld), (short)0, (int)((int64_t)W * D * 4), 0x00020000);
      const __amdgpu_buffer_rsrc_t ts = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(uintptr_t)(T + n * (int64_t)D * KP), (short)0, (int)((int64_t)D * KP * 4), 0x00020000);
      sg_f32x4 xb[2][SG_UB][NWT];
      float bb[2][SG_UB][4][KTM];
      auto load_batch = [&](int s0, int buf) {
#pragma unroll
        for (int u = 0; u < SG_UB; ++u) {
          const int d0 = 16 * (s0 + u);
#pragma unroll
          for (int h = 0; h < NWT; ++h)
            xb[buf][u][h] = __builtin_bit_cast(sg_f32x4, __builtin_amdgcn_raw_buffer_load_b128(xs, xvo[h], 4 * d0, 0));
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int tt = 0; tt < KTM; ++tt)
              bb[buf][u][m][tt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ts, tvo, 4 * ((d0 + m) * KP + 16 * tt), 0));
        }
      };
      auto compute = [&](int s0, int buf) {
#pragma unroll
        for (int u = 0; u < SG_UB; ++u) {
          const int db = 16 * (s0 + u) + 4 * q;
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int h = 0; h < NWT; ++h) {
              const float a = db + m < D ? xb[buf][u][h][m] : 0.f;  // (a quad straddling D: the next row's values)
#pragma unroll
              for (int tt = 0; tt < KTM; ++tt) acc[h][tt] = sg_mfma(a, bb[buf][u][m][tt], acc[h][tt]);
            }
        }
      };
      load_batch(0, 0);
      for (int s0 = 0; s0 < nds; s0 += 2 * SG_UB) {
        if (s0 + SG_UB < nds) load_batch(s0 + SG_UB, 1);
        compute(s0, 0);
        if (s0 + SG_UB < nds) {
          if (s0 + 2 * SG_UB < nds) load_batch(s0 + 2 * SG_UB, 0);
          compute(s0 + SG_UB, 1);
        }
      }
    }
  }
  if (w00 >= W) return;
  float* sl = slab + (int64_t)blockIdx.y * slab_stride;
#pragma unroll
  for (int h = 0; h < NWT; ++h)
#pragma unroll
    for (int tt = 0; tt < KTM; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ww = w00 + 16 * h + 4 * q + r, k = tt * 16 + i;
        if (ww < W && k < K) {
          const int64_t dst = k < Rn ? g.offA0 + (int64_t)ww * Rn + k : g.offC0 + (int64_t)ww * Rs * Cc + (k - Rn);
          sl[dst] = acc[h][tt][r];
        }
      }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
size_t specg_epi_lds_bytes(const SpecGeom& g) {
  const int64_t R2 = g.Rn + g.Rs, D = g.D, NO = g.NO, KP = g.gKP;
  const int64_t f = D * (KP + 1) + D * R2 + NO * R2 + NO + R2 + KP + R2 + NO + (D + NO) * R2 + NO;
  return (size_t)f * 4;
}

#define SG_KT_CASES(CALL)   \
  switch ((g.gKP / 16 + 1) / 2 * 2) { \
    case 2: CALL(2); break;            \
    case 4: CALL(4); break;            \
    case 6: CALL(6); break;            \
    case 8: CALL(8); break;            \
    default: CALL(16); break;          \
  }

hipError_t specg_prepare(const SpecGeom& g) {
  const size_t lds = specg_epi_lds_bytes(g);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_specg_epi<SPEC_TRAIN>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_specg_epi<SPEC_PRED>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_specg_epi<SPEC_LATENT>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

hipError_t launch_specg(int mode, const SpecGeom& g, int nchunks, const float* X, int64_t N, int64_t xld,
                        const float* phi, const float* Phi0, const float* wts, const float* y, float scale,
                        float* T, float* slab, int64_t slab_stride, double* dpart, float* out,
                        const int32_t* stop, hipStream_t st) {
  if (N < 1 || nchunks < 1) return hipSuccess;
  const int64_t rpb = (N + nchunks - 1) / nchunks;
  const unsigned nblk = (unsigned)((N + rpb - 1) / rpb);
  static const bool scalar_fwd = [] {  // TR_SPECG_SCALAR=1: the round-1 scalar forward (A/B)
    const char* v = std::getenv("TR_SPECG_SCALAR");
    return v != nullptr && v[0] == '1';
  }();
  if (g.gKP <= 64 && !scalar_fwd) {
    // (its own sample blocks: it writes no slabs; about 8 waves per CU per d group; the k tile count
    // compiled in)
    const int64_t rpf = (N + 4095) / 4096;
    const dim3 grid((unsigned)((g.D + 63) / 64), (unsigned)((N + rpf - 1) / rpf));
#define SG_F4(KM) hipLaunchKernelGGL((k_specg_fwd4<KM>), grid, dim3(64), 0, st, X, N, xld, g, Phi0, T, rpf, stop)
    switch (g.gKP / 16) {
      case 1: SG_F4(1); break;
      case 2: SG_F4(2); break;
      case 3: SG_F4(3); break;
      default: SG_F4(4); break;
    }
#undef SG_F4
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  } else {
    const dim3 grid((unsigned)((g.D + 63) / 64), nblk);
#define SG_FWD(KM) hipLaunchKernelGGL((k_specg_fwd<KM>), grid, dim3(256), 0, st, X, N, xld, g, Phi0, T, rpb, stop)
    SG_KT_CASES(SG_FWD)
#undef SG_FWD
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const size_t lds = specg_epi_lds_bytes(g);
  if (mode == SPEC_TRAIN)
    hipLaunchKernelGGL(k_specg_epi<SPEC_TRAIN>, dim3(nblk), dim3(256), lds, st, N, g, phi, wts, y, scale, T, slab,
                       slab_stride, dpart, out, rpb, stop);
  else if (mode == SPEC_PRED)
    hipLaunchKernelGGL(k_specg_epi<SPEC_PRED>, dim3(nblk), dim3(256), lds, st, N, g, phi, wts, y, scale, T, slab,
                       slab_stride, dpart, out, rpb, stop);
  else
    hipLaunchKernelGGL(k_specg_epi<SPEC_LATENT>, dim3(nblk), dim3(256), lds, st, N, g, phi, wts, y, scale, T, slab,
                       slab_stride, dpart, out, rpb, stop);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || mode != SPEC_TRAIN) return e;
  const bool vec = (g.D % 4 == 0) && (xld % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15u) == 0);
  const dim3 grid((unsigned)((g.W + 63) / 64), nblk);
#define SG_BWD(KM)                                                                                              \
  if (vec)                                                                                                      \
    hipLaunchKernelGGL((k_specg_bwd<KM, 1>), grid, dim3(256), 0, st, X, N, xld, g, T, slab, slab_stride, rpb, stop); \
  else                                                                                                          \
    hipLaunchKernelGGL((k_specg_bwd<KM, 0>), grid, dim3(256), 0, st, X, N, xld, g, T, slab, slab_stride, rpb, stop)
  if (g.gKP <= 64 && !scalar_fwd) {
    const dim3 grid4((unsigned)((g.W + 127) / 128), nblk);
#define SG_B4(KM) \
  hipLaunchKernelGGL((k_specg_bwd4<KM>), grid4, dim3(256), 0, st, X, N, xld, g, T, slab, slab_stride, rpb, stop)
    switch (g.gKP / 16) {
      case 1: SG_B4(1); break;
      case 2: SG_B4(2); break;
      case 3: SG_B4(3); break;
      default: SG_B4(4); break;
    }
#undef SG_B4
    return hipGetLastError();
  }
  SG_KT_CASES(SG_BWD)
#undef SG_BWD
  return hipGetLastError();
}

}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_spectral_gen() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_specg_epi<SPEC_TRAIN>));
}
}  // namespace tr
