// tr_spectral.hip — gfx950 kernels of the spectral CP regression model
// (spectral_tensor_regression.py).
//
// Fit model (stepwise_spectral_model :339-390 + lin_model :118-165, summed at :716-717):
//   T_n[d, k]  = sum_w X[n, w, d] Phi0[w, k]                      (one MFMA GEMM per sample)
//   Z_n[r]     = sum_d T_n[d, r] phi(A1)[d, r]                    r < Rn
//   M_n[d, r]  = || T_n[d, Rn + r*Cc : Rn + (r+1)*Cc] ||_2         r < Rs
//   V_n[r]     = sum_d M_n[d, r] phi(C1)[d, r]
//   yhat[n, o] = (sum_r w_r phi(A2)[o, r] Z_n[r] + b[o]) + (sum_r phi(C2)[o, r] V_n[r] + b[o])
// loss = MSELoss(yhat, y) (mean over N*NO); the backward pass needs only T_n:
//   dT_n[d, r]           = dZ_n[r] phi(A1)[d, r]
//   dT_n[d, Rn+r*Cc+c]   = dV_n[r] phi(C1)[d, r] T_n[d, Rn+r*Cc+c] / M_n[d, r]   (0 where M = 0,
//                          torch's norm backward)
//   dPhi0[w, k]         += sum_d X[n, w, d] dT_n[d, k]              (second MFMA GEMM per sample)
// so each workgroup streams its samples from HBM exactly ONCE per iteration: X_n is copied
// into LDS, both GEMMs and the epilogue run out of LDS, and the next sample is already in
// flight in registers.  The reference makes ≈6 passes over X (permute copy, bmm, norm, ...).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "tr_common.h"
#include "tr_spectral.h"

#ifndef TR_SPEC_SKIP
#define TR_SPEC_SKIP 0  // profiling ablation only: 1 fwd GEMM, 2 epilogue, 4 grad GEMM, 8 X staging
#endif

#ifndef TR_SPEC_PROFILE
#define TR_SPEC_PROFILE 0  // profiling build only: per-phase cycle counts of workgroup 0..255
#endif
#if TR_SPEC_PROFILE
__device__ unsigned long long g_spec_prof[256][8];
#define TR_PROF_MARK(ph)                                               \
  do {                                                                 \
    const unsigned long long _now = __builtin_readcyclecounter();      \
    prof[ph] += _now - prof_t;                                         \
    prof_t = _now;                                                     \
  } while (0)
#else
#define TR_PROF_MARK(ph) \
  do {                   \
  } while (0)
#endif

namespace tr {

typedef float tr_f32x4_s __attribute__((ext_vector_type(4)));

constexpr int kSpecNW = 8;  // waves per workgroup (two per SIMD, 256 registers each: the MFMA B
                            // fragments of one column tile + 1/512 of the next sample in flight)
constexpr int kSpecT = kSpecNW * TR_WAVE;

__device__ __forceinline__ tr_f32x4_s mfma4(float a, float b, tr_f32x4_s c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// prep: phi / dphi over the whole arena + Phi0 (W x K)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int spec_factor_of(const SpecGeom& g, int64_t e) {
  if (e >= g.offB) return 6;
  if (e >= g.offC2) return 5;
  if (e >= g.offC1) return 4;
  if (e >= g.offC0) return 3;
  if (e >= g.offA2) return 2;
  if (e >= g.offA1) return 1;
  return 0;
}

__global__ __launch_bounds__(256) void k_spec_prep(SpecGeom g, const float* __restrict__ params, float beta,
                                                   float thr, float* __restrict__ phi, float* __restrict__ dphi,
                                                   float* __restrict__ Phi0, const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  const int64_t n1 = g.nparams, n2 = (int64_t)g.W * g.K;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n1 + n2; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < n1) {
      const int f = spec_factor_of(g, e);
      const float a = params[e];
      float v = a, d = 1.f;
      if (f < 6 && g.nonneg[f % 3]) {
        v = tr_softplus(a, beta, thr);
        d = tr_softplus_grad(a, beta, thr);
      }
      phi[e] = v;
      dphi[e] = d;
    } else {
      const int64_t q = e - n1;
      const int w = (int)(q / g.K), k = (int)(q - (int64_t)w * g.K);
      const int64_t src = k < g.Rn ? g.offA0 + (int64_t)w * g.Rn + k : g.offC0 + (int64_t)w * g.Rs * g.Cc + (k - g.Rn);
      const float a = params[src];
      Phi0[q] = g.nonneg[0] ? tr_softplus(a, beta, thr) : a;  // A0 and C0 share non_negative[0]
    }
  }
}

__global__ __launch_bounds__(256) void k_spec_chain(int64_t n, const float* __restrict__ G,
                                                    const float* __restrict__ dphi, float* __restrict__ grad,
                                                    const int32_t* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    grad[e] = G[e] * dphi[e];
}

// ------------------------------------------------------------------------------------------
// LDS barrier that leaves LDS-DMA (global_load_lds) in flight: each wave retires its own LDS
// accesses, then s_barrier.  (__syncthreads() would also wait vmcnt(0) while a glds is
// outstanding, cdna_hip_programming.md §5 "Pipelining across barriers".)
__device__ __forceinline__ void spec_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// LDS-DMA pieces (16 B or 4 B per lane to LDS byte address m0 + size * lane) issued from inline
// asm, so the compiler does not see an LDS write in flight: with the builtin it cannot tell the
// row block being filled from the one being read and puts an `s_waitcnt vmcnt(0)` in front of the
// GEMMs' LDS reads, draining the DMA this kernel overlaps with them.  The kernel orders the
// pieces itself (counted spec_wait_vm + spec_barrier).  m0 is compiler-reserved: saved and
// restored inside the statement.
__device__ __forceinline__ uint32_t spec_lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}
__device__ __forceinline__ void spec_dma16(const float* gsrc, const float* lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(spec_lds_addr(lds_dst)))  // wave-uniform
               : "memory");
}
__device__ __forceinline__ void spec_dma4(const float* gsrc, const float* lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(spec_lds_addr(lds_dst)))  // wave-uniform
               : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the counter is an immediate)
__device__ __forceinline__ void spec_wait_vm(int n) {
#define TR_VM_CASE(k) \
  case k:             \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
  switch (n < 0 ? 0 : n) {
    TR_VM_CASE(0) TR_VM_CASE(1) TR_VM_CASE(2) TR_VM_CASE(3) TR_VM_CASE(4) TR_VM_CASE(5) TR_VM_CASE(6)
    TR_VM_CASE(7) TR_VM_CASE(8) TR_VM_CASE(9) TR_VM_CASE(10) TR_VM_CASE(11) TR_VM_CASE(12) TR_VM_CASE(13)
    TR_VM_CASE(14) TR_VM_CASE(15) TR_VM_CASE(16) TR_VM_CASE(17) TR_VM_CASE(18) TR_VM_CASE(19) TR_VM_CASE(20)
    TR_VM_CASE(21) TR_VM_CASE(22) TR_VM_CASE(23) TR_VM_CASE(24) TR_VM_CASE(25) TR_VM_CASE(26) TR_VM_CASE(27)
    TR_VM_CASE(28) TR_VM_CASE(29) TR_VM_CASE(30) TR_VM_CASE(31)
    default:
      asm volatile("s_waitcnt vmcnt(31)" ::: "memory");  // stricter than asked: still safe
  }
#undef TR_VM_CASE
}

// ------------------------------------------------------------------------------------------
// The fused kernel.  WSMAX: compile-time bound on the forward k steps (the B fragments of
// one Phi0 column tile live in registers, bf[s]); KT: 16-column tiles of K.
//
// X_n is staged in LDS in row blocks of RB = 16 * 8/KT rows (64 rows at KT = 2).  Per sample:
//   fwd   T_n = X_n^T Phi0: wave (grp, ktw) owns d tiles grp + NGRP*u and column tile ktw; k step s
//         reads rows 64*(s/16) + 16*j + s%16, so the steps of phase p touch only row block p and
//         wait only for that block's LDS-DMA; the partial d tile's 8-step chunks are dealt to
//         the wave groups (partials summed in the epilogue)
//   epi   column sums over d (Z, V or U; the partial tile's rows are materialised here),
//         y_hat / residual / small-factor gradients, dT_n and the A1/C1 gradients (in place)
//   grad  dPhi0 += X_n dT_n by row blocks (wave = (w tile, column tile)); after block p every
//         wave has finished reading those rows and block p of sample n+1 is issued by DMA into
//         them, so it streams in during the rest of this gradient GEMM and the next forward
// ------------------------------------------------------------------------------------------
template <int MODE, int WSMAX, int KT>
__global__ __launch_bounds__(kSpecT) void k_spec_fused(
    const float* __restrict__ X, int64_t N, int64_t xld, SpecGeom g, const float* __restrict__ phi,
    const float* __restrict__ Phi0, const float* __restrict__ wts, const float* __restrict__ y, float scale,
    float* __restrict__ slab, int64_t slab_stride, double* __restrict__ dpart, float* __restrict__ out,
    int64_t rows_per_wg, int reverse, const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NW = kSpecNW;
  constexpr int KP = 16 * KT;       // padded K
  constexpr int NGRP = NW / KT;     // wave groups over d tiles (= w tiles per row block)
  constexpr int TPW = KT;           // d tiles per wave per set (NGRP * TPW = 8 tiles per set)
  constexpr int RB = 128;           // rows per LDS-DMA / gradient block
  constexpr int PHS = RB / 4;       // forward k steps per block
  constexpr int NBMAX = 256 / RB;   // row blocks at W = 256
  constexpr int NPH = WSMAX / PHS;  // forward phases the step bound allows
  constexpr int CHK = 8;            // k steps per double-buffered chunk
  static_assert(PHS % CHK == 0, "phase must hold whole chunks");
  if (stop != nullptr && *stop != 0) return;
  const int t = threadIdx.x;
  const int lane = t & (TR_WAVE - 1);
  const int wv = t / TR_WAVE;
  const int KS = g.KS, D = g.D, K = g.K, Rn = g.Rn, Rs = g.Rs, Cc = g.Cc, NO = g.NO;
  const int ktw = wv % KT;
  const int grp = wv / KT;
  const int NB = (g.W + RB - 1) / RB;

  float* sX = lds;
  float* sT = lds + g.oT;
  float* sTail = lds + g.oTail;    // [NGRP][Dtail][KP] partial-tile partials
  float* sZV = lds + g.oSm;        // [64]  Z (Rn) | V (Rs)     or  Z | U (K) in predict mode
  float* sDZ = sZV + 32;           // [32]  dZ (Rn) | dV (Rs)   (the fit mode reduces <= 32 values)
  float* sRv = sZV + 64;           // [NO]  residual * MSE scale (NO <= 256 fits with sY after it)
  float* sY = sRv + 256;           // [NO]  y of the current sample
  float* sAcc = lds + g.oAcc;      // [NO*Rn] dA2 | [NO*Rs] dC2 | [NO] dbias
  float* sPA1 = lds + g.oPhi;      // [Rn][D]  phi(A1), transposed: consecutive d -> consecutive banks
  float* sPC1 = sPA1 + D * Rn;     // [Rs][D]  phi(C1), transposed
  float* sPA2 = sPC1 + D * Rs;     // [NO][Rn] w_r phi(A2)
  float* sPC2 = sPA2 + NO * Rn;    // [NO][Rs] phi(C2) (fit) or w_{Rn+r} phi(C2) (predict)
  float* sB = sPC2 + NO * Rs;      // [NO]     bias
  float* sWt = sB + NO;            // [Rn+Rs]  weights

  // zero the whole carve once: pad rows and the dT row D must read as 0
  for (int e = t; e < g.lds_floats; e += kSpecT) lds[e] = 0.f;
  __syncthreads();
  for (int e = t; e < D * Rn; e += kSpecT) sPA1[(e % Rn) * D + e / Rn] = phi[g.offA1 + e];
  for (int e = t; e < D * Rs; e += kSpecT) sPC1[(e % Rs) * D + e / Rs] = phi[g.offC1 + e];
  if (MODE != SPEC_LATENT) {  // (the latent mode takes no weights)
    for (int e = t; e < NO * Rn; e += kSpecT) sPA2[e] = wts[e % Rn] * phi[g.offA2 + e];
    for (int e = t; e < NO * Rs; e += kSpecT)
      sPC2[e] = MODE == SPEC_PRED ? wts[Rn + e % Rs] * phi[g.offC2 + e] : phi[g.offC2 + e];
    for (int e = t; e < NO; e += kSpecT) sB[e] = phi[g.offB + e];
    for (int e = t; e < Rn + Rs; e += kSpecT) sWt[e] = wts[e];
  }

  // B fragments of this wave's column tile: lane (i, gq) of step s holds Phi0[row(s, gq), ktw*16 + i],
  // row(s, j) = 64*(s/16) + 16*j + s%16 (rows >= W give 0)
  float bf[WSMAX];
  {
    const int i = lane & 15, gq = lane >> 4;
#pragma unroll
    for (int s = 0; s < WSMAX; ++s) {
      const int w = 64 * (s >> 4) + 16 * gq + (s & 15);
      const int col = ktw * 16 + i;
      bf[s] = (w < g.W && col < K) ? Phi0[(int64_t)w * K + col] : 0.f;
    }
  }
  // gradient tiles: w tiles 8p + grp + NGRP*u (u < KT) of block p, column tile ktw; two
  // accumulators each (even / odd k steps)
  tr_f32x4_s gacc[NBMAX][KT][2];
#pragma unroll
  for (int p = 0; p < NBMAX; ++p)
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      gacc[p][u][0] = tr_f32x4_s{0.f, 0.f, 0.f, 0.f};
      gacc[p][u][1] = tr_f32x4_s{0.f, 0.f, 0.f, 0.f};
    }
  float* sl = slab != nullptr ? slab + (int64_t)blockIdx.x * slab_stride : nullptr;
  // gradients of A1 / C1 in phi space, item e = j*D + d (j < Rn: A1[d, j]; else C1[d, j - Rn]),
  // thread t owns items t + 512*m (D*(Rn+Rs) <= 256*32 = 512*16)
  constexpr int AMAX = 16;
  const int nitems = D * (Rn + Rs);
  const float invD = 1.0f / (float)D;
  auto item = [&](int e, int& j, int& d) {
    j = (int)((float)e * invD);
    d = e - j * D;
    if (d < 0) { --j; d += D; }
    if (d >= D) { ++j; d -= D; }
  };
  float acc[AMAX];
#pragma unroll
  for (int m = 0; m < AMAX; ++m) acc[m] = 0.f;
  double lsum = 0.0;

  const int64_t n0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t n1 = n0 + rows_per_wg < N ? n0 + rows_per_wg : N;
  const int64_t nr = n1 > n0 ? n1 - n0 : 0;
  auto sample_of = [&](int64_t k) -> int64_t { return reverse ? (n1 - 1 - k) : (n0 + k); };

  // LDS-DMA of rows [RB*p, RB*(p+1)) of sample n into the same rows of sX (lane-linear image:
  // S == D).  16-B pieces when W*D % 4 == 0, else 4-B pieces.  Returns the instructions this
  // wave issued (wave-uniform), for the counted vmcnt waits.
  auto issue = [&](int64_t n, int p) -> int {
    const int64_t r0 = (int64_t)p * RB * D;
    int64_t r1 = (int64_t)(p + 1) * RB * D;
    if (r1 > g.WD) r1 = g.WD;
    const float* src = X + n * xld;
    int cnt = 0;
    if (g.vec) {
      const int64_t a = r0 >> 2, b = r1 >> 2;  // float4 range (RB*D and W*D are multiples of 4)
      for (int64_t base = a + (int64_t)wv * TR_WAVE; base < b; base += kSpecT) {
        const int64_t e4 = base + lane;
        if (e4 < b) spec_dma16(src + 4 * e4, sX + 4 * base);
        ++cnt;
      }
    } else {
      for (int64_t base = r0 + (int64_t)wv * TR_WAVE; base < r1; base += kSpecT) {
        const int64_t e = base + lane;
        if (e < r1) spec_dma4(src + e, sX + base);
        ++cnt;
      }
    }
    return cnt;
  };
#if TR_SPEC_PROFILE
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long prof_t = 0;
#endif
  int cnt_blk[NBMAX];  // this wave's DMA instructions per block of the sample in flight
#pragma unroll
  for (int p = 0; p < NBMAX; ++p) cnt_blk[p] = 0;
  auto issue_all = [&](int64_t n) {
#pragma unroll
    for (int p = 0; p < NBMAX; ++p)
      if (p < NB) cnt_blk[p] = issue(n, p);
  };
  // wait until blocks <= p of the sample in flight are in LDS (own DMA), then barrier (everyone's)
  auto wait_block = [&](int p) {
    int later = 0;
#pragma unroll
    for (int q = 0; q < NBMAX; ++q)
      if (q > p && q < NB) later += cnt_blk[q];
#if TR_SPEC_PROFILE
    const unsigned long long w0 = __builtin_readcyclecounter();
#endif
    spec_wait_vm(later);
    spec_barrier();
#if TR_SPEC_PROFILE
    prof[5] += __builtin_readcyclecounter() - w0;
#endif
  };

  // y of the next sample is prefetched into a register one iteration ahead (thread o = t < NO)
  float ycur = (MODE == SPEC_TRAIN && nr > 0 && t < NO) ? y[sample_of(0) * NO + t] : 0.f;
  // retire the prologue's register loads with a wait the compiler sees (values first used in
  // the loop would otherwise keep a conservative vmcnt(0) inside it)
  __builtin_amdgcn_s_waitcnt(0);
  if (nr > 0 && !(TR_SPEC_SKIP & 8)) issue_all(sample_of(0));

#if TR_SPEC_PROFILE
  prof_t = __builtin_readcyclecounter();
#endif
#pragma unroll 1
  for (int64_t k = 0; k < nr; ++k) {
    const int64_t n = sample_of(k);
    const bool has_next = k + 1 < nr && !(TR_SPEC_SKIP & 8);
    // Opaque per-iteration copies of the lane index and the LDS stride: every address below is
    // recomputed inside the loop (a few SALU/VALU ops beside the MFMAs) instead of being
    // hoisted out of it into hundreds of live registers.
    int t_ = threadIdx.x, S_ = g.S;
    asm volatile("" : "+v"(t_));
    asm volatile("" : "+s"(S_));
    const int t = t_, S = S_;
    const int i = t & 15, gq = (t >> 4) & 3;

    // ---- forward GEMM, full 16-row d tiles (+ this wave group's chunks of the partial tile) ----
    const int nsets = (g.nDF + NGRP * TPW - 1) / (NGRP * TPW);
    const int nsets1 = nsets > 0 ? nsets : 1;  // set 0 also carries the waits and the partial tile
    for (int set = 0; set < nsets1; ++set) {
      int S2 = S;
      asm volatile("" : "+s"(S2));  // keep the per-step offsets inside this loop
      const bool full = set < nsets;
      const bool tail = set == 0 && g.Dtail > 0;
      tr_f32x4_s a[TPW], at = tr_f32x4_s{0.f, 0.f, 0.f, 0.f};
      const float* xa[TPW];
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        a[u] = tr_f32x4_s{0.f, 0.f, 0.f, 0.f};
        int dt = grp + NGRP * (set * TPW + u);
        dt = dt < g.nDF ? dt : (g.nDF > 0 ? g.nDF - 1 : 0);  // clamped duplicate: computed, not stored
        xa[u] = sX + 16 * gq * S2 + dt * 16 + i;
      }
      const float* xt = sX + 16 * gq * S2 + g.nDF * 16 + i;
      float xc[TPW][CHK], xn[TPW][CHK];
      auto ldchunk = [&](float(&xb)[TPW][CHK], int c) {
#pragma unroll
        for (int v = 0; v < CHK; ++v) {
          const int s = c * CHK + v;
          const int off = (64 * (s >> 4) + (s & 15)) * S2;
#pragma unroll
          for (int u = 0; u < TPW; ++u) xb[u][v] = xa[u][off];
        }
      };
#pragma unroll
      for (int ph = 0; ph < NPH; ++ph) {
        if (ph < NB) {
          if (set == 0 && !(TR_SPEC_SKIP & 8)) wait_block(ph);
          if (!(TR_SPEC_SKIP & 1)) {
            constexpr int CPP = PHS / CHK;  // chunks per phase
            if (full) ldchunk(xc, ph * CPP);
#pragma unroll
            for (int cc = 0; cc < CPP; ++cc) {
              const int c = ph * CPP + cc;
              if (full) {
                if (cc + 1 < CPP) ldchunk(xn, c + 1);
#pragma unroll
                for (int v = 0; v < CHK; ++v)
#pragma unroll
                  for (int u = 0; u < TPW; ++u) a[u] = mfma4(xc[u][v], bf[c * CHK + v], a[u]);
                if (cc + 1 < CPP) {
#pragma unroll
                  for (int v = 0; v < CHK; ++v)
#pragma unroll
                    for (int u = 0; u < TPW; ++u) xc[u][v] = xn[u][v];
                }
              }
              if (tail && c % NGRP == grp) {
#pragma unroll
                for (int v = 0; v < CHK; ++v) {
                  const int s = c * CHK + v;
                  at = mfma4(xt[(64 * (s >> 4) + (s & 15)) * S2], bf[s], at);
                }
              }
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int dt = grp + NGRP * (set * TPW + u);
        if (full && dt < g.nDF)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) sT[(dt * 16 + 4 * gq + reg) * KS + ktw * 16 + i] = a[u][reg];
      }
      if (tail) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int row = 4 * gq + reg;
          if (row < g.Dtail) sTail[(grp * g.Dtail + row) * KP + ktw * 16 + i] = at[reg];
        }
      }
    }
    if (MODE == SPEC_TRAIN && t < NO) sY[t] = ycur;
    spec_barrier();
    if (MODE != SPEC_TRAIN && has_next) issue_all(sample_of(k + 1));  // X_n is no longer read
    if (g.Dtail > 0) {  // partial d tile: sum the wave groups' partials into T
      const int d16 = 16 * g.nDF;
      for (int e = t; e < g.Dtail * K; e += kSpecT) {
        const int row = e / K, col = e - row * K;
        float v = sTail[row * KP + col];
#pragma unroll
        for (int gg = 1; gg < NGRP; ++gg) v += sTail[(gg * g.Dtail + row) * KP + col];
        sT[(d16 + row) * KS + col] = v;
      }
      spec_barrier();
    }
    TR_PROF_MARK(0);

    // ---- epilogue: column sums over d (Z, V or U) by groups of TPV lanes --------------------
    // value j is summed by lanes [j*TPV, (j+1)*TPV) over rows d = q, q + TPV, ... and reduced
    // with a fixed xor butterfly inside the group (deterministic)
    const int nred = (TR_SPEC_SKIP & 2) ? 0 : (MODE == SPEC_TRAIN ? Rn + Rs : (MODE == SPEC_PRED ? K : Rn));
    {
      const int TPV = nred <= 16 ? 32 : 16;
      const int j = t / TPV, q = t - j * TPV;
      auto tval = [&](int d, int col) -> float { return sT[d * KS + col]; };
      float v = 0.f;
      if (j < nred) {
        // rows d = q + TPV*m, m < 16 (D <= 256): unrolled so that every LDS read is in flight at once
        if (j < Rn || MODE != SPEC_TRAIN) {
          const float* ph = (j < Rn ? sPA1 + j * D : sPC1 + ((j - Rn) / Cc) * D);
          for (int m0 = 0; m0 < 16 && q + TPV * m0 < D; m0 += 8) {
            float tv[8], pv[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
              const int d = q + TPV * (m0 + m);
              tv[m] = d < D ? tval(d, j) : 0.f;
              pv[m] = d < D ? ph[d] : 0.f;
            }
#pragma unroll
            for (int m = 0; m < 8; ++m) v = fmaf(tv[m], pv[m], v);
          }
        } else {
          const int r = j - Rn;
          const float* ph = sPC1 + r * D;
          const int c0 = Rn + r * Cc;
          for (int m0 = 0; m0 < 16 && q + TPV * m0 < D; m0 += 8) {
          float ss[8], pv[8];
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const int d = q + TPV * (m0 + m);
            float acc2 = 0.f;
            if (d < D) {
              if (Cc <= 4) {
#pragma unroll
                for (int c = 0; c < 4; ++c)
                  if (c < Cc) {
                    const float x = tval(d, c0 + c);
                    acc2 = fmaf(x, x, acc2);
                  }
              } else {
                for (int c = 0; c < Cc; ++c) {
                  const float x = tval(d, c0 + c);
                  acc2 = fmaf(x, x, acc2);
                }
              }
            }
            ss[m] = acc2;
            pv[m] = d < D ? ph[d] : 0.f;
          }
#pragma unroll
          for (int m = 0; m < 8; ++m) v = fmaf(sqrtf(ss[m]), pv[m], v);
          }
        }
      }
      if (TPV == 32) v += tr_swz_xor<0x401F>(v);  // xor 16
      v += tr_swz_xor<0x201F>(v);                 // xor 8
      v += tr_swz_xor<0x101F>(v);                 // xor 4
      v += tr_swz_xor<0x081F>(v);                 // xor 2
      v += tr_swz_xor<0x041F>(v);                 // xor 1
      if (q == 0 && j < nred) sZV[j] = v;
    }
    spec_barrier();
    TR_PROF_MARK(1);

    if (MODE == SPEC_LATENT) {
      if (t < Rn) out[n * Rn + t] = sZV[t];
      continue;
    }
    if (MODE == SPEC_PRED) {
      for (int o = t; o < NO; o += kSpecT) {
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

    // ---- SPEC_TRAIN: y_hat, residual, loss and the small-factor gradients --------------------
    // lane (o, r) = (t / 32, t % 32) holds coefficient r of output o; y_hat_o by a 32-lane xor
    // butterfly; the residual (times the MSE scale) goes to sRv for the dT step
    {
      const int KR = Rn + Rs;
      const float bm = (float)((Rn > 0) + (Rs > 0));  // the bias is added by both terms (Q10)
      if (NO <= kSpecT / 32) {
        const int o = t >> 5, r = t & 31;
        const bool act = o < NO && r < KR;
        float c = 0.f, zr = 0.f;
        if (act) {
          c = r < Rn ? sPA2[o * Rn + r] : sPC2[o * Rs + (r - Rn)];
          zr = sZV[r];
        }
        float pl = r < Rn ? c * zr : 0.f;
        float ps = r < Rn ? 0.f : c * zr;
        pl += tr_swz_xor<0x401F>(pl);
        ps += tr_swz_xor<0x401F>(ps);
        pl += tr_swz_xor<0x201F>(pl);
        ps += tr_swz_xor<0x201F>(ps);
        pl += tr_swz_xor<0x101F>(pl);
        ps += tr_swz_xor<0x101F>(ps);
        pl += tr_swz_xor<0x081F>(pl);
        ps += tr_swz_xor<0x081F>(ps);
        pl += tr_swz_xor<0x041F>(pl);
        ps += tr_swz_xor<0x041F>(ps);
        if (o < NO) {
          const float b = sB[o];
          const float yh = (Rn > 0 ? pl + b : 0.f) + (Rs > 0 ? ps + b : 0.f);
          const float e = yh - sY[o];
          const float rv = e * scale;
          if (act) {
            if (r < Rn)
              sAcc[o * Rn + r] += sWt[r] * rv * zr;
            else
              sAcc[NO * Rn + o * Rs + (r - Rn)] += rv * zr;
          }
          if (r == 0) {
            sRv[o] = rv;
            sAcc[NO * KR + o] += bm * rv;
            lsum += (double)e * (double)e;
            if (out != nullptr) out[n * NO + o] = yh;
          }
        }
      } else {  // many outputs: one thread per output, then one per coefficient
        for (int o = t; o < NO; o += kSpecT) {
          const float b = sB[o];
          float yl = 0.f, ys = 0.f;
          for (int r = 0; r < Rn; ++r) yl = fmaf(sPA2[o * Rn + r], sZV[r], yl);
          for (int r = 0; r < Rs; ++r) ys = fmaf(sPC2[o * Rs + r], sZV[Rn + r], ys);
          const float yh = (Rn > 0 ? yl + b : 0.f) + (Rs > 0 ? ys + b : 0.f);
          const float e = yh - sY[o];
          const float rv = e * scale;
          sRv[o] = rv;
          sAcc[NO * KR + o] += bm * rv;
          lsum += (double)e * (double)e;
          if (out != nullptr) out[n * NO + o] = yh;
        }
        spec_barrier();
        for (int e2 = t; e2 < NO * KR; e2 += kSpecT) {
          const int o = e2 / KR, r = e2 - o * KR;
          const float rv = sRv[o];
          if (r < Rn)
            sAcc[o * Rn + r] += sWt[r] * rv * sZV[r];
          else
            sAcc[NO * Rn + o * Rs + (r - Rn)] += rv * sZV[r];
        }
      }
    }
    spec_barrier();
    // dZ_j / dV_j = sum_o residual_o * coefficient(o, j)  (one thread per coefficient column)
    if (t < Rn + Rs) {
      float dz = 0.f;
      if (t < Rn)
        for (int o = 0; o < NO; ++o) dz = fmaf(sRv[o], sPA2[o * Rn + t], dz);  // sPA2 = w_r phi(A2)
      else
        for (int o = 0; o < NO; ++o) dz = fmaf(sRv[o], sPC2[o * Rs + (t - Rn)], dz);
      sDZ[t] = dz;
    }
    spec_barrier();
    TR_PROF_MARK(2);
    // dT_n in place and the A1 / C1 gradients, one (d, j) item per lane (all 512 lanes busy)
#pragma unroll
    for (int m = 0; m < AMAX; ++m) {
      const int e = t + kSpecT * m;
      if (e < nitems) {
        int j, d;
        item(e, j, d);
        float* Tw = sT + d * KS;
        const float dz = sDZ[j];
        if (j < Rn) {
          const float tv = Tw[j];
          const float ph = sPA1[j * D + d];
          acc[m] = fmaf(dz, tv, acc[m]);
          Tw[j] = dz * ph;
        } else {
          const int r = j - Rn;
          float* tp = Tw + Rn + r * Cc;
          const float ph = sPC1[r * D + d];
          if (Cc <= 4) {
            float xv[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) xv[c] = c < Cc ? tp[c] : 0.f;
            float ss = 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c) ss = fmaf(xv[c], xv[c], ss);
            const float mg = sqrtf(ss);
            acc[m] = fmaf(dz, mg, acc[m]);
            const float qq = mg > 0.f ? dz * ph * __builtin_amdgcn_rcpf(mg) : 0.f;
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (c < Cc) tp[c] = qq * xv[c];
          } else {
            float ss = 0.f;
            for (int c = 0; c < Cc; ++c) ss = fmaf(tp[c], tp[c], ss);
            const float mg = sqrtf(ss);
            acc[m] = fmaf(dz, mg, acc[m]);
            const float qq = mg > 0.f ? dz * ph * __builtin_amdgcn_rcpf(mg) : 0.f;
            for (int c = 0; c < Cc; ++c) tp[c] *= qq;
          }
        }
      }
    }
    // y of the next sample (issued before this sample's DMA, so the counted waits stay exact)
    if (k + 1 < nr && t < NO) ycur = y[sample_of(k + 1) * NO + t];
    spec_barrier();
    TR_PROF_MARK(3);

    // ---- gradient GEMM by row blocks: dPhi0[w, k] += sum_d X_n[w, d] dT_n[d, k] ----------------
    // wave = (w tiles 8p + grp + NGRP*u, column tile ktw); step s covers d = 64*(s/16) + 16*j +
    // s%16 (conflict-free A and B reads; rows d >= D read the zero row D of dT); 4-step chunks,
    // the next chunk's loads issued right behind the current chunk's MFMAs
    const int nch = (g.DS + 3) >> 2;
#pragma unroll
    for (int p = 0; p < NBMAX; ++p) {
      if (p < NB) {
        if (!(TR_SPEC_SKIP & 4)) {
          const float* xw[KT];
          bool wok[KT];
#pragma unroll
          for (int u = 0; u < KT; ++u) {
            const int wt = 8 * p + grp + NGRP * u;
            wok[u] = wt < g.nWT;
            xw[u] = sX + ((wok[u] ? wt : 0) * 16 + i) * S + 16 * gq;
          }
          const float* tb = sT + ktw * 16 + i;
          float xA[KT][4], xB[KT][4], bA[4], bB[4];
          auto ld = [&](float(&xx)[KT][4], float(&bb)[4], int c) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int st = 4 * c + v;
              const int d0 = 64 * (st >> 4) + (st & 15);
              const int d = d0 + 16 * gq;
#pragma unroll
              for (int u = 0; u < KT; ++u) xx[u][v] = xw[u][d0];
              bb[v] = tb[(d < D ? d : D) * KS];
            }
          };
          auto mm = [&](const float(&xx)[KT][4], const float(&bb)[4]) {
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
              for (int u = 0; u < KT; ++u) gacc[p][u][v & 1] = mfma4(xx[u][v], bb[v], gacc[p][u][v & 1]);
          };
          ld(xA, bA, 0);
          for (int c = 0; c < nch; c += 2) {
            mm(xA, bA);
            if (c + 1 < nch) {
              ld(xB, bB, c + 1);
              mm(xB, bB);
            }
            if (c + 2 < nch) ld(xA, bA, c + 2);
          }
        }
        if (has_next) {
#if TR_SPEC_PROFILE
          const unsigned long long w0 = __builtin_readcyclecounter();
#endif
          spec_barrier();  // every wave's reads of rows [RB*p, RB*(p+1)) have retired
          cnt_blk[p] = issue(sample_of(k + 1), p);
#if TR_SPEC_PROFILE
          prof[6] += __builtin_readcyclecounter() - w0;
#endif
        }
      }
    }
    TR_PROF_MARK(4);
  }

#if TR_SPEC_PROFILE
  if (t == 0 && blockIdx.x < 256)
    for (int q = 0; q < 8; ++q) g_spec_prof[blockIdx.x][q] = prof[q];
#endif
  if (MODE != SPEC_TRAIN) return;
  __syncthreads();
  // ---- per-workgroup slab (arena layout, phi space) ------------------------------------------
  {
    const int i = lane & 15, gq = lane >> 4;
#pragma unroll
    for (int p = 0; p < NBMAX; ++p)
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const int wt = 8 * p + grp + NGRP * u;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int w = wt * 16 + 4 * gq + reg, kk = ktw * 16 + i;
          if (p < NB && wt < g.nWT && w < g.W && kk < K) {
            const int64_t dst =
                kk < Rn ? g.offA0 + (int64_t)w * Rn + kk : g.offC0 + (int64_t)w * Rs * Cc + (kk - Rn);
            sl[dst] = gacc[p][u][0][reg] + gacc[p][u][1][reg];
          }
        }
      }
  }
#pragma unroll
  for (int m = 0; m < AMAX; ++m) {
    const int e = t + kSpecT * m;
    if (e < nitems) {
      int j, d;
      item(e, j, d);
      if (j < Rn)
        sl[g.offA1 + (int64_t)d * Rn + j] = acc[m];
      else
        sl[g.offC1 + (int64_t)d * Rs + (j - Rn)] = acc[m];
    }
  }
  for (int e = t; e < NO * Rn; e += kSpecT) sl[g.offA2 + e] = sAcc[e];
  for (int e = t; e < NO * Rs; e += kSpecT) sl[g.offC2 + e] = sAcc[NO * Rn + e];
  for (int e = t; e < NO; e += kSpecT) sl[g.offB + e] = sAcc[NO * (Rn + Rs) + e];
  // data loss partial: fixed-order block reduction (each output's thread accumulated its own)
  {
    double* dred = reinterpret_cast<double*>(lds + g.oRed);
    const double ls = tr_wave_allreduce_d(lsum);
    __syncthreads();
    if (lane == 0) dred[wv] = ls;
    __syncthreads();
    if (t == 0) {
      double tot = 0.0;
      for (int w = 0; w < NW; ++w) tot += dred[w];
      dpart[2 * blockIdx.x] = tot;
      dpart[2 * blockIdx.x + 1] = 0.0;
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static inline int cdiv_i(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
static inline int round4(int64_t a) { return (int)((a + 3) & ~(int64_t)3); }

bool spec_geom_init(SpecGeom* g, int64_t W, int64_t D, int64_t NO, int Rn, int Rs, int Cc, const int32_t* nonneg,
                    std::string* why) {
  std::memset(g, 0, sizeof(*g));
  if (W < 1 || D < 1 || NO < 1 || Rn < 0 || Rs < 0 || Cc < 1) {
    *why = "spectral dims / ranks out of range";
    return false;
  }
  const int64_t K = Rn + (int64_t)Rs * Cc;
  if (Rn + Rs < 1) {
    *why = "rank_normal + rank_spectral must be >= 1";
    return false;
  }
  if (K > 256) {
    *why = "rank_normal + rank_spectral*(n_complex_dim+1) > 256 is outside the gfx950 spectral kernels";
    return false;
  }
  if (W > (1 << 24) || D > (1 << 16) || NO > (1 << 16)) {
    *why = "spectral dims out of range";
    return false;
  }
  // the fused single-pass kernel holds one sample + scratch in a CU's LDS; beyond that (or when
  // forced) the generic path stages T_n through HBM (tr_spectral_gen.hip)
  const char* force = std::getenv("TR_SPEC_GENERIC");
  bool fused_ok = K <= 32 && W <= 256 && D <= 256 && NO <= 256 && !(force != nullptr && force[0] == '1');
  g->W = (int)W;
  g->D = (int)D;
  g->NO = (int)NO;
  g->Rn = Rn;
  g->Rs = Rs;
  g->Cc = Cc;
  g->K = (int)K;
  g->KT = cdiv_i(K, 16);
  g->S = (int)D;  // lane-linear LDS image of the sample (LDS-DMA); odd D => conflict-free MFMA reads
  g->KS = 16 * g->KT + 1;
  g->nWT = cdiv_i(W, 16);
  g->Wrows = 128 * cdiv_i(W, 128);  // zero-padded rows: the forward walks whole 128-row blocks
  g->nDF = (int)(D / 16);
  g->Dtail = (int)(D % 16);
  g->WS = g->Wrows / 4;  // forward k steps over the zero-padded row blocks
  g->DS = 16 * (int)(D / 64) + (int)((D % 64) < 16 ? (D % 64) : 16);  // steps of the 64-block walk
  g->WD = W * D;
  g->vec = (g->WD % 4) == 0 ? 1 : 0;  // 16-B DMA pieces (else 4-B)
  int64_t off = 0;
  g->offA0 = off;
  off += W * Rn;
  g->offA1 = off;
  off += D * Rn;
  g->offA2 = off;
  off += NO * Rn;
  g->offC0 = off;
  off += W * Rs * Cc;
  g->offC1 = off;
  off += D * Rs;
  g->offC2 = off;
  off += NO * Rs;
  g->offB = off;
  off += NO;
  g->nparams = off;
  for (int f = 0; f < 3; ++f) g->nonneg[f] = nonneg ? (nonneg[f] != 0) : 0;
  // LDS carve
  const int XF = round4((int64_t)g->Wrows * g->S + 128);  // pad: the 64-block walks overrun row W-1
  const int TF = round4((int64_t)(D + 1) * g->KS);  // + one zero row (the gradient GEMM's pad rows)
  const int TailF = kSpecNW * g->Dtail * 16 * g->KT;
  const int RedF = 64;  // loss reduction (one double per wave)
  const int SmF = round4(64 + 256 + NO);  // Z/V (or U), residuals, y
  const int AccF = round4(NO * (int64_t)(Rn + Rs + 1));
  g->oT = XF;
  g->oTail = g->oT + TF;
  g->oRed = g->oTail + TailF;
  g->oSm = g->oRed + RedF;
  g->oAcc = g->oSm + SmF;
  g->oPhi = g->oAcc + AccF;
  const int PhiF = round4((D + NO) * (int64_t)(Rn + Rs) + NO + Rn + Rs);
  g->lds_floats = g->oPhi + PhiF;
  if (fused_ok && (int64_t)g->lds_floats * 4 > 160 * 1024) fused_ok = false;
  g->gKP = 16 * cdiv_i(K, 16);
  g->gen = fused_ok ? 0 : 1;
  spec_slice_geom(g);  // the column-slice training kernel where it covers the shape
  if (g->gen) {
    g->KT = g->gKP / 16;
    if (specg_epi_lds_bytes(*g) > 160 * 1024 - 256) {  // (+ the kernel's static loss scratch)
      *why = "the spectral epilogue of one sample (X.shape[2] * (K + 1) + (X.shape[2] + n_out) * (rank_normal + "
             "rank_spectral) floats) exceeds the 160 KiB LDS of a CU";
      return false;
    }
  }
  return true;
}

template <int MODE, int WSMAX, int KT>
struct SpecInst {
  static const void* ptr() { return reinterpret_cast<const void*>(&k_spec_fused<MODE, WSMAX, KT>); }
  static hipError_t launch(const SpecGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                           const float* Phi0, const float* wts, const float* y, float scale, float* slab,
                           int64_t slab_stride, double* dpart, float* out, int64_t rpw, int reverse,
                           const int32_t* stop, hipStream_t st) {
    hipLaunchKernelGGL((k_spec_fused<MODE, WSMAX, KT>), dim3(grid), dim3(kSpecT), (size_t)g.lds_floats * 4, st,
                       X, N, xld, g, phi, Phi0, wts, y, scale, slab, slab_stride, dpart, out, rpw, reverse, stop);
    return hipGetLastError();
  }
};

// instantiation for (mode, forward k-step bound, column tiles)
template <template <int, int, int> class F, typename... A>
static auto spec_dispatch(const SpecGeom& g, int mode, A... a) {
  const bool small = g.WS <= 32;  // W <= 128: 32 forward k steps
  const bool kt1 = g.KT == 1;
#define TR_SPEC_CASE(M)                                      \
  if (mode == M) {                                           \
    if (small) return kt1 ? F<M, 32, 1>::call(a...) : F<M, 32, 2>::call(a...); \
    return kt1 ? F<M, 64, 1>::call(a...) : F<M, 64, 2>::call(a...);            \
  }
  TR_SPEC_CASE(SPEC_TRAIN)
  TR_SPEC_CASE(SPEC_PRED)
#undef TR_SPEC_CASE
  if (small) return kt1 ? F<SPEC_LATENT, 32, 1>::call(a...) : F<SPEC_LATENT, 32, 2>::call(a...);
  return kt1 ? F<SPEC_LATENT, 64, 1>::call(a...) : F<SPEC_LATENT, 64, 2>::call(a...);
}

template <int M, int WSMAX, int KT>
struct SpecPtr {
  static const void* call() { return SpecInst<M, WSMAX, KT>::ptr(); }
};
template <int M, int WSMAX, int KT>
struct SpecLaunch {
  template <typename... A>
  static hipError_t call(A... a) { return SpecInst<M, WSMAX, KT>::launch(a...); }
};

static const void* spec_kernel_for(const SpecGeom& g, int mode) { return spec_dispatch<SpecPtr>(g, mode); }

hipError_t spec_prepare(const SpecGeom& g, int mode, int* ok) {
  *ok = 0;
  if (g.gen) {
    *ok = 1;
    return mode == SPEC_TRAIN ? specg_prepare(g) : hipSuccess;
  }
  const void* k = spec_kernel_for(g, mode);
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g.lds_floats * 4);
  if (e != hipSuccess) return e;
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kSpecT, (size_t)g.lds_floats * 4);
  if (e != hipSuccess) return e;
  *ok = per_cu >= 1;
  return hipSuccess;
}

hipError_t launch_spec_prep(const SpecGeom& g, const float* params, float beta, float thr, float* phi,
                            float* dphi, float* Phi0, const int32_t* stop, hipStream_t st) {
  const int64_t n = g.nparams + (int64_t)g.W * g.K;
  int blocks = cdiv_i(n, 256);
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(k_spec_prep, dim3(blocks), dim3(256), 0, st, g, params, beta, thr, phi, dphi, Phi0, stop);
  return hipGetLastError();
}

hipError_t launch_spec_fused(int mode, const SpecGeom& g, int grid, const float* X, int64_t N, int64_t xld,
                             const float* phi,
                             const float* Phi0, const float* wts, const float* y, float scale, float* slab,
                             int64_t slab_stride, double* dpart, float* out, int64_t rows_per_wg, int reverse,
                             const int32_t* stop, hipStream_t st) {
return spec_dispatch<SpecLaunch>(g, mode, g, grid, X, N, xld, phi, Phi0, wts, y, scale, slab, slab_stride, dpart, out,
                                   rows_per_wg, reverse, stop, st);
}

#if TR_SPEC_PROFILE
}  // namespace tr
extern "C" int tr_spec_profile_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spec_prof), sizeof(g_spec_prof));
}
namespace tr {
#endif

hipError_t launch_spec_chain(int64_t n, const float* G, const float* dphi, float* grad, const int32_t* stop,
                             hipStream_t st) {
  int blocks = cdiv_i(n, 256);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_spec_chain, dim3(blocks), dim3(256), 0, st, n, G, dphi, grad, stop);
  return hipGetLastError();
}

}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_spectral() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_spec_prep));
}
}  // namespace tr
