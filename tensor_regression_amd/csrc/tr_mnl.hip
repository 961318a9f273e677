// tr_mnl.hip — single pass over X for the multinomial model with two feature modes
// (BASELINE config 3: X (65536, 128, 64), 10 classes, rank 8).
//
// Replaces the forward `softmax(inner(X, cp_to_tensor(w, Phi)))` (multinomial…py:148-187), the
// CrossEntropyLoss on those probabilities (:448-456, the double softmax) and the autograd
// backward (:457) — which the reference runs as two (N x P) . (P x C) GEMMs, i.e. two passes over
// X.  Here each X row crosses HBM once and the dense (P x C) coefficient tensor is never built:
// with B[i, j, c] = sum_r w_r Phi0[i, r] Phi1[j, r] PhiC[c, r] the per-sample chain is
//     T[i, r] = sum_j X_n[i, j] Phi1[j, r]        V[j, r] = sum_i X_n[i, j] Phi0[i, r]
//     U[r]    = sum_i Phi0[i, r] T[i, r]          Z[c]    = sum_r w_r PhiC[c, r] U[r]
//     S = softmax(Z), Q = softmax(S), CE = -log Q[y]; dZ = S * (dS - <dS, S>), dS = (Q - e_y) cw_y / W
//     Wv[r]   = w_r sum_c dZ[c] PhiC[c, r]
//     dPhi0[i, r] += Wv[r] T[i, r]    dPhi1[j, r] += Wv[r] V[j, r]    dPhiC[c, r] += w_r dZ[c] U[r]
// (the same numbers as autograd through cp_to_tensor + inner, re-associated).  Both T and V
// are independent of the epilogue, so both GEMMs run as soon as X_n is in LDS.
//
// Work split (512 threads, one workgroup per CU, contiguous sample range):
//   * X_n lands in an LDS ring (nbuf samples) by LDS-DMA (global_load_lds_dwordx4), the chunk
//     index of row i XOR-swizzled by (i & smask) through the per-lane source address, so both
//     GEMM orientations read LDS conflict-free; nbuf - 1 samples are in flight.
//   * GEMM units: a unit is 64 output rows x a 64-deep k range x 4 ranks of T or V on
//     v_mfma_f32_4x4x1_16b_f32 (lane l = output row, 4 ranks per block: no rank padding).  Its B
//     operand (64 factor values per lane) stays in registers for the whole launch.
//   * Epilogue of sample n-1 runs after the barrier of sample n (one barrier per sample): every
//     wave sums the A-units' U partials (fixed order), forms Z / softmax / CE / dZ in a 16-lane
//     DPP row, and scales its own units' T / V into register accumulators; wave 0 keeps dPhiC
//     and the loss.
//   * End: units add their accumulators into an LDS image of the arena in fixed unit order;
//     the workgroup writes one phi-space slab (k_reduce_slabs sums the slabs in index order,
//     k_spec_chain applies softplus').  No float atomics: runs are bitwise reproducible.
#include <cstdlib>
#include <cstring>

#include "tr_common.h"
#include "tr_mnl.h"


// The ring refill is issued between GEMM steps (a burst after the barrier stalled on the memory
// issue queue), and the first MN_HOIST operand quads of pair member a are loaded before the
// previous pair's epilogue.
constexpr int MN_HOIST = 4;
#ifndef TR_MNL_PROFILE
#define TR_MNL_PROFILE 0  // profiling build only: per-phase cycle counts of every wave of WG 0..255
#endif
#if TR_MNL_PROFILE
__device__ unsigned long long g_mnl_prof[256][8][8];
#define TR_MNL_MARK(ph)                                           \
  do {                                                            \
    const unsigned long long _now = __builtin_readcyclecounter(); \
    prof[ph] += _now - prof_t;                                    \
    prof_t = _now;                                                \
  } while (0)
#else
#define TR_MNL_MARK(ph) \
  do {                  \
  } while (0)
#endif

namespace tr {

namespace {
constexpr int MN_NW = 8;
constexpr int MN_T = MN_NW * TR_WAVE;
typedef float mn_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ mn_f32x4 mfma_4x4(float a, float b, mn_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// 16-lane row reductions by DPP: quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror,
// row_mirror.  Each step adds the same two operands in every lane of a pair, so all 16 lanes
// end with the bitwise-identical value.
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return v;
}
// v_permlane16_swap / v_permlane32_swap (CDNA4) of a value with itself: the two results hold, in
// every lane, the lane's own row pair / half and the partner's, so their sum is the xor-16 /
// xor-32 butterfly step without an LDS round trip (ds_bpermute).  Same operand order in every
// lane: bitwise-identical results across the pair.
__device__ __forceinline__ float xor16_sum(float v) {
  const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
// (lower-half value, upper-half value) of v at lane (l mod 32) and (l mod 32) + 32, in every lane
__device__ __forceinline__ void halves(float v, float& lo, float& hi) {
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  lo = __uint_as_float(q[0]);
  hi = __uint_as_float(q[1]);
}
__device__ __forceinline__ float rfl(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// LDS barrier that leaves LDS-DMA in flight (__syncthreads() would wait vmcnt(0))
__device__ __forceinline__ void mn_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// One LDS-DMA piece per lane (16 B from gsrc to LDS byte address m0 + 16 * lane), issued from
// inline asm: the compiler then does not see an LDS write in flight and does not put an
// s_waitcnt vmcnt(0) in front of every later LDS read (it cannot tell the ring slot being
// filled from the one being read).  The kernel orders the pieces itself: counted vmcnt waits
// (mn_wait_vm) + barrier before a slot is read, barrier before a slot is refilled.
__device__ __forceinline__ void mn_dma16(const float* gsrc, const float* lds_dst) {
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)lds_dst);
  uint32_t keep;  // m0 is compiler-reserved: save and restore it inside the statement
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(a)
               : "memory");  // (without the clobber the compiler may move LDS reads across it)
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (stricter than asked above 31: still safe)
__device__ __forceinline__ void mn_wait_vm(int n) {
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
      asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
  }
#undef TR_VM_CASE
}
}  // namespace

enum { MN_ROLE_A = 0, MN_ROLE_B = 1, MN_ROLE_IDLE = 2 };

struct MnArgs {
  const float* X;
  int64_t N, xld;
  const float* phi;
  const float* w;
  const int64_t* lab;
  const float* class_w;
  float scale;
  float* gpart;
  double* dpart;
  int64_t rows_per_wg;
  int reverse;
};

// The whole per-workgroup pipeline for one wave role (A-unit, B-unit, or no unit), so that no
// role branch sits inside the sample loop and the compiler can interleave the epilogue of
// sample k-1 with the GEMM of sample k.
//
// A-unit (ib, jb, rb): lane l = X row i = 64 ib + l; 16 steps of one ds_read_b128 (4 j) and
//   4 MFMAs with B = Phi1[j][4 rb + (l & 3)] (64 registers); the 16 x 4x4 blocks are 64 rows x
//   4 ranks of T.  Then U partial -> Z partial of this unit (16 classes) -> LDS.
// B-unit (jb, ib, rb): the 16 blocks take DIFFERENT k (rows i = 64 ib + 4 s + (l >> 4) at step
//   s): lane l reads X[i][64 jb + 4 (l & 15) .. +3] with one ds_read_b128 and feeds 4 MFMAs
//   (one per float of the read, 4 accumulators), B = Phi0[i][4 rb + (l & 3)] (16 registers).
//   Accumulator q, register v of lane 4b + n holds V[j = 64 jb + 16 (b & 3) + 4 v + q]
//   [r = 4 rb + n] summed over the rows with (i - 64 ib) & 3 == b >> 2; the four row classes
//   are added once, at the end (everything per sample is linear in V).
template <int ROLE, bool FULL, int SPI>
__device__ __forceinline__ void mnl_body(const MnlGeom& g, const MnArgs& a, const int64_t* __restrict__ lab,
                                         const float* __restrict__ class_w, float* lds, const int wv,
                                         const int lane) {
  const int t = threadIdx.x;
  const int I = g.I, J = g.J, R = g.R, C = g.C;
  const int SPF = I * J;
  float* sZ = lds + g.oZ;  // [2][SPI][16][4] Z partials of the A-units (unused entries stay zero)
  const float* P0 = a.phi;
  const float* P1 = a.phi + g.offP1;
  const float* PC = a.phi + g.offPC;
  const int c = lane & 15, grow = lane >> 4;
  const bool cok = c < C;
  // class weight of class c in lane c of every 16-lane row: a label's weight is one readlane, not
  // a second scalar load that waits on the label load (and, through lgkmcnt, on the GEMM's LDS reads)
  const float cwl = cok ? class_w[c] : 0.f;

  int ib = 0, jb = 0, rb = 0;
  if (ROLE == MN_ROLE_A) {
    rb = wv % g.nrb;
    const int q = wv / g.nrb;
    jb = q % g.njb;
    ib = q / g.njb;
  } else if (ROLE == MN_ROLE_B) {
    const int u2 = wv - g.nA;
    rb = u2 % g.nrb;
    const int q = u2 / g.nrb;
    ib = q % g.nib;
    jb = q / g.nib;
  }
  const int rq = 4 * rb + (lane & 3);  // rank of this lane's accumulator column
  const bool rqv = rq < R;
  const int klen = ROLE == MN_ROLE_A ? (J - 64 * jb < 64 ? J - 64 * jb : 64) : (I - 64 * ib < 64 ? I - 64 * ib : 64);
  constexpr int NB = ROLE == MN_ROLE_A ? 64 : 16;
  float bop[NB];
  float phiU[4] = {0.f, 0.f, 0.f, 0.f}, wpc[4] = {0.f, 0.f, 0.f, 0.f};
  float pcg = 0.f, wg = 0.f;
  if (ROLE == MN_ROLE_A) {
#pragma unroll
    for (int k = 0; k < 64; ++k) bop[k] = (rqv && k < klen) ? P1[(int64_t)(64 * jb + k) * R + rq] : 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = 64 * ib + 4 * (lane >> 2) + v;
      phiU[v] = (rqv && row < I) ? P0[(int64_t)row * R + rq] : 0.f;
      const int r = 4 * rb + v;
      wpc[v] = (cok && r < R) ? a.w[r] * PC[c * R + r] : 0.f;
    }
    wg = 4 * rb + grow < R ? a.w[4 * rb + grow] : 0.f;
  } else if (ROLE == MN_ROLE_B) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * s + grow;
      bop[s] = (rqv && k < klen) ? P0[(int64_t)(64 * ib + k) * R + rq] : 0.f;
    }
  }
  // pairs: Wv needs 4 ranks per member but a member has 2 rows: two passes of rows (rank
  // q = 2 pass + (g & 1)), weights pcp0 / pcp1
  float pcp0 = 0.f, pcp1 = 0.f;
  if (ROLE != MN_ROLE_IDLE) {
    const int r = 4 * rb + grow;
    pcg = (cok && r < R) ? a.w[r] * PC[c * R + r] : 0.f;
    const int r0 = 4 * rb + (grow & 1), r1 = 4 * rb + 2 + (grow & 1);
    pcp0 = (cok && r0 < R) ? a.w[r0] * PC[c * R + r0] : 0.f;
    pcp1 = (cok && r1 < R) ? a.w[r1] * PC[c * R + r1] : 0.f;
  }

  // LDS-DMA map: wave wv issues groups gi (64 chunks = 1 KiB each) = wv + 8 gi of every sample
  const int ngroups = (g.nchunk + TR_WAVE - 1) / TR_WAVE;
  const int gcnt = ngroups > wv ? (ngroups - wv + MN_NW - 1) / MN_NW : 0;
  int goff[kMnlGMax];
#pragma unroll
  for (int gi = 0; gi < kMnlGMax; ++gi) {
    const int slot = (wv + MN_NW * gi) * TR_WAVE + lane;
    if (gi < gcnt && slot < g.nchunk) {
      const int i = slot / g.JQ;
      const int q = slot - i * g.JQ;
      goff[gi] = i * J + 4 * (q ^ (i & g.smask));
    } else {
      goff[gi] = -1;
    }
  }
  const int64_t n0 = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t n1 = n0 + a.rows_per_wg < a.N ? n0 + a.rows_per_wg : a.N;
  const int64_t nr = n1 > n0 ? n1 - n0 : 0;
  auto sample_of = [&](int64_t k) -> int64_t { return a.reverse ? (n1 - 1 - k) : (n0 + k); };
  // (the sample's base pointers are formed once per call site; FULL shapes have every piece of
  // every group valid, so no per-lane test -- and no exec-mask branch -- around the DMA)
  auto issue_at = [&](const float* src, float* dst, int gi) {
    if (FULL || goff[gi] >= 0) mn_dma16(src + goff[gi], dst + MN_NW * gi * 256);
  };
  auto dma_src = [&](int64_t n) { return a.X + n * a.xld; };
  auto dma_dst = [&](int buf) { return lds + buf * SPF + wv * 256; };
  auto issue_group = [&](int64_t n, int buf, int gi) { issue_at(dma_src(n), dma_dst(buf), gi); };

  for (int e = t; e < 4 * 16 * 4; e += MN_T) sZ[e] = 0.f;
  __syncthreads();
  // Retire every register load of the prologue with a wait the compiler sees: otherwise values
  // first used inside the loop keep a conservative s_waitcnt vmcnt(0) in the loop body, which
  // would also drain the LDS-DMA ring on every sample.
  __builtin_amdgcn_s_waitcnt(0);
  const int nbuf = g.nbuf;

  mn_f32x4 gacc[4];  // A: gacc[0] (rows x ranks of dPhi0); B: all four (dPhi1 by row class)
#pragma unroll
  for (int q = 0; q < 4; ++q) gacc[q] = mn_f32x4{0.f, 0.f, 0.f, 0.f};
  float dpc = 0.f;  // A: dPhiC[c][4 rb + grow]
  double lsum = 0.0;
  const float NEG = -__builtin_huge_valf();
  const int l3 = lane & 3;

  // GEMM of the sample in ring slot `buf`: A-units T (summed into acc[0]) and their Z partial
  // -> sZ[zidx]; B-units V (acc[0..3]).  u0..u3: the A-unit's U partial (ranks 4 rb + q).
  // dma_on: also issue this wave's LDS-DMA pieces of sample dma_n into ring slot dma_buf, one
  // piece every other k step between the MFMAs (a burst of them right after the barrier stalls
  // on the vector-memory issue queue)
  // the member's X operands from ring slot `buf` into xr (issued early by the pair loop, so that
  // their LDS latency hides under the previous pair's epilogue)
  auto load1 = [&](int buf, float4(&xr)[16], int s0 = 0, int s1 = 16) {
    const float* sb = lds + buf * SPF;
    if (ROLE == MN_ROLE_A) {
      int row = 64 * ib + lane;
      if (!FULL) row = row < I ? row : I - 1;
      const float* rp = sb + row * J;
      const int sw = row & g.smask;
#pragma unroll
      for (int c4 = 0; c4 < 16; ++c4)
        if (c4 >= s0 && c4 < s1 && (FULL || 4 * c4 < klen))
          xr[c4] = *reinterpret_cast<const float4*>(rp + 4 * ((16 * jb + c4) ^ sw));
    } else if (ROLE == MN_ROLE_B) {
      int cq = 16 * jb + c;
      if (!FULL) cq = cq < g.JQ ? cq : g.JQ - 1;
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        if (st >= s0 && st < s1 && (FULL || 4 * st < klen)) {
          int i = 64 * ib + 4 * st + grow;
          if (!FULL) i = i < I ? i : I - 1;
          xr[st] = *reinterpret_cast<const float4*>(sb + i * J + 4 * (cq ^ (i & g.smask)));
        }
      }
    }
  };
  // GEMM of the sample whose operands are in xr: A-units T (summed into acc[0]) and their Z
  // partial -> sZ[zidx]; B-units V (acc[0..3]).  u0..u3: the A-unit's U partial (ranks 4 rb + q).
  // dma_on: also issue this wave's LDS-DMA pieces of sample dma_n into ring slot dma_buf, one
  // piece every other k step between the MFMAs (a burst of them right after the barrier stalls
  // on the vector-memory issue queue)
  auto gemm1 = [&](const float4(&xr)[16], int zidx, mn_f32x4(&acc)[4], float& u0, float& u1, float& u2, float& u3,
                   bool dma_on, int64_t dma_n, int dma_buf) {
    const float* dsrc = dma_on ? dma_src(dma_n) : a.X;
    float* ddst = dma_dst(dma_buf);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = mn_f32x4{0.f, 0.f, 0.f, 0.f};
    if (ROLE == MN_ROLE_A) {
#pragma unroll
      for (int c4 = 0; c4 < 16; ++c4) {
        if (dma_on && (c4 & 1) == 0 && (c4 >> 1) < gcnt) issue_at(dsrc, ddst, c4 >> 1);
        if (FULL || 4 * c4 < klen) {
          acc[0] = mfma_4x4(xr[c4].x, bop[4 * c4 + 0], acc[0]);
          acc[1] = mfma_4x4(xr[c4].y, bop[4 * c4 + 1], acc[1]);
          acc[2] = mfma_4x4(xr[c4].z, bop[4 * c4 + 2], acc[2]);
          acc[3] = mfma_4x4(xr[c4].w, bop[4 * c4 + 3], acc[3]);
        }
      }
      acc[0] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      float u = phiU[0] * acc[0].x;
      u = fmaf(phiU[1], acc[0].y, u);
      u = fmaf(phiU[2], acc[0].z, u);
      u = fmaf(phiU[3], acc[0].w, u);
      u += dpp_f<0x124>(u);  // row_ror:4
      u += dpp_f<0x128>(u);  // row_ror:8
      u = xor16_sum(u);
      u = xor32_sum(u);
      u0 = rdl(u, 0);
      u1 = rdl(u, 1);
      u2 = rdl(u, 2);
      u3 = rdl(u, 3);
      float zpart = wpc[0] * u0;
      zpart = fmaf(wpc[1], u1, zpart);
      zpart = fmaf(wpc[2], u2, zpart);
      zpart = fmaf(wpc[3], u3, zpart);
      if (lane < 16) sZ[(zidx * 16 + lane) * 4 + wv] = zpart;
    } else {
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        if (dma_on && (st & 1) == 0 && (st >> 1) < gcnt) issue_at(dsrc, ddst, st >> 1);
        if (FULL || 4 * st < klen) {
          acc[0] = mfma_4x4(xr[st].x, bop[st], acc[0]);
          acc[1] = mfma_4x4(xr[st].y, bop[st], acc[1]);
          acc[2] = mfma_4x4(xr[st].z, bop[st], acc[2]);
          acc[3] = mfma_4x4(xr[st].w, bop[st], acc[3]);
        }
      }
    }
  };
  // double softmax + weighted CE of the 16-lane row (lane c = class): returns dZ[c], adds wave
  // 0's loss term for the lanes `loss_lanes` select
  auto softmax_ce = [&](float z, int64_t y, float cw, bool loss_lanes) -> float {
    const float zz = cok ? z : NEG;
    const float mx = row_max16(zz);
    const float ez = cok ? expf(zz - mx) : 0.f;
    const float sum = row_sum16(ez);
    const float S = ez * __builtin_amdgcn_rcpf(sum);  // softmax (model, multinomial…py:187)
    const float m2 = row_max16(cok ? S : NEG);
    const float q = cok ? expf(S - m2) : 0.f;
    const float s2 = row_sum16(q);
    const bool is_y = cok && (int64_t)c == y;
    const float dS = cok ? (q * __builtin_amdgcn_rcpf(s2) - (is_y ? 1.0f : 0.0f)) * (cw * a.scale) : 0.f;
    const float dot = row_sum16(dS * S);
    if (ROLE == MN_ROLE_A) {
      const float ce = -((S - m2) - logf(s2));  // CrossEntropyLoss on the probabilities
      lsum += (wv == 0 && is_y && loss_lanes) ? (double)cw * (double)ce : 0.0;
    }
    return cok ? S * (dS - dot) : 0.f;
  };
#if TR_MNL_PROFILE
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long prof_t = __builtin_readcyclecounter();
#endif

  if constexpr (SPI == 1) {
    // ---- one sample per barrier: epilogue of k-1, then GEMM of k ----
    for (int64_t k = 0; k < nbuf - 1 && k < nr; ++k)
#pragma unroll
      for (int gi = 0; gi < kMnlGMax; ++gi)
        if (gi < gcnt) issue_group(sample_of(k), (int)k, gi);
    mn_f32x4 accP[4], accC[4];
    float uP0 = 0.f, uP1 = 0.f, uP2 = 0.f, uP3 = 0.f, uC0 = 0.f, uC1 = 0.f, uC2 = 0.f, uC3 = 0.f;
    int64_t yP = 0, yC = 0;
    float cwP = 0.f, cwC = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) accP[q] = accC[q] = mn_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t k = 0; k <= nr; ++k) {
      if (k < nr) {
        int64_t ahead = nr - 1 - k;
        if (ahead > nbuf - 2) ahead = nbuf - 2;
        mn_wait_vm(gcnt * (int)ahead);  // sample k has landed (this wave's pieces)
      }
      TR_MNL_MARK(0);
      mn_barrier();  // every wave's pieces of sample k; Z partials of k - 1; slot (k - 1) % nbuf free
      TR_MNL_MARK(1);
      const bool pre = k + nbuf - 1 < nr;  // refill slot (k - 1) % nbuf with sample k + nbuf - 1
      const int64_t npre = pre ? sample_of(k + nbuf - 1) : 0;
      const int bpre = (int)((k + nbuf - 1) % nbuf);
      const bool pre_in_gemm = ROLE != MN_ROLE_IDLE && k < nr;
      if (pre && !pre_in_gemm) {
#pragma unroll
        for (int gi = 0; gi < kMnlGMax; ++gi)
          if (gi < gcnt) issue_group(npre, bpre, gi);
      }
      TR_MNL_MARK(2);
      if (ROLE != MN_ROLE_IDLE) {
        if (k >= 1) {
          const int zs = (int)((k - 1) & 1);
          const float4 zp = *reinterpret_cast<const float4*>(sZ + (zs * 16 + c) * 4);
          const float dz = softmax_ce(((zp.x + zp.y) + zp.z) + zp.w, yP, cwP, lane < 16);
          // Wv[4 rb + g] = sum_c dZ[c] w PhiC[c][4 rb + g] in DPP row g; lane rank 4 rb + (l & 3)
          const float wrow = row_sum16(dz * pcg);
          const float w0 = rdl(wrow, 0), w1 = rdl(wrow, 16), w2 = rdl(wrow, 32), w3 = rdl(wrow, 48);
          const float wvl = l3 == 0 ? w0 : l3 == 1 ? w1 : l3 == 2 ? w2 : w3;
          if (ROLE == MN_ROLE_A) {
            gacc[0] += wvl * accP[0];
            const float ug = grow == 0 ? uP0 : grow == 1 ? uP1 : grow == 2 ? uP2 : uP3;
            dpc = fmaf(dz, wg * ug, dpc);
          } else {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) gacc[qq] += wvl * accP[qq];
          }
        }
        if (k < nr) {
          yC = lab[sample_of(k)];
          cwC = rdl(cwl, (int)yC);
          float4 xr[16];
          load1((int)(k % nbuf), xr);
          gemm1(xr, (int)(k & 1), accC, uC0, uC1, uC2, uC3, pre, npre, bpre);
#pragma unroll
          for (int q = 0; q < 4; ++q) accP[q] = accC[q];
          uP0 = uC0;
          uP1 = uC1;
          uP2 = uC2;
          uP3 = uC3;
          yP = yC;
          cwP = cwC;
        }
      }
      TR_MNL_MARK(4);
    }
  } else {
    // ---- two samples (a pair) per barrier: ring slots 2 (p % nps) + h, member h in 16-lane
    // rows 2h, 2h+1 of the epilogue (both members' softmax chains in the same instructions) ----
    const int nps = nbuf / 2;
    const int np = (int)((nr + 1) / 2);  // (rows per workgroup < 2^31)
    // an odd range's last pair repeats the last sample with class weight 0 (contributes 0)
    auto member_sample = [&](int kk) -> int64_t { return sample_of(kk < nr ? kk : nr - 1); };
    auto issue_pair = [&](int p, int slot) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float* src = dma_src(member_sample(2 * p + h));
        float* dst = dma_dst(2 * slot + h);
#pragma unroll
        for (int gi = 0; gi < kMnlGMax; ++gi)
          if (gi < gcnt) issue_at(src, dst, gi);
      }
    };
    for (int p = 0; p < nps - 1 && p < np; ++p) issue_pair(p, p);
    int slot_cur = 0, slot_pre = nps - 1;  // ring slots of pair p and of pair p + nps - 1 (mod nps)
    mn_f32x4 accA[4], accB[4];  // members a, b of the previous pair (GEMM output of this pair)
#pragma unroll
    for (int q = 0; q < 4; ++q) accA[q] = accB[q] = mn_f32x4{0.f, 0.f, 0.f, 0.f};
    float ua0 = 0.f, ua1 = 0.f, ua2 = 0.f, ua3 = 0.f, ub0 = 0.f, ub1 = 0.f, ub2 = 0.f, ub3 = 0.f;
    int64_t ya = 0, yb = 0;
    float cwa = 0.f, cwb = 0.f;
    const int h = lane >> 5;  // epilogue member of this lane
    for (int p = 0; p <= np; ++p) {
      if (p < np) {
        int ahead = np - 1 - p;
        if (ahead > nps - 2) ahead = nps - 2;
        mn_wait_vm(2 * gcnt * ahead);  // pair p has landed (this wave's pieces)
      }
      TR_MNL_MARK(0);
      mn_barrier();  // every wave's pieces of pair p; Z partials of p - 1; slots of pair p - 1 free
      TR_MNL_MARK(1);
      const bool pre = p + nps - 1 < np;  // refill the slots of pair p - 1 with pair p + nps - 1
      const bool pre_in_gemm = ROLE != MN_ROLE_IDLE && p < np;
      if (pre && !pre_in_gemm) issue_pair(p + nps - 1, slot_pre);
      const int pq = p + nps - 1;
      const int spre = 2 * slot_pre;
      TR_MNL_MARK(2);
      float4 xra[16];  // member a's first MN_HOIST operand quads, in flight across the epilogue
      constexpr int HO = FULL ? MN_HOIST : 0;
      if (HO > 0 && ROLE != MN_ROLE_IDLE && p < np) load1(2 * slot_cur, xra, 0, HO);
      if (ROLE != MN_ROLE_IDLE) {
        if (p >= 1) {
          const int zs = (int)((p - 1) & 1);
          const float4 zp = *reinterpret_cast<const float4*>(sZ + ((zs * 2 + h) * 16 + c) * 4);
          const int64_t yh = h ? yb : ya;
          const float cwh = h ? cwb : cwa;
          const float dz = softmax_ce(((zp.x + zp.y) + zp.z) + zp.w, yh, cwh, (lane & 31) < 16);
          const float s0 = row_sum16(dz * pcp0), s1 = row_sum16(dz * pcp1);
          // member a: ranks q = 0, 1 in rows 0, 1 of pass 0; q = 2, 3 of pass 1; member b rows 2, 3
          const float wa = l3 == 0 ? rdl(s0, 0) : l3 == 1 ? rdl(s0, 16) : l3 == 2 ? rdl(s1, 0) : rdl(s1, 16);
          const float wb = l3 == 0 ? rdl(s0, 32) : l3 == 1 ? rdl(s0, 48) : l3 == 2 ? rdl(s1, 32) : rdl(s1, 48);
          if (ROLE == MN_ROLE_A) {
            gacc[0] += wa * accA[0];
            gacc[0] += wb * accB[0];
            float dza, dzb;  // both members' dZ[c] in every lane
            halves(dz, dza, dzb);
            const float uga = grow == 0 ? ua0 : grow == 1 ? ua1 : grow == 2 ? ua2 : ua3;
            const float ugb = grow == 0 ? ub0 : grow == 1 ? ub1 : grow == 2 ? ub2 : ub3;
            dpc = fmaf(dza, wg * uga, dpc);
            dpc = fmaf(dzb, wg * ugb, dpc);
          } else {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
              gacc[qq] += wa * accA[qq];
              gacc[qq] += wb * accB[qq];
            }
          }
        }
        TR_MNL_MARK(3);
        if (p < np) {
          const int s0 = 2 * slot_cur, zs = p & 1;
          ya = lab[member_sample(2 * p)];
          cwa = rdl(cwl, (int)ya);
          yb = lab[member_sample(2 * p + 1)];
          cwb = 2 * p + 1 < nr ? rdl(cwl, (int)yb) : 0.f;
          load1(s0, xra, HO, 16);
          gemm1(xra, zs * 2, accA, ua0, ua1, ua2, ua3, pre, pre ? member_sample(2 * pq) : 0, spre);
          TR_MNL_MARK(5);
          load1(s0 + 1, xra);
          gemm1(xra, zs * 2 + 1, accB, ub0, ub1, ub2, ub3, pre, pre ? member_sample(2 * pq + 1) : 0, spre + 1);
          TR_MNL_MARK(6);
        }
      }
      TR_MNL_MARK(4);
      slot_cur = slot_cur + 1 == nps ? 0 : slot_cur + 1;
      slot_pre = slot_pre + 1 == nps ? 0 : slot_pre + 1;
    }
  }
#if TR_MNL_PROFILE
  if (lane == 0 && blockIdx.x < 256)
    for (int q = 0; q < 8; ++q) g_mnl_prof[blockIdx.x][wv][q] = prof[q];
#endif

  // ---- fixed-order reduction of the units into an LDS image of the arena, then the slab ----
  if (ROLE == MN_ROLE_B) {  // fold the four row classes (lanes l, l^16, l^32, l^48)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float x = gacc[q][v];
        x += __shfl_xor(x, 16, TR_WAVE);
        x += __shfl_xor(x, 32, TR_WAVE);
        gacc[q][v] = x;
      }
  }
  float* sG = lds + g.oG;
  __syncthreads();
  for (int64_t e = t; e < g.slab; e += MN_T) sG[e] = 0.f;
  __syncthreads();
  for (int ws = 0; ws < MN_NW; ++ws) {
    if (ws == wv) {
      if (ROLE == MN_ROLE_A) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = 64 * ib + 4 * (lane >> 2) + v;
          if (row < I && rqv) sG[row * R + rq] += gacc[0][v];
        }
        const int r = 4 * rb + grow;
        if (cok && r < R) sG[g.offPC + c * R + r] += dpc;
      } else if (ROLE == MN_ROLE_B) {
        if (lane < 16 && rqv) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int j = 64 * jb + 16 * (lane >> 2) + 4 * v + q;
              if (j < J) sG[g.offP1 + j * R + rq] += gacc[q][v];
            }
        }
      }
    }
    __syncthreads();
  }
  if (ROLE == MN_ROLE_A && wv == 0) {
    lsum = tr_wave_allreduce_d(lsum);
    if (lane == 0) {
      a.dpart[2 * blockIdx.x] = lsum;
      a.dpart[2 * blockIdx.x + 1] = 0.0;
    }
  }
  float* slab = a.gpart + (int64_t)blockIdx.x * g.slab;
  for (int64_t e = t; e < g.slab; e += MN_T) slab[e] = sG[e];
}

template <bool FULL, int SPI>
__global__ __launch_bounds__(MN_T) void k_mnl_fused(MnlGeom g, MnArgs a, const int64_t* __restrict__ lab,
                                                    const float* __restrict__ class_w,
                                                    const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / TR_WAVE);  // wave-uniform
  if (wv < g.nA)
    mnl_body<MN_ROLE_A, FULL, SPI>(g, a, lab, class_w, lds, wv, lane);
  else if (wv < g.nunits)
    mnl_body<MN_ROLE_B, FULL, SPI>(g, a, lab, class_w, lds, wv, lane);
  else
    mnl_body<MN_ROLE_IDLE, FULL, SPI>(g, a, lab, class_w, lds, wv, lane);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static const void* mnl_kernel(const MnlGeom& g) {
  if (g.spi == 2)
    return g.full ? reinterpret_cast<const void*>(&k_mnl_fused<true, 2>) : reinterpret_cast<const void*>(&k_mnl_fused<false, 2>);
  return g.full ? reinterpret_cast<const void*>(&k_mnl_fused<true, 1>) : reinterpret_cast<const void*>(&k_mnl_fused<false, 1>);
}

bool mnl_geom_init(MnlGeom* g, int64_t I, int64_t J, int R, int C, std::string* why) {
  std::memset(g, 0, sizeof(*g));
  auto no = [&](const char* m) {
    if (why) *why = m;
    return false;
  };
  if (R < 1 || R > kMnlRMax) return no("rank outside [1, 32]");
  if (C < 1 || C > kMnlCMax) return no("classes outside [1, 16]");
  if (I < 1 || J < 4 || J % 4 != 0) return no("second feature dim must be a multiple of 4");
  if (I * J > (int64_t)1 << 28) return no("sample larger than 1 GiB");
  g->I = (int)I;
  g->J = (int)J;
  g->R = R;
  g->C = C;
  g->JQ = (int)(J / 4);
  const int lowbit = g->JQ & -g->JQ;
  g->smask = (lowbit < 16 ? lowbit : 16) - 1;
  g->nchunk = (int)(I * J / 4);
  g->nib = (int)((I + 63) / 64);
  g->njb = (int)((J + 63) / 64);
  g->nrb = (R + 3) / 4;
  g->Rp = 4 * g->nrb;
  g->nA = g->nib * g->njb * g->nrb;
  g->nunits = 2 * g->nA;
  g->fused_ok = 1;
  auto no_fused = [&](const char* m) {
    if (why && g->fused_ok) *why = m;
    g->fused_ok = 0;
  };
  // (samples above 64 KiB: only the split body's row-block form, tr_mnl_duo.hip, streams them)
  if (I * J * 4 > 64 * 1024) no_fused("sample larger than 64 KiB");
  if (g->nunits > MN_NW) no_fused("more than 8 GEMM units (I, J or R too large)");
  g->upw = 1;
  g->nsets = g->nib * g->njb;
  g->full = (I % 64 == 0 && J % 64 == 0) ? 1 : 0;
  g->offP1 = I * R;
  g->offPC = (I + J) * R;
  g->nfelem = (I + J + C) * R;
  g->slab = (g->nfelem + 3) & ~(int64_t)3;
  // ring depth: about 128 KiB of samples (nbuf - 1 in flight), 2..8
  const int64_t sb = I * J * 4;
  int nbuf = (int)((128 * 1024) / sb);
  if (nbuf > 8) nbuf = 8;
  if (nbuf < 2) nbuf = 2;
  const int64_t small = 4LL * 16 * 4 + 64;
  while (nbuf > 2 && nbuf * I * J + small > 160 * 1024 / 4) --nbuf;
  // two samples per barrier when the ring holds at least two pairs (TR_MNL_SPI=1 forces one)
  const char* spi_env = std::getenv("TR_MNL_SPI");
  g->spi = (nbuf >= 4 && !(spi_env != nullptr && std::atoi(spi_env) == 1)) ? 2 : 1;
  if (g->spi == 2) nbuf &= ~1;
  g->nbuf = nbuf;
  int64_t o = (int64_t)nbuf * I * J;
  g->oZ = (int)o;
  o += 4LL * 16 * 4;
  if (g->slab <= (int64_t)nbuf * I * J) {
    g->oG = 0;  // the arena image aliases the (drained) ring at the end
  } else {
    g->oG = (int)o;
    o += g->slab;
  }
  o = (o + 3) & ~(int64_t)3;
  if (o * 4 > 160 * 1024) no_fused("LDS budget exceeded");
  g->lds_floats = g->fused_ok ? (int)o : 0;
  return true;
}

hipError_t mnl_prepare(const MnlGeom& g, int* ok) {
  *ok = 0;
  if (!g.fused_ok) return hipSuccess;
  const void* k = mnl_kernel(g);
  const size_t lds = (size_t)g.lds_floats * 4;
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipFuncAttributes attr;
  e = hipFuncGetAttributes(&attr, k);
  if (e != hipSuccess) return e;
  if (attr.localSizeBytes > 0) return hipSuccess;  // spills: outside the envelope
  int nb = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, MN_T, lds);
  if (e != hipSuccess) return e;
  *ok = nb >= 1 ? 1 : 0;
  return hipSuccess;
}

hipError_t launch_mnl_fused(const MnlGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                            const float* w, const int64_t* lab, const float* class_w, float scale, float* gpart,
                            double* dpart, int64_t rows_per_wg, int reverse, const int32_t* stop, hipStream_t st) {
  if (grid < 1 || rows_per_wg < 0 || xld % 4 != 0 || (int64_t)grid * rows_per_wg < N) return hipErrorInvalidValue;
  const size_t lds = (size_t)g.lds_floats * 4;
MnArgs a{X, N, xld, phi, w, lab, class_w, scale, gpart, dpart, rows_per_wg, reverse};
#define TR_MNL_LAUNCH(F, S) hipLaunchKernelGGL((k_mnl_fused<F, S>), dim3(grid), dim3(MN_T), lds, st, g, a, lab, class_w, stop)
  if (g.spi == 2) {
    if (g.full)
      TR_MNL_LAUNCH(true, 2);
    else
      TR_MNL_LAUNCH(false, 2);
  } else {
    if (g.full)
      TR_MNL_LAUNCH(true, 1);
    else
      TR_MNL_LAUNCH(false, 1);
  }
#undef TR_MNL_LAUNCH
  return hipGetLastError();
}

}  // namespace tr

#if TR_MNL_PROFILE
extern "C" int tr_mnl_profile_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mnl_prof), sizeof(g_mnl_prof));
}
#endif

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_mnl() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_mnl_fused<true, 2>));
}
}  // namespace tr
