// tr_mnl_duo.hip — the factored multinomial single pass as TWO workgroups per CU (BASELINE
// config 3: X (65536, 128, 64), 10 classes, rank 8; multinomial_tensor_regression.py model
// :148-187, CrossEntropyLoss of fit_Adam :448-457, autograd :457).
//
// Same math and unit decomposition as k_mnl_fused (tr_mnl.hip header): per sample
//     T[i, r] = sum_j X_n[i, j] Phi1[j, r]   (A-units)     V[j, r] = sum_i X_n[i, j] Phi0[i, r]  (B-units)
//     U -> Z -> softmax, CE on the probabilities, dZ -> Wv -> dPhi0 += Wv T, dPhi1 += Wv V, dPhiC
// on v_mfma_f32_4x4x1_16b_f32.  k_mnl_fused runs ONE 8-wave workgroup per CU over a 4-sample LDS
// ring: every wave waits at one barrier per pair, and between barriers each wave does its GEMM
// unit and the softmax epilogue back to back, so the matrix pipe is busy ~22 % and the
// kernel is latency-bound.  Here a workgroup is 4 waves (2 A-waves, 2 B-waves, each
// wave owning BOTH rank blocks of its (i, j) block: one set of X operand reads feeds two units)
// over a 2-sample ring (2 x 32 KiB), and TWO workgroups share a CU: while one workgroup sits in
// its barrier or its latency-bound epilogue, the other's MFMAs run on the same SIMDs.
//
// What bounds it (round 5): the sample stream.  The timing ablations of round 4 kept the LDS-DMA
// instructions (the "no DMA" build refilled the same, L2-resident sample) and so pointed at the
// instruction stream; with the DMA removed entirely the bf16-split body below runs in 0.256 ms at
// config 3 against 0.368 ms with it.  The non-temporal policy on the sample pieces (as
// k_mnl_fused and k_linear_fused use) takes 6-7 % off both bodies (rank-block 0.364 -> 0.339 ms);
// a second sample in flight per workgroup does not help at config 3 (two 4-wave
// workgroups per CU already hold 128 KiB in flight).  The split body's one-workgroup-per-CU
// shapes at 5 and 6 waves (80 / 96 KiB with two slots) do take a ring of three (+3-4 points).
//
// Envelope (mnl_duo_geom): the rank-block body at (128, 64) / (64, 128) rank 5..8; the bf16-split
// body at those shapes rank <= 4 and at every (32 NW, 64) sample (NW = 2..8) and (16 NW, 128)
// sample (NW = 4, 6, 8) rank <= 8, any other I <= 256 / <= 128 and J % 4 == 0 in 28..128
// padded to the next of those shapes when it fills a third of it; taller samples whose rows are 2 or 3
// such blocks (NW = 8 or 6) streamed through the ring one row block per slot; ranks 9..16 in a 16-rank
// form of the split body (RK = 16); <= 16 classes.  Other two-mode
// shapes run k_mnl_fused (tr_mnl.hip) where it fits and the sample is >= 24 KiB, else the two-pass
// kernels (DESIGN.md "Multinomial, round 5").
//
// Per sample k of a workgroup: wait own LDS-DMA of k -> barrier -> epilogue of k-1 (Z partials
// of the 2 A-waves, double softmax, Wv, gradient scaling) -> GEMM of k with the DMA of k+1 into
// the other ring slot interleaved.  The A-waves read Phi1 (their B operand) from a transposed
// LDS table instead of 128 resident registers.  Numerics: the GEMM units, the Z partial slots and
// the slab accumulation order are those of k_mnl_fused, but the epilogue is NOT bitwise equal to
// it: exp / log run on the hardware base-2 units (v_exp_f32 / v_log_f32 with a premultiplied
// log2 e, ~1 ulp), the second softmax skips its max shift (S in [0, 1]), and Wv / <dS, S> are
// re-associated into closed forms over independent class sums (below); the file is also built
// with -fno-honor-nans.  It is pinned to the reference separately from k_mnl_fused, at the same
// 1e-5 bars (test_multinomial_golden kinds auto / noduo, including the mnl_duo_* fixtures at
// its own shapes).
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

#include "tr_common.h"
#include "tr_mnl.h"

#ifndef TR_DUO_PROFILE
#define TR_DUO_PROFILE 0  // profiling build only: per-phase cycle counts of every wave (tools/duo_profile.py)
#endif
#if TR_DUO_PROFILE
__device__ unsigned long long g_duo_prof[512][8][4];  // [workgroup][wave][phase]
#define TR_DUO_MARK(ph)                                           \
  do {                                                            \
    const unsigned long long _now = __builtin_readcyclecounter(); \
    prof[ph] += _now - prof_t;                                    \
    prof_t = _now;                                                \
  } while (0)
#else
#define TR_DUO_MARK(ph) \
  do {                  \
  } while (0)
#endif
#ifndef TR_DUO_SKIP
#define TR_DUO_SKIP 0  // profiling ablation only (results invalid): 1 loop LDS-DMA, 2 MFMAs, 4 epilogue;
                       // bsp form: 8 no LDS-DMA at all after the first sample, 16 no label loads
#endif

namespace tr {

namespace {
constexpr int DU_NW = 4;
constexpr int DU_T = DU_NW * TR_WAVE;
// Kept from the round-2..5 experiments (each measured on one box against the build without it;
// DESIGN.md "Two-workgroups-per-CU multinomial kernel" and "Multinomial, round 5"; the variants that
// were not kept — early issue of sample k + 2, an L2 prefetch, interleaved sample order, two
// samples in flight per workgroup — are in the git history):
//  - rank-block body: operand quads read XL (V unit) / XLA (T unit) GEMM steps ahead of their MFMAs,
//    and at (128, 64) the T unit's Phi1 quads held in 64 VGPRs for the launch (a third fewer
//    operand bytes; read-ahead 3 / 3 to fit 256 registers; the (64, 128) shape would spill);
//  - one LDS-DMA piece of the next sample per GEMM step (bursts stall the memory issue queue);
//  - a scheduling fence after every GEMM step: the operand reads stay ahead of their MFMAs (left
//    alone, the scheduler issues the T unit's reads one step ahead and waits on them) and the
//    epilogue stages stay between the steps;
//  - the non-temporal policy on the sample pieces (rank-block 0.364 -> 0.339 ms at c3).
constexpr int XL = 6, XLA = 4;
typedef float du_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ du_f32x4 du_mfma(float a, float b, du_f32x4 c) {
  if (TR_DUO_SKIP & 2) return c + a * b;  // one VALU op instead of the MFMA (keeps the operand reads)
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}
template <int CTRL>
__device__ __forceinline__ float du_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float du_row_sum16(float v) {
  v += du_dpp<0xB1>(v);
  v += du_dpp<0x4E>(v);
  v += du_dpp<0x141>(v);
  v += du_dpp<0x140>(v);
  return v;
}
__device__ __forceinline__ float du_row_max16(float v) {
  v = fmaxf(v, du_dpp<0xB1>(v));
  v = fmaxf(v, du_dpp<0x4E>(v));
  v = fmaxf(v, du_dpp<0x141>(v));
  v = fmaxf(v, du_dpp<0x140>(v));
  return v;
}
__device__ __forceinline__ float du_xor16_sum(float v) {
  const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ float du_xor32_sum(float v) {
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
// exp / log on the hardware base-2 units (v_exp_f32 / v_log_f32, ~1 ulp): the epilogue's
// arguments are bounded (exp of values <= 0 and of S in [0, 1], log of a sum in [1, 16 e])
__device__ __forceinline__ float du_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float du_log(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }
__device__ __forceinline__ float du_rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ void du_barrier() {  // leaves LDS-DMA in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void du_dma16(const float* gsrc, const float* lds_dst) {
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(a))
               : "memory");
}
// ---- bf16 split helpers (the bsp form below; same pieces as tr_spectral_slice.hip) ----
typedef __bf16 bs_bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bs_bf2 __attribute__((ext_vector_type(2)));
typedef uint32_t sl_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ du_f32x4 bs_mfma(sl_u4 a, const uint32_t (&b)[4], du_f32x4 c) {
  if (TR_DUO_SKIP & 2) return c + __uint_as_float(a[0]) * __uint_as_float(b[0]);
  const sl_u4 bb = sl_u4{b[0], b[1], b[2], b[3]};
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bs_bf8, a), __builtin_bit_cast(bs_bf8, bb), c, 0,
                                                 0, 0);
}
// two values -> one VGPR of packed round-to-nearest-even bf16 (element 0 = a), v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t sl_pack_rne(float a, float b) {
  return __builtin_bit_cast(uint32_t, bs_bf2{(__bf16)a, (__bf16)b});
}
typedef _Float16 bs_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 bs_h2 __attribute__((ext_vector_type(2)));
// two values -> one VGPR of packed round-to-nearest-even f16, v_cvt_pk_f16_f32
__device__ __forceinline__ uint32_t bs_pack_h(float a, float b) {
  return __builtin_bit_cast(uint32_t, bs_h2{(_Float16)a, (_Float16)b});
}
__device__ __forceinline__ du_f32x4 bs_mfma_h(sl_u4 a, const uint32_t (&b)[4], du_f32x4 c) {
  if (TR_DUO_SKIP & 2) return c + __uint_as_float(a[0]) * __uint_as_float(b[0]);
  const sl_u4 bb = sl_u4{b[0], b[1], b[2], b[3]};
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(bs_h8, a), __builtin_bit_cast(bs_h8, bb), c, 0, 0,
                                                0);
}
__device__ __forceinline__ float sl_lo_f32(uint32_t h) { return __uint_as_float(__builtin_amdgcn_perm(h, h, 0x01000c0cu)); }
__device__ __forceinline__ float sl_hi_f32(uint32_t h) { return __uint_as_float(h & 0xffff0000u); }
// a (element 2m), b (element 2m + 1) -> three packed round-to-nearest pieces: x = x1 + x2 + x3 exactly
__device__ __forceinline__ void sl_split2(float a, float b, uint32_t& h1, uint32_t& h2, uint32_t& h3) {
  h1 = sl_pack_rne(a, b);
  const float ra = a - sl_lo_f32(h1), rb = b - sl_hi_f32(h1);
  h2 = sl_pack_rne(ra, rb);
  h3 = sl_pack_rne(ra - sl_lo_f32(h2), rb - sl_hi_f32(h2));
}
}  // namespace

struct DuArgs {
  const float* X;
  int64_t N, xld;
  const float* phi;
  const float* w;
  float scale;
  float* gpart;
  double* dpart;
  int64_t rows_per_wg;
  int reverse;
};

// One LDS-DMA piece per lane with a scalar base: 16 B from sbase + voff (bytes, per lane) to LDS
// byte address m0v + 16 * lane.  No per-piece 64-bit address arithmetic; m0 is compiler-reserved
// and is saved / restored inside the statement.
__device__ __forceinline__ void du_dma_s(uint32_t voff, const float* sbase, uint32_t m0v) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(m0v)
               : "memory");
}

// Wave wv = (block s = wv & 1, rank block rb = wv >> 1): the T unit AND the V unit of its X
// sub-block (64 x 64) and rank block, so all four waves carry the same instruction mix (an
// A/B role split left the T waves on the critical path and the V waves idle at the barrier).
// Shape fixed at compile time: J = JT (64 or 128), I = 8192 / JT (a 32 KiB sample, two 64-row
// blocks), R in 5..8 (two rank blocks), every LDS-DMA group valid, chunk swizzle q ^ (i & 15).
template <int JT>
__device__ __forceinline__ void duo_body(const MnlGeom& g, const DuArgs& a, const int64_t* __restrict__ lab,
                                         const float* __restrict__ class_w, float* lds, const int wv, const int lane) {
  const int t = threadIdx.x;
  constexpr int J = JT, I = 8192 / JT, SPF = 8192, JQ = J / 4;
  constexpr int NJB = J / 64, NIB = I / 64;
  const int R = g.R, C = g.C;
  float* sZ = lds + g.du_oZ;    // [2 parity][16 classes][4 T-unit slots]
  float* sP1 = lds + g.du_oP1;  // Phi1^T [8][J + 4] (T units' B operand, 4 consecutive k per b128)
  constexpr int P1S = J + 4;
  const float* P0 = a.phi;
  const float* P1 = a.phi + g.offP1;
  const float* PC = a.phi + g.offPC;
  const int c = lane & 15, grow = lane >> 4, l3 = lane & 3;
  const bool cok = c < C;
  const float cwl = cok ? class_w[c] : 0.f;  // class weight of class c in lane c of every row
  const float NEG = -__builtin_huge_valf();
  float sel[4], gsel[4];  // 1 where l & 3 == q / where the DPP row (l >> 4) == q
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    sel[q] = l3 == q ? 1.f : 0.f;
    gsel[q] = grow == q ? 1.f : 0.f;
  }

  const int s = wv & 1, rb = wv >> 1;
  const int ib = NIB == 2 ? s : 0, jb = NJB == 2 ? s : 0;
  const int rq = 4 * rb + l3;  // rank of this lane's accumulator column
  const bool rqv = rq < R;
  // T unit: U partial weights phiU[v] = Phi0[64 ib + 4 (l >> 2) + v][rq], Z partial weights
  // wpc[v] = w_r PhiC[c][r] (r = 4 rb + v); epilogue weights pcg = w_r PhiC[c][r] (r = 4 rb + row)
  // V unit: B operand bopB[st] = Phi0[64 ib + 4 st + row][rq]
  float phiU[4], wpc[4], bopB[16];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    phiU[v] = rqv ? P0[(int64_t)(64 * ib + 4 * (lane >> 2) + v) * R + rq] : 0.f;
    const int r = 4 * rb + v;
    wpc[v] = (cok && r < R) ? a.w[r] * PC[c * R + r] : 0.f;
  }
  const int rg = 4 * rb + grow;
  const float pcg = (cok && rg < R) ? a.w[rg] * PC[c * R + rg] : 0.f;
  const float wg = rg < R ? a.w[rg] : 0.f;
#pragma unroll
  for (int st = 0; st < 16; ++st) bopB[st] = rqv ? P0[(int64_t)(64 * ib + 4 * st + grow) * R + rq] : 0.f;
  // Phi1^T table, rank rows padded to 8 with zeros (a padded rank's T column must stay finite:
  // U sums every lane's column times phiU, which is 0 there)
  for (int e = t; e < 8 * J; e += DU_T) {
    const int r = e / J, j = e - r * J;
    sP1[r * P1S + j] = r < R ? P1[(int64_t)j * R + r] : 0.f;
  }
  for (int e = t; e < 2 * 16 * 4; e += DU_T) sZ[e] = 0.f;

  // LDS-DMA map: wave wv issues the 1 KiB groups wv + 4 gi (gi < 8) of every sample; LDS bytes
  // of group G at ring slot b: 32 KiB b + 1 KiB G
  uint32_t goff[8];
#pragma unroll
  for (int gi = 0; gi < 8; ++gi) {
    const int slot = (wv + DU_NW * gi) * TR_WAVE + lane;
    const int i = slot / JQ;
    const int q = slot - i * JQ;
    goff[gi] = 4u * (uint32_t)(i * J + 4 * (q ^ (i & 15)));
  }
  const uint32_t lbase = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)lds));
  // LDS read offsets (floats): T quad c4 of this lane's row at aoff[c4]; V quad of step st at
  // boff[st & 3] + 4 J st; Phi1 quad of step st at pb + 4 st
  constexpr bool P1R = JT == 64;  // (the (64, 128) shape spills one register with it)
  int aoff[P1R ? 1 : 16], boff[4];
  const int abase = (64 * ib + lane) * J + 64 * jb, c4s = 4 * c;  // (P1R: aoff of step st = abase + (c4s ^ 4 st))
  if constexpr (!P1R) {
#pragma unroll
    for (int c4 = 0; c4 < 16; ++c4) aoff[c4] = (64 * ib + lane) * J + 64 * jb + 4 * (c4 ^ c);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) boff[m] = (64 * ib + grow) * J + 64 * jb + 4 * (c ^ (4 * m + grow));
  const int pb = rq * P1S + 64 * jb;
  const int64_t n0 = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t n1 = n0 + a.rows_per_wg < a.N ? n0 + a.rows_per_wg : a.N;
  const int nr = (int)(n1 > n0 ? n1 - n0 : 0);
  auto sample_of = [&](int k) -> int64_t { return n0 + (a.reverse ? (nr - 1 - k) : k); };
  auto src_of = [&](int k) -> const float* { return a.X + sample_of(k) * a.xld; };

  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);  // retire the prologue's loads (the loop waits are counted)
  float4 p1r[P1R ? 16 : 1];  // (P1R) the T unit's B operand quads of every step, for the launch
  if constexpr (P1R) {
#pragma unroll
    for (int st = 0; st < 16; ++st) p1r[st] = *reinterpret_cast<const float4*>(sP1 + pb + 4 * st);
    __builtin_amdgcn_s_waitcnt(0);
  }

  du_f32x4 gT = du_f32x4{0.f, 0.f, 0.f, 0.f};  // dPhi0 rows x ranks of the T unit
  du_f32x4 gV[4];                                // dPhi1 of the V unit, by row class
#pragma unroll
  for (int q = 0; q < 4; ++q) gV[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
  float dpc = 0.f;  // dPhiC[c][4 rb + row] of the T unit
  double lsum = 0.0;

  du_f32x4 TP = du_f32x4{0.f, 0.f, 0.f, 0.f};  // previous sample's T (summed) and V (by row class)
  du_f32x4 VP[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) VP[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
  float uP[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t yP = 0;  // label / class weight of the sample in the epilogue
  float cwP = 0.f;

  // ---- epilogue of one sample, in 8 stages (the chain of dependent steps is cut so that the
  // stages can sit between the next sample's GEMM steps: its latency hides under MFMAs) ----
  // S = softmax(Z) (multinomial…py:187), Q = softmax(S), CE = log sum exp(S) - S_y (S lies in
  // [0, 1]: the second softmax needs no max shift), dS = (Q - e_y) cw_y / W, dZ = S (dS - <dS, S>),
  // Wv[r] = sum_c dZ[c] w_r PhiC[c, r].  Every sum over the 16 classes that the chain needs after
  // S is formed at once (independent DPP row sums, so their latencies overlap):
  //   s2 = sum q, d1 = sum S q, e1 = S_y, a_r = sum S q p_r, b_r = sum S p_r, y_r = S_y p_{y,r}
  // with q = exp(S), p_r = w_r PhiC[., r] (r = 4 rb + row: this wave's rank block); then
  // <dS, S> = k (d1 / s2 - e1) and Wv[r] = k (a_r / s2 - y_r) - <dS, S> b_r  (k = cw_y / W).
  float4 e_zp = make_float4(0.f, 0.f, 0.f, 0.f);
  float e_x = 0.f, e_ez = 0.f, e_sum = 0.f, e_S = 0.f, e_q = 0.f, e_Sq = 0.f, e_Sy = 0.f;
  float e_s2 = 0.f, e_d1 = 0.f, e_e1 = 0.f, e_dz = 0.f, e_ar = 0.f, e_br = 0.f, e_yr = 0.f, e_wr = 0.f, e_wv = 0.f;
  bool e_isy = false;
  // epilogue stage st of the sample with Z partials in parity slot zs, label yE, class weight cwE
  // (for the first call of a workgroup: zero partials, zero accumulators, cwE = 0 -> adds 0)
  auto epi = [&](int st, int zs, int64_t yE, float cwE) {
    if (TR_DUO_SKIP & 4) return;
    if (st == 0) {
      e_zp = *reinterpret_cast<const float4*>(sZ + (zs * 16 + c) * 4);
    } else if (st == 1) {
      const float zz = cok ? ((e_zp.x + e_zp.y) + e_zp.z) + e_zp.w : NEG;
      e_x = zz - du_row_max16(zz);
    } else if (st == 2) {
      e_ez = cok ? du_exp(e_x) : 0.f;
      e_sum = du_row_sum16(e_ez);
    } else if (st == 3) {
      e_S = e_ez * __builtin_amdgcn_rcpf(e_sum);
      e_q = cok ? du_exp(e_S) : 0.f;
      e_isy = cok && (int64_t)c == yE;
      e_Sq = e_S * e_q;
      e_Sy = e_isy ? e_S : 0.f;
    } else if (st == 4) {
      e_s2 = du_row_sum16(e_q);
      e_d1 = du_row_sum16(e_Sq);
      e_e1 = du_row_sum16(e_Sy);
      e_ar = du_row_sum16(e_Sq * pcg);
      e_br = du_row_sum16(e_S * pcg);
      e_yr = du_row_sum16(e_Sy * pcg);
    } else if (st == 5) {
      const float is2 = __builtin_amdgcn_rcpf(e_s2);
      const float kk = cwE * a.scale;
      const float dot = kk * (e_d1 * is2 - e_e1);
      lsum += (wv == 0 && lane == 0) ? (double)cwE * (double)(du_log(e_s2) - e_e1) : 0.0;
      const float dS = cok ? kk * (e_q * is2 - (e_isy ? 1.0f : 0.0f)) : 0.f;
      e_dz = cok ? e_S * (dS - dot) : 0.f;
      e_wr = kk * (e_ar * is2 - e_yr) - dot * e_br;
    } else if (st == 6) {
      // Wv[4 rb + g] in DPP row g -> lane rank 4 rb + (l & 3) by 0/1 lane masks (no branches)
      const float w0 = du_rdl(e_wr, 0), w1 = du_rdl(e_wr, 16), w2 = du_rdl(e_wr, 32), w3 = du_rdl(e_wr, 48);
      e_wv = fmaf(w3, sel[3], fmaf(w2, sel[2], fmaf(w1, sel[1], w0 * sel[0])));
    } else {
      gT += e_wv * TP;
      const float ug = fmaf(uP[3], gsel[3], fmaf(uP[2], gsel[2], fmaf(uP[1], gsel[1], uP[0] * gsel[0])));
      dpc = fmaf(e_dz, wg * ug, dpc);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) gV[qq] += e_wv * VP[qq];
    }
  };

#if TR_DUO_PROFILE
  unsigned long long prof[4] = {0, 0, 0, 0};
  unsigned long long prof_t = __builtin_readcyclecounter();
#endif
  auto dma_sample = [&](const float* src, int slot) {
#pragma unroll
    for (int gi = 0; gi < 8; ++gi)
      du_dma_s(goff[gi], src, lbase + (uint32_t)(slot * 4 * SPF) + (uint32_t)(wv + DU_NW * gi) * 1024u);
  };
  if (nr > 0) dma_sample(src_of(0), 0);
  int64_t yN = nr > 0 ? lab[sample_of(0)] : 0;  // label of the next GEMM sample (scalar, one ahead)

  // iteration k (ring slot SL = k & 1, a compile-time constant: the loop is unrolled by two so
  // every LDS read is a base register + immediate): barrier -> GEMM of sample k with the
  // epilogue of k - 1 between its steps and the LDS-DMA of k + 1 into the other slot (of sample k
  // itself when k is the last one: a harmless refill of a free slot, no guard per piece)
  auto iter = [&](auto slot_c, int k) {
    constexpr int SL = decltype(slot_c)::value;
    // the label of the next GEMM sample is a scalar load issued BEFORE the waits below: an SMEM
    // load in flight (it may return out of order) would make every counted lgkmcnt wait of the
    // GEMM's LDS reads a full lgkmcnt(0) drain; here the barrier's lgkmcnt(0) retires it while
    // the wave waits for its LDS-DMA anyway
    const int64_t yC = yN;
    const bool more = k + 1 < nr;
    yN = lab[sample_of(more ? k + 1 : k)];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    TR_DUO_MARK(0);
    du_barrier();  // everyone's pieces of k; Z partials of k - 1; slot SL ^ 1 free
    TR_DUO_MARK(1);
    const float cwC = du_rdl(cwl, (int)yC);
    const float* psrc = (more && !(TR_DUO_SKIP & 1)) ? src_of(k + 1) : src_of(k);
    const uint32_t pm0 = lbase + (uint32_t)((SL ^ 1) * 4 * SPF) + (uint32_t)wv * 1024u;
    epi(0, SL ^ 1, yP, cwP);
    const float* sb = lds + SL * SPF;
    du_f32x4 aT[4], aV[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) aT[q] = aV[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
    // operand quads read ahead of their MFMAs (bounded live registers)
    float4 xt[16], bq[16], xv[16];
    auto ldT = [&](int st) {
      if constexpr (P1R) {
        xt[st] = *reinterpret_cast<const float4*>(sb + abase + (c4s ^ (4 * st)));
        bq[st] = p1r[st];
      } else {
        xt[st] = *reinterpret_cast<const float4*>(sb + aoff[st]);
        bq[st] = *reinterpret_cast<const float4*>(sP1 + pb + 4 * st);
      }
    };
    auto ldV = [&](int st) { xv[st] = *reinterpret_cast<const float4*>(sb + boff[st & 3] + 4 * J * st); };
    constexpr int XLT = P1R ? 3 : XLA, XLV = P1R ? 3 : XL;  // read-ahead depths of this form
#pragma unroll
    for (int st = 0; st < XLT; ++st) ldT(st);
#pragma unroll
    for (int st = 0; st < XLV; ++st) ldV(st);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      if (st + XLT < 16) ldT(st + XLT);
      if (st + XLV < 16) ldV(st + XLV);
      if (st < 8) du_dma_s(goff[st], psrc, pm0 + (uint32_t)st * 4096u);
      aT[0] = du_mfma(xt[st].x, bq[st].x, aT[0]);
      aT[1] = du_mfma(xt[st].y, bq[st].y, aT[1]);
      aT[2] = du_mfma(xt[st].z, bq[st].z, aT[2]);
      aT[3] = du_mfma(xt[st].w, bq[st].w, aT[3]);
      aV[0] = du_mfma(xv[st].x, bopB[st], aV[0]);
      aV[1] = du_mfma(xv[st].y, bopB[st], aV[1]);
      aV[2] = du_mfma(xv[st].z, bopB[st], aV[2]);
      aV[3] = du_mfma(xv[st].w, bopB[st], aV[3]);
      if ((st & 1) == 1 && st < 15) epi(1 + (st >> 1), SL ^ 1, yP, cwP);
      __builtin_amdgcn_sched_barrier(0);
    }
    TR_DUO_MARK(2);
    // T of sample k -> U partial of this unit -> Z partial (16 classes) -> LDS
    const du_f32x4 T = (aT[0] + aT[1]) + (aT[2] + aT[3]);
    TP = T;
#pragma unroll
    for (int q = 0; q < 4; ++q) VP[q] = aV[q];
    float u = phiU[0] * T.x;
    u = fmaf(phiU[1], T.y, u);
    u = fmaf(phiU[2], T.z, u);
    u = fmaf(phiU[3], T.w, u);
    u += du_dpp<0x124>(u);  // row_ror:4
    u += du_dpp<0x128>(u);  // row_ror:8
    u = du_xor16_sum(u);
    u = du_xor32_sum(u);
    uP[0] = du_rdl(u, 0);
    uP[1] = du_rdl(u, 1);
    uP[2] = du_rdl(u, 2);
    uP[3] = du_rdl(u, 3);
    float zpart = wpc[0] * uP[0];
    zpart = fmaf(wpc[1], uP[1], zpart);
    zpart = fmaf(wpc[2], uP[2], zpart);
    zpart = fmaf(wpc[3], uP[3], zpart);
    // every row holds the same 16 class partials: all four rows store (same value, same slot)
    sZ[(SL * 16 + c) * 4 + rb + 2 * s] = zpart;
    yP = yC;
    cwP = cwC;
    TR_DUO_MARK(3);
  };
  for (int k = 0; k < nr; k += 2) {
    iter(std::integral_constant<int, 0>(), k);
    if (k + 1 < nr) iter(std::integral_constant<int, 1>(), k + 1);
  }
#if TR_DUO_PROFILE
  if (lane == 0 && blockIdx.x < 512)
    for (int q = 0; q < 4; ++q) g_duo_prof[blockIdx.x][wv][q] = prof[q];
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (harmless) refill has landed
  du_barrier();  // Z partials of the last sample
  if (nr > 0) {
#pragma unroll
    for (int st = 0; st < 8; ++st) epi(st, (nr - 1) & 1, yP, cwP);
  }

  // ---- fixed-order reduction into an LDS image of the arena (wave order), slab ----
#pragma unroll
  for (int q = 0; q < 4; ++q)  // fold the V unit's four row classes (lanes l, l^16, l^32, l^48)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float x = gV[q][v];
      x += __shfl_xor(x, 16, TR_WAVE);
      x += __shfl_xor(x, 32, TR_WAVE);
      gV[q][v] = x;
    }
  float* sG = lds + g.du_oG;
  __syncthreads();
  for (int64_t e = t; e < g.slab; e += DU_T) sG[e] = 0.f;
  __syncthreads();
  for (int ws = 0; ws < DU_NW; ++ws) {
    if (ws == wv) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = 64 * ib + 4 * (lane >> 2) + v;
        if (rqv) sG[row * R + rq] += gT[v];
      }
      if (cok && rg < R) sG[g.offPC + c * R + rg] += dpc;
      if (lane < 16 && rqv) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int j = 64 * jb + 16 * (lane >> 2) + 4 * v + q;
            sG[g.offP1 + j * R + rq] += gV[q][v];
          }
      }
    }
    __syncthreads();
  }
  if (wv == 0) {
    lsum = tr_wave_allreduce_d(lsum);
    if (lane == 0) {
      a.dpart[2 * blockIdx.x] = lsum;
      a.dpart[2 * blockIdx.x + 1] = 0.0;
    }
  }
  float* slab = a.gpart + (int64_t)blockIdx.x * g.slab;
  for (int64_t e = t; e < g.slab; e += DU_T) slab[e] = sG[e];
}

// ------------------------------------------------------------------------------------------
// bf16-split form (g.bsp, the default where it fits): the same per-sample math on the 16x16x32
// MFMAs with the fp32 operands split into round-to-nearest pieces, as the spectral slice kernel
// does (tr_spectral_slice.hip "bf16 split"); the factors in three bf16 pieces and the rank columns
// packed, B12 = [b1 | b2] (columns 0-7 | 8-15, rank = column & 7), B3 = [b3 | 0], so that one
// 16-wide MFMA carries two piece products (columns r and r + 8 are folded at the end).  X in one
// of two forms, a template parameter the plan sets from X's range (tr_plan_set_x_range):
//  - fast (EXACT = false): x1 = bf16(x) and ONE f16 piece x2 = f16(x - x1), against
//    H = [f16(phi) | f16(phi - f16(phi))]; three MFMAs per tile and k step:
//      acc += x2.H + x1.B3 + x1.B12   (= x1b1 + x1b2 + x1b3 + x2 phi)
//    x1 + x2 is within 2^-20 |x| + 2^-25 of x (the f16 residual of |x| < 2^-5 is subnormal, of
//    |x| >= 2^24 it overflows): normwise over X within 2^-20 + 2^-25 / rms(X), so the plan takes
//    it only while rms(X) >= 2^-5 and max |X| < 2^23;
//  - exact (EXACT = true, any other X: data in small units, large raw counts): x = x1 + x2 + x3
//    EXACTLY in bf16 pieces (x2 = bf16(x - x1), x3 = x - x1 - x2, at most 8 significant bits;
//    bf16 has fp32's exponent range), four MFMAs:
//      acc += x3.B12 + x2.B12 + x1.B3 + x1.B12   (dropped: x2b3, x3b3, < 2^-24 |xb|)
//    15-20 % slower on these shapes (11 instead of 6 VALU per pair of X values: issue-bound).
// Round 5 ran the fast form on any X: 2e-4 off at |X| ~ 1e-4, inf above 2^24
// (tests/test_gpu_parity.py::test_multinomial_split_body_x_scale runs both forms at 1e-4 .. 3e7).
// A 32 KiB sample takes 96 MFMAs per workgroup instead of 512 4x4x1 ones: the rank-block form
// spends 1,024 issue cycles per wave-sample on MFMAs alone.  J = 64 samples of 32 NW rows run NW
// waves (NW = 2..8), J = 128 ones of 16 NW rows NW waves (NW = 4, 6, 8); 8 / NW workgroups per
// CU.  Work of wave wv:
//   T[i, r] over i-tiles of 16 rows (J = 64: tiles 2 wv, 2 wv + 1; J = 128: tile wv) and every
//     32-deep j k-step: A = X rows (two ds_read_b128 of consecutive chunks per lane)
//   V[j, r] over 4 j-tiles for ONE 32-deep i k-step (J = 64: k-step wv; J = 128: k-step
//     wv % (NW / 2), chunk group wv / (NW / 2)): j-tile t holds j = 4 c + t for chunk c = lane row, so one ds_read_b128
//     of chunk c of row i gives element i of four tiles (eight reads: the k-step's 32 i)
// The chunk swizzle q ^ (i & 15) makes both reads conflict-free.  T is complete per wave (its
// U partial over its rows goes through LDS: NW partials per sample); V is a partial over the
// wave's i k-step, and dPhi1 = sum_n Wv_n V_n is linear in it: the waves' partials are summed
// once, at the end.  Every wave runs the softmax epilogue of the previous sample (staged between
// its GEMM steps) for all ranks; wave 0 alone accumulates dPhiC and the loss.
template <int... T, class F>
__device__ __forceinline__ void for_each_ic(std::integer_sequence<int, T...>, F&& f) {
  (f(std::integral_constant<int, T>()), ...);
}

template <int JT, int NW, int NS, bool PAD, bool EXACT, int NB, int RK>
__device__ __forceinline__ void bsp_body(const MnlGeom& g, const DuArgs& a, const int64_t* __restrict__ lab,
                                         const float* __restrict__ class_w, float* lds, const int wv, const int lane) {
  const int t = threadIdx.x;
  // J = 64: NW waves, each owning 32 rows of a (32 NW, 64) sample; J = 128: NW waves over a
  // (16 NW, 128) sample, each owning 16 T rows and one (32-row k-step, 16-chunk group) of V
  // (J = 32: NW waves over a (32 NW, 32) sample, each owning 32 T rows and one V k-step of 32
  // rows; see J32 below)
  constexpr bool J32 = JT == 32;
  constexpr int J = JT, I = JT == 128 ? 16 * NW : 32 * NW, SPF = I * J, JQ = J / 4, NT_ = NW * TR_WAVE;
  static_assert(JT != 128 || NW % 2 == 0, "J = 128: two chunk groups per V k-step");
  constexpr int NT = JT == 128 ? 1 : 2;  // T i-tiles per wave
  constexpr int NKS = I / 32;            // V k-steps (J = 128: NW / 2 of them, two chunk groups each)
  constexpr int NKT = J / 32;  // T k-steps (j)
  // J = 32: V's 32 columns are two j-tiles of 16 (tile t: lane n's column j = 4 (n & 7) + t +
  // 2 (n >> 3), lanes n and n + 8 read one chunk), one V k-step's 32 rows are ordered i = iv0 +
  // 4 e + gq (lane groups gq, gq + 1 on rows of both parities: conflict-free chunk reads), and the
  // 128-byte rows take the chunk swizzle q ^ ((i / 2 + 2) & 7) (T's 16-lane read groups cover the 16
  // (row parity, chunk slot) pairs)
  constexpr int NVS = J32 ? 2 : 4;  // V steps (j-tiles)
  constexpr int NG = SPF / (NW * 256);  // 1 KiB LDS-DMA pieces per wave per sample (8; J = 32: 4)
  static_assert(NG == NT * NKT + NVS, "one LDS-DMA piece per GEMM step");
  static_assert(!J32 || (NB == 1 && RK == 8), "J = 32: one block, 8 rank columns");
  auto swz = [](int i) { return J32 ? ((i >> 1) + 2) & 7 : i & 15; };
  // DIST (J = 32): the epilogue of sample s runs on wave s % NW alone (every wave ran every sample's:
  // at 4 KiB of sample per wave its VALU work was a quarter of the kernel, profiles/r06_mnl_j32), which
  // publishes Wv(s) in LDS; every wave applies it to its T(s), V(s) after the next barrier, one
  // iteration later than the owner's stages (T, V of two samples live across the loop's back edge)
  constexpr bool DIST = J32;
  static_assert(!DIST || NB == 1, "one-wave epilogue: one block");
  float* sWv = lds + g.bs_oW;  // [NS][8] Wv, then [NW] double loss partials
  double* sLs = reinterpret_cast<double*>(sWv + NS * 8);
  const int R = g.R, C = g.C;
  // PAD: the sample's g.I x g.J (g.J % 4 == 0) fills only part of the compiled I x J; the padding
  // rows and column chunks read the sample's first chunk (valid memory) and meet zero Phi0 / Phi1 rows
  // NB > 1 (BLK): a sample of NB * I rows streams through the ring as NB row blocks of I rows, each
  // one ring slot; T, its U partial and the dPhi0 rows are per block, V accumulates over the blocks,
  // and the epilogue runs once per sample (no row padding there: g.I = NB * I).  NB is compiled in:
  // with the block index a run-time value, the block-dependent choices (epilogue or not, V carried
  // or folded) cost ~300 VALU per block in selects and moves (profiled: 25 % slower per block)
  constexpr bool BLK = NB > 1;
  constexpr int nb = NB;
  static_assert(!BLK || NS == 2, "row blocks: a ring of two");
  // RK = 16 (ranks 9..16): the accumulator's 16 columns are 16 ranks of one piece (B operands b1,
  // b2, b3 and the f16 h in four registers each, one MFMA per piece: 4 per tile and k step in the
  // fast form, 6 in the exact one) instead of 8 ranks x two pieces folded (RK = 8: 3 / 4); the
  // epilogue's DPP row gq carries ranks gq + 4 k, k < RK / 4
  static_assert(RK == 8 || RK == 16, "8 or 16 rank columns");
  constexpr bool R16 = RK == 16;
  constexpr int KR = RK / 4;  // ranks per epilogue row
  static_assert(!(BLK && R16), "row blocks at rank <= 8");
  const int Ir = (PAD && !BLK) ? g.I : I, Jr = PAD ? g.J : J;
  // NS = 3: a ring of three samples (the DMA of sample k + 2 goes into the slot of k - 1 while k
  // is computed: two samples in flight), where three fit the workgroup's LDS share
  static_assert(NS == 2 || NS == 3, "ring of two or three slots");
  float* sU = lds + g.bs_oU;  // [NS slots][NW waves][RK ranks] U partials
  const float* P0 = a.phi;
  const float* P1 = a.phi + g.offP1;
  const float* PC = a.phi + g.offPC;
  // r8: the rank of this lane's accumulator column (RK = 8: columns r and r + 8 hold two pieces of
  // rank r, lanes n >= 8 duplicate it after the fold and weigh 0; RK = 16: rank n)
  const int n = lane & 15, gq = lane >> 4, r8 = R16 ? n : n & 7;
  const bool lo8 = R16 || n < 8, rok = r8 < R;
  const int c = n;  // epilogue: class lane c, DPP row gq (ranks gq + 4 k)
  const bool cok = c < C;
  const float cwl = cok ? class_w[c] : 0.f;
  const float NEG = -__builtin_huge_valf();

  const int it0 = NT == 2 ? 32 * wv : 16 * wv;                    // first T row of this wave
  const int iv0 = JT == 128 ? 32 * (wv % NKS) : 32 * wv;          // V k-step (rows) of this wave
  const int cv = J32 ? (n & 7) : n + (J == 128 ? 16 * (wv / NKS) : 0);  // V chunk (j = 4 cv + tile)
  auto vrow = [&](int e) { return J32 ? iv0 + 4 * e + gq : iv0 + 8 * gq + e; };  // V element e's row
  // B operands, split once per launch: T (Phi1, element e of lane group gq <-> j = 32 s + 8 gq + e)
  // (RK = 16: bT12 / bV12 hold b1, bT2 / bV2 b2, bT3 / bV3 b3, hT / hV f16(x))
  constexpr int N2 = R16 ? NKT : 1;
  uint32_t bT12[NKT][4], bT2[N2][4], bT3[NKT][4], hT[NKT][4], bV12[4], bV2[4], bV3[4], hV[4];
  auto bsplit = [&](float x0, float x1, uint32_t& b12, uint32_t& b2, uint32_t& b3, uint32_t& hh) {
    uint32_t h1, h2, h3;
    sl_split2(x0, x1, h1, h2, h3);
    if constexpr (R16) {
      b12 = h1;
      b2 = h2;
      b3 = h3;
      hh = EXACT ? 0u : bs_pack_h(x0, x1);
    } else {
      b12 = lo8 ? h1 : h2;
      b2 = 0u;
      b3 = lo8 ? h3 : 0u;
      if constexpr (!EXACT) {  // f16 pieces for the fast form's f16 X piece: [f16(x) | f16(x - f16(x))]
        const uint32_t f1 = bs_pack_h(x0, x1);
        const bs_h2 f1v = __builtin_bit_cast(bs_h2, f1);
        const uint32_t f2 = bs_pack_h(x0 - (float)f1v[0], x1 - (float)f1v[1]);
        hh = lo8 ? f1 : f2;
      } else {
        hh = 0u;
      }
    }
  };
#pragma unroll
  for (int s = 0; s < NKT; ++s)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int j = 32 * s + 8 * gq + 2 * v;
      bsplit((rok && (!PAD || j < Jr)) ? P1[(int64_t)j * R + r8] : 0.f,
             (rok && (!PAD || j + 1 < Jr)) ? P1[(int64_t)(j + 1) * R + r8] : 0.f, bT12[s][v], bT2[R16 ? s : 0][v],
             bT3[s][v], hT[s][v]);
    }
  // V (Phi0, element e <-> i = vrow(e)) and the U weights: T accumulator (lane (n, gq), reg
  // v) = T[it0 + 16 tt + 4 gq + v][n & 7] after the column fold; lanes n >= 8 hold the same values
  // and weigh 0.  Both depend on the row block: BLK loads the raw Phi0 values of the next block at
  // the end of a block (they land with that block's LDS-DMA wait) and splits them after its barrier
  float pvr[8], phiU[NT][4];
  // BLK: buffer loads at one per-lane byte offset each for the V and U rows, the block's row as the
  // scalar offset (64-bit addresses per element, hoisted out of the sample loop, held 32 VGPRs);
  // lanes whose rank is past R (or whose U weight is unused) point past the buffer and read 0
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)P0, (short)0, (int)(g.I * R * 4), 0x00020000);
  const int vo_v = rok ? ((iv0 + 8 * gq) * R + r8) * 4 : 0x40000000;
  const int vo_u = (lo8 && rok) ? ((it0 + 4 * gq) * R + r8) * 4 : 0x40000000;
  auto load_rows = [&](int i0, float (&pu)[NT][4]) {
    if constexpr (BLK) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        pvr[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, vo_v, (i0 + e) * R * 4, 0));
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          pu[tt][v] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, vo_u, (i0 + 16 * tt + v) * R * 4, 0));
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = vrow(e);
        pvr[e] = (rok && (!PAD || i < Ir)) ? P0[(int64_t)i * R + r8] : 0.f;
      }
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int i = it0 + 16 * tt + 4 * gq + v;
          pu[tt][v] = (lo8 && rok && (!PAD || i < Ir)) ? P0[(int64_t)i * R + r8] : 0.f;
        }
    }
  };
  auto split_rows = [&]() {
#pragma unroll
    for (int v = 0; v < 4; ++v) bsplit(pvr[2 * v], pvr[2 * v + 1], bV12[v], bV2[v], bV3[v], hV[v]);
    if constexpr (BLK)  // the U weights' loads complete here too, before this block's first LDS-DMA piece
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int v = 0; v < 4; ++v) asm volatile("" : "+v"(phiU[tt][v]));
  };
  load_rows(0, phiU);
  if constexpr (!BLK) split_rows();
  // epilogue weights: pc[r] = w_r PhiC[c][r]; row gq's ranks gq + 4 k.  BLK and RK = 16 read them
  // from an LDS table in the rank-block body's Phi1 slots (unused here) in the epilogue: those forms
  // need the registers
  constexpr bool PCL = BLK || R16;  // pc[] from the LDS table
  float pc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) pc[r] = (!PCL && cok && r < R) ? a.w[r] * PC[c * R + r] : 0.f;
  // row gq's ranks gq + 4 k: pc and w (PCL: read from the table in the epilogue stage that uses them)
  float pcg[PCL ? 1 : KR], wg[PCL ? 1 : KR];
#pragma unroll
  for (int k = 0; k < (PCL ? 1 : KR); ++k) {
    pcg[k] = pc[4 * k + (gq & 3)];
    wg[k] = gq + 4 * k < R ? a.w[gq + 4 * k] : 0.f;
  }
  // PCL table: [class 16][RK] pc, then [RK] w
  float* sPC = lds + g.du_oP1;
  if constexpr (PCL)
    for (int e = t; e < 16 * RK + RK; e += NT_)
      sPC[e] = e >= 16 * RK ? (e - 16 * RK < R ? a.w[e - 16 * RK] : 0.f)
                            : (e / RK < C && e % RK < R) ? a.w[e % RK] * PC[(e / RK) * R + e % RK] : 0.f;
  auto pcg_of = [&](int k) { return PCL ? sPC[RK * c + gq + 4 * k] : pcg[k]; };
  auto wg_of = [&](int k) { return PCL ? sPC[16 * RK + gq + 4 * k] : wg[k]; };
  for (int e = t; e < NS * NW * RK; e += NT_) sU[e] = 0.f;
  if constexpr (DIST)
    for (int e = t; e < NS * 8; e += NT_) sWv[e] = 0.f;
  // BLK: the folded T of blocks 0 .. nb - 2 of the previous sample and this wave's dPhi0 rows of
  // those blocks, [2][nb - 1][NW][NT][gq][rank 8][v 4] (lanes n < 8 only; the last block's in registers)
  float* sTB = lds + g.bs_oTB;
  const int tbn = (nb - 1) * NW * NT * 128;
  auto tb_at = [&](int bb, int tt) { return ((bb * NW + wv) * NT + tt) * 128 + gq * 32 + r8 * 4; };
  if constexpr (BLK)
    for (int e = t; e < 2 * tbn; e += NT_) sTB[e] = 0.f;

  // LDS-DMA map (as the rank-block form): wave wv issues the 1 KiB groups wv + NW gi of every sample
  uint32_t goff[NG];
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    const int slot = (wv + NW * gi) * TR_WAVE + lane;
    const int i = slot / JQ;
    const int q = slot - i * JQ;
    if (PAD) {  // source offset in the real (Ir x Jr) sample; padding: its first chunk
      const int cq = q ^ swz(i);
      goff[gi] = (i < Ir && 4 * cq < Jr) ? 4u * (uint32_t)(i * Jr + 4 * cq) : 0u;
    } else {
      goff[gi] = 4u * (uint32_t)(i * J + 4 * (q ^ swz(i)));
    }
  }
  const uint32_t lbase = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)lds));
  // LDS read offsets (floats): T row it0 + 16 tt + n, chunks 8 s + 2 gq (+1); V rows vrow(e), chunk cv
  int tro[NT], vro[8];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) tro[tt] = (it0 + 16 * tt + n) * J;
  const int tsw = swz(n);  // swz(it0 + 16 tt + n) = swz(n)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int i = vrow(e);
    vro[e] = i * J + 4 * (cv ^ swz(i));
  }

  const int64_t n0 = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t n1 = n0 + a.rows_per_wg < a.N ? n0 + a.rows_per_wg : a.N;
  const int nr = (int)(n1 > n0 ? n1 - n0 : 0);
  auto sample_of = [&](int k) -> int64_t { return n0 + (a.reverse ? (nr - 1 - k) : k); };
  auto src_of = [&](int k) -> const float* { return a.X + sample_of(k) * a.xld; };

  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);

  du_f32x4 gT[NT], gV[NVS];  // dPhi0 rows of this wave's T tiles, dPhi1 partial of its V tiles
#pragma unroll
  for (int q = 0; q < NT; ++q) gT[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < NVS; ++q) gV[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
  float dpc[KR];  // wave 0: dPhiC[c][gq + 4 k]
#pragma unroll
  for (int k = 0; k < KR; ++k) dpc[k] = 0.f;
  double lsum = 0.0;
  du_f32x4 TP[NT], VP[NVS];  // the previous sample's T and V (folded), for its epilogue
  du_f32x4 TN[NT], VN[NVS];  // DIST: this sample's, from the fold to the next iteration's top
#pragma unroll
  for (int q = 0; q < NT; ++q) TP[q] = TN[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < NVS; ++q) VP[q] = VN[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
  // DIST: Wv of the sample in ring slot zs (published by its owner) onto the held T, V; then the
  // newest sample's T, V are the held ones
  auto dist_apply = [&](int zs) {
    const float wa = sWv[zs * 8 + r8];
#pragma unroll
    for (int q = 0; q < NT; ++q) gT[q] += wa * TP[q];
#pragma unroll
    for (int q = 0; q < NVS; ++q) gV[q] += wa * VP[q];
#pragma unroll
    for (int q = 0; q < NT; ++q) TP[q] = TN[q];
#pragma unroll
    for (int q = 0; q < NVS; ++q) VP[q] = VN[q];
  };
  int64_t yP = 0;
  float cwP = 0.f;

  // ---- epilogue of one sample in 8 stages (duo_body's chain, every rank: DPP row gq carries ranks
  // gq + 4 k, k < RK / 4) ----
  // (the stages' values, one instance per epilogue: an instance shared across iterations would be
  // carried around the BLK loop, whose stages run only in a sample's first block)
  struct EpiSt {
    float uS, uR[RK];
    float e_x, e_ez, e_sum, e_S, e_q, e_Sq, e_Sy;
    float e_s2, e_d1, e_e1, e_dz, e_a[KR], e_b[KR], e_y[KR], e_w[KR], e_wv;
    bool e_isy;
  };
  auto epi = [&](EpiSt& E, int st, int zs, int64_t yE, float cwE) {
    if (TR_DUO_SKIP & 4) return;
    if (st == 0) {  // U[r] = sum of the NW waves' partials (lane r), wave order
      const float* pu = sU + zs * (RK * NW) + r8;
      E.uS = pu[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) E.uS += pu[RK * w];
    } else if (st == 1) {
#pragma unroll
      for (int r = 0; r < RK; ++r) E.uR[r] = du_rdl(E.uS, r);
      float zz;
      if constexpr (PCL) {
        du_f32x4 pq[RK / 4];
#pragma unroll
        for (int h = 0; h < RK / 4; ++h) pq[h] = *reinterpret_cast<const du_f32x4*>(sPC + RK * c + 4 * h);
        zz = pq[0][0] * E.uR[0];
#pragma unroll
        for (int r = 1; r < RK; ++r) zz = fmaf(pq[r / 4][r % 4], E.uR[r], zz);
      } else {
        zz = pc[0] * E.uR[0];
#pragma unroll
        for (int r = 1; r < 8; ++r) zz = fmaf(pc[r], E.uR[r], zz);
      }
      zz = cok ? zz : NEG;
      E.e_x = zz - du_row_max16(zz);
    } else if (st == 2) {
      E.e_ez = cok ? du_exp(E.e_x) : 0.f;
      E.e_sum = du_row_sum16(E.e_ez);
    } else if (st == 3) {
      E.e_S = E.e_ez * __builtin_amdgcn_rcpf(E.e_sum);
      E.e_q = cok ? du_exp(E.e_S) : 0.f;
      E.e_isy = cok && (int64_t)c == yE;
      E.e_Sq = E.e_S * E.e_q;
      E.e_Sy = E.e_isy ? E.e_S : 0.f;
    } else if (st == 4) {
      E.e_s2 = du_row_sum16(E.e_q);
      E.e_d1 = du_row_sum16(E.e_Sq);
      E.e_e1 = du_row_sum16(E.e_Sy);
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        const float pk = pcg_of(k);
        E.e_a[k] = du_row_sum16(E.e_Sq * pk);
        E.e_b[k] = du_row_sum16(E.e_S * pk);
        E.e_y[k] = du_row_sum16(E.e_Sy * pk);
      }
    } else if (st == 5) {
      const float is2 = __builtin_amdgcn_rcpf(E.e_s2);
      const float kk = cwE * a.scale;
      const float dot = kk * (E.e_d1 * is2 - E.e_e1);
      lsum += ((DIST || wv == 0) && lane == 0) ? (double)cwE * (double)(du_log(E.e_s2) - E.e_e1) : 0.0;
      const float dS = cok ? kk * (E.e_q * is2 - (E.e_isy ? 1.0f : 0.0f)) : 0.f;
      E.e_dz = cok ? E.e_S * (dS - dot) : 0.f;
#pragma unroll
      for (int k = 0; k < KR; ++k) E.e_w[k] = kk * (E.e_a[k] * is2 - E.e_y[k]) - dot * E.e_b[k];  // Wv[gq + 4 k]
    } else if (st == 6 && DIST) {  // publish Wv: row gq's first lane holds Wv[gq + 4 k]
      if (n == 0)
#pragma unroll
        for (int k = 0; k < KR; ++k) sWv[zs * 8 + gq + 4 * k] = E.e_w[k];
    } else if (st == 6) {
      // Wv[r] of this lane's accumulator rank r: row (r & 3)'s e_w[r >> 2], fetched from lane 16 (r & 3)
      const int src = 64 * (r8 & 3);
      float wk[KR];
#pragma unroll
      for (int k = 0; k < KR; ++k) wk[k] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(E.e_w[k])));
      if constexpr (R16)
        E.e_wv = r8 < 8 ? (r8 < 4 ? wk[0] : wk[1]) : (r8 < 12 ? wk[2] : wk[3]);
      else
        E.e_wv = r8 < 4 ? wk[0] : wk[1];
    } else if (DIST) {  // (Wv published at stage 6; every wave applies it after the next barrier)
    } else {
#pragma unroll
      for (int q = 0; q < NT; ++q) gT[q] += E.e_wv * TP[q];
#pragma unroll
      for (int q = 0; q < NVS; ++q) gV[q] += E.e_wv * VP[q];
      if constexpr (BLK) {
        if (lo8)
#pragma unroll
          for (int bb = 0; bb < nb - 1; ++bb)
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
              const du_f32x4 tp = *reinterpret_cast<const du_f32x4*>(sTB + tb_at(bb, tt));
              du_f32x4* gp = reinterpret_cast<du_f32x4*>(sTB + tbn + tb_at(bb, tt));
              *gp += E.e_wv * tp;
            }
      }
    }
    if (st == 7) {
      if (DIST || wv == 0) {  // dPhiC[c][r] += dZ[c] w_r U[r], r = gq + 4 k (DIST: the owner's partial)
#pragma unroll
        for (int k = 0; k < KR; ++k) {
          // U[gq + 4 k] (DIST: four uniform values by readlane and a select, no LDS round trip on the
          // owner's chain; selecting among E.uR[] elements would put E in scratch)
          float uk;
          if constexpr (DIST) {
            const float u0 = du_rdl(E.uS, 4 * k), u1 = du_rdl(E.uS, 4 * k + 1), u2 = du_rdl(E.uS, 4 * k + 2),
                        u3 = du_rdl(E.uS, 4 * k + 3);
            uk = gq < 2 ? (gq == 0 ? u0 : u1) : (gq == 2 ? u2 : u3);
          } else {
            uk = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * gq + 16 * k, __float_as_int(E.uS)));
          }
          dpc[k] = fmaf(E.e_dz, wg_of(k) * uk, dpc[k]);
        }
      }
    }
  };

  auto dma_piece = [&](uint32_t off, const float* src, uint32_t m0v) { du_dma_s(off, src, m0v); };
  // at NW = 8 (unpadded) a wave's group gi starts 16 (J = 128) or 32 (J = 64) rows after its group 0,
  // with the same chunk swizzle: one per-lane offset and 8 KiB more of scalar base per group (seven
  // VGPRs fewer)
  constexpr bool GAFF = NW == 8 && !PAD;
  auto goff_of = [&](int gi) { return GAFF ? goff[0] : goff[gi]; };
  auto src_of_group = [&](const float* p, int gi) { return GAFF ? p + 2048 * gi : p; };
  auto dma_sample = [&](const float* src, int slot) {
#pragma unroll
    for (int gi = 0; gi < NG; ++gi)
      dma_piece(goff_of(gi), src_of_group(src, gi), lbase + (uint32_t)(slot * 4 * SPF) + (uint32_t)(wv + NW * gi) * 1024u);
  };
  // the kernel is bound by the bytes in flight per CU, not by its issue stream (no-LDS-DMA
  // ablation: 0.256 vs 0.368 ms at c3): a ring of three keeps two samples in flight
  if (nr > 0) dma_sample(src_of(0), 0);
  if (nr > 0 && NS == 3) dma_sample(src_of(nr > 1 ? 1 : 0), 1);
  int64_t yN = nr > 0 ? lab[sample_of(0)] : 0;
#if TR_DUO_PROFILE
  unsigned long long prof[4] = {0, 0, 0, 0};
  unsigned long long prof_t = __builtin_readcyclecounter();
#endif

  // BLK: the current sample's label and class weight (set at its first block) and this wave's U
  // partial, carried over the sample's blocks; its V partial is carried in VP, which is free once
  // the first block's epilogue stage 7 has consumed the previous sample's
  int64_t yB = 0;
  float cwB = 0.f, uacc = 0.f;
  // (!BLK: k is the sample and b = 0; BLK: block b of sample k, ring slot = block-iteration parity)
  auto iter = [&](auto slot_c, int k, auto b_c) {
    constexpr int SL = decltype(slot_c)::value;
    constexpr int b = decltype(b_c)::value;
    constexpr bool bfirst = b == 0, blast = b == nb - 1;
    int64_t yC;
    if constexpr (BLK) {
      if (bfirst) {
        yB = yN;
        if (!(TR_DUO_SKIP & 16)) yN = lab[sample_of(k + 1 < nr ? k + 1 : k)];
      }
      yC = yB;
    } else {
      yC = yN;
      const bool more = k + 1 < nr;
      if (!(TR_DUO_SKIP & 16)) yN = lab[sample_of(more ? k + 1 : k)];
    }
    if (NS == 3 && J32)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // own pieces of k (those of k + 1 may be in flight)
    else if (NS == 3)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    TR_DUO_MARK(0);
    du_barrier();  // everyone's pieces of k; U partials of k - 1
    TR_DUO_MARK(1);
    float cwC;
    if constexpr (BLK) {
      if (bfirst) cwB = du_rdl(cwl, (int)yC);
      cwC = cwB;
      split_rows();  // this block's Phi0 operands (loaded at the end of the previous block)
    } else {
      cwC = du_rdl(cwl, (int)yC);
    }
    if constexpr (DIST) dist_apply((SL + 2 * NS - 2) % NS);  // Wv(k - 2), published at the end of k - 1
    // sample k + 2 into this slot once it is read (past the end: a harmless refill of a valid sample)
    const int kd = k + NS - 1;  // the sample this iteration's DMA brings in
    constexpr int PS = (SL + NS - 1) % NS;     // slot of sample k - 1 (and of the DMA's target)
    const float* psrc;
    if constexpr (BLK) {  // the next block (of this sample or the next), or this one again past the end
      const float* cur = src_of(k) + (int64_t)b * I * Jr;
      psrc = (TR_DUO_SKIP & 1) ? cur : b + 1 < nb ? cur + (int64_t)I * Jr : k + 1 < nr ? src_of(k + 1) : cur;
    } else {
      psrc = (kd < nr && !(TR_DUO_SKIP & 1)) ? src_of(kd) : src_of(nr - 1);
    }
    const uint32_t pm0 = lbase + (uint32_t)(PS * 4 * SPF) + (uint32_t)wv * 1024u;
    // U partial slots: per ring slot (!BLK), per sample parity (BLK)
    const int zsP = BLK ? ((k - 1) & 1) : PS, zsC = BLK ? (k & 1) : SL;
    EpiSt E;
    // DIST: this wave runs the epilogue of k - 1 if it owns that sample
    const bool own = !DIST || (k + NW - 1) % NW == wv;
    if (bfirst && own) epi(E, 0, zsP, yP, cwP);
    const float* sb = lds + SL * SPF;
    du_f32x4 aT[NT], aV[NVS];
#pragma unroll
    for (int q = 0; q < NT; ++q) aT[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NVS; ++q) aV[q] = du_f32x4{0.f, 0.f, 0.f, 0.f};
    // every operand of sample k into registers
    constexpr int NU = NT * NKT;  // T steps (4; J = 32: 2); then NVS V steps (one j-tile each)
    du_f32x4 xv[8], xt[NU][2];
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = *reinterpret_cast<const du_f32x4*>(sb + vro[e]);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int tt = u / NKT, s = u - tt * NKT;
      const int q0 = 8 * s + 2 * gq;
      xt[u][0] = *reinterpret_cast<const du_f32x4*>(sb + tro[tt] + 4 * (q0 ^ tsw));
      xt[u][1] = *reinterpret_cast<const du_f32x4*>(sb + tro[tt] + 4 * ((q0 + 1) ^ tsw));
    }
#pragma unroll
    for (int st = 0; st < NU + NVS; ++st) {
      if (!(TR_DUO_SKIP & 8)) dma_piece(goff_of(st), src_of_group(psrc, st), pm0 + (uint32_t)st * (uint32_t)(NW * 1024));
      sl_u4 x1, x2, x3;  // the k step's X pieces (pairs per VGPR)
      auto split = [&](float e0, float e1, int v) {
        if constexpr (EXACT) {
          uint32_t h1, h2, h3;
          sl_split2(e0, e1, h1, h2, h3);
          x1[v] = h1;
          x2[v] = h2;
          x3[v] = h3;
        } else {
          const uint32_t h = sl_pack_rne(e0, e1);
          x1[v] = h;
          x2[v] = bs_pack_h(e0 - sl_lo_f32(h), e1 - sl_hi_f32(h));
        }
      };
      // smallest products first into the accumulator
      // (RK = 16: acc += x3 b1 + x2 b2 + x2 b1 + x1 b3 + x1 b2 + x1 b1 exact, x2 h + x1 b3 + x1 b2 +
      // x1 b1 fast; dropped x3 b2, x2 b3, x3 b3: < 2^-25 |x b|)
      auto gemm = [&](du_f32x4& acc, const uint32_t (&b12)[4], const uint32_t (&b2)[4], const uint32_t (&b3)[4],
                      const uint32_t (&hh)[4]) {
        if constexpr (R16) {
          if constexpr (EXACT) {
            acc = bs_mfma(x3, b12, acc);
            acc = bs_mfma(x2, b2, acc);
            acc = bs_mfma(x2, b12, acc);
          } else {
            acc = bs_mfma_h(x2, hh, acc);
          }
          acc = bs_mfma(x1, b3, acc);
          acc = bs_mfma(x1, b2, acc);
          acc = bs_mfma(x1, b12, acc);
        } else {
          if constexpr (EXACT) {
            acc = bs_mfma(x3, b12, acc);
            acc = bs_mfma(x2, b12, acc);
          } else {
            acc = bs_mfma_h(x2, hh, acc);
          }
          acc = bs_mfma(x1, b3, acc);
          acc = bs_mfma(x1, b12, acc);
        }
      };
      if (st < NU) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const du_f32x4& xr = xt[st][v >> 1];
          split(xr[2 * (v & 1)], xr[2 * (v & 1) + 1], v);
        }
        const int tt = st / NKT, s = st - tt * NKT;
        gemm(aT[tt], bT12[s], bT2[R16 ? s : 0], bT3[s], hT[s]);
      } else {
        const int tv = st - NU;  // j-tile: element tv of each row's chunk
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          if constexpr (J32) {  // element tv (lanes n < 8) or tv + 2 (n >= 8) of each row's chunk
            const bool hi = n >= 8;
            split(hi ? xv[2 * v][tv + 2] : xv[2 * v][tv], hi ? xv[2 * v + 1][tv + 2] : xv[2 * v + 1][tv], v);
          } else {
            split(xv[2 * v][tv], xv[2 * v + 1][tv], v);
          }
        }
        gemm(aV[tv], bV12, bV2, bV3, hV);
      }
      if constexpr (J32) {  // four steps: stages 1..6 two per step, 7 after them
        if (bfirst && st >= 1 && own) {
          epi(E, 2 * st - 1, zsP, yP, cwP);
          epi(E, 2 * st, zsP, yP, cwP);
        }
      } else {
        if (bfirst && st >= 1 && st <= 7) epi(E, st, zsP, yP, cwP);  // (bfirst, st: compile-time)
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (J32)
      if (bfirst && own) epi(E, 7, zsP, yP, cwP);
    TR_DUO_MARK(2);
    // fold the piece columns (rank r = column r + column r + 8), U partial of this wave -> LDS
    float u = BLK ? uacc : 0.f;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if constexpr (!R16) aT[tt][v] += du_dpp<0x128>(aT[tt][v]);  // row_ror:8
        u = fmaf(phiU[tt][v], aT[tt][v], u);
      }
      if (blast && DIST) {
        TN[tt] = aT[tt];
      } else if (blast) {
        TP[tt] = aT[tt];
      } else if (lo8) {  // (BLK) block b's T until the sample's epilogue
        *reinterpret_cast<du_f32x4*>(sTB + tb_at(b, tt)) = aT[tt];
      }
    }
    if constexpr (BLK) {
      uacc = blast ? 0.f : u;
      // the next block's Phi0 rows (issuing them at the first V step instead, with the U weights
      // double-buffered, measured no faster)
      load_rows(b + 1 < nb ? (b + 1) * I : 0, phiU);
    }
    if constexpr (BLK) {  // V over the blocks (folded at the last)
#pragma unroll
      for (int q = 0; q < NVS; ++q) aV[q] = bfirst ? aV[q] : VP[q] + aV[q];
      if (!blast)
#pragma unroll
        for (int q = 0; q < NVS; ++q) VP[q] = aV[q];
    }
    if (blast) {
#pragma unroll
      for (int q = 0; q < NVS; ++q) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if constexpr (!R16) aV[q][v] += du_dpp<0x128>(aV[q][v]);
        if constexpr (DIST)
          VN[q] = aV[q];
        else
          VP[q] = aV[q];
      }
      u = du_xor32_sum(du_xor16_sum(u));  // lane (n < RK, any row): this wave's U partial of rank n
      if (lane < RK) sU[zsC * (RK * NW) + wv * RK + lane] = u;
      yP = yC;
      cwP = cwC;
    }
    TR_DUO_MARK(3);
    if constexpr (BLK) __builtin_amdgcn_sched_barrier(0);  // (no scheduling across the block boundary)
  };
  using B0 = std::integral_constant<int, 0>;
  if constexpr (BLK) {
    // one trip: the blocks of one sample (NB even) or of two (NB odd), so that every block's ring
    // slot (block-iteration parity) is a compile-time constant
    constexpr int TRIP = NB % 2 == 0 ? NB : 2 * NB;
    for (int k = 0; k < nr; k += TRIP / NB) {
      for_each_ic(std::make_integer_sequence<int, TRIP>(), [&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
        if (TRIP == NB || k + t / NB < nr)
          iter(std::integral_constant<int, t % 2>(), k + t / NB, std::integral_constant<int, t % NB>());
      });
    }
  } else {
    for (int k = 0; k < nr; k += NS) {
      iter(std::integral_constant<int, 0>(), k, B0());
      if (k + 1 < nr) iter(std::integral_constant<int, 1>(), k + 1, B0());
      if (NS == 3 && k + 2 < nr) iter(std::integral_constant<int, NS == 3 ? 2 : 0>(), k + 2, B0());
    }
  }
#if TR_DUO_PROFILE
  if (lane == 0 && blockIdx.x < 512)
    for (int q = 0; q < 4; ++q) g_duo_prof[blockIdx.x][wv][q] = prof[q];
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (harmless) refill has landed
  du_barrier();  // U partials of the last sample
  if (DIST && nr > 0) {  // Wv(nr - 2) onto its T, V; the last sample's epilogue on its owner; its Wv
    dist_apply((nr + NS - 2) % NS);
    if ((nr - 1) % NW == wv) {
      EpiSt E;
#pragma unroll
      for (int st = 0; st < 8; ++st) epi(E, st, (nr - 1) % NS, yP, cwP);
    }
    du_barrier();
    dist_apply((nr - 1) % NS);
  } else if (nr > 0) {
    EpiSt E;
#pragma unroll
    for (int st = 0; st < 8; ++st) epi(E, st, BLK ? (nr - 1) & 1 : (nr - 1) % NS, yP, cwP);
  }
  if constexpr (DIST)
    if (lane == 0) sLs[wv] = lsum;  // (read after the reduction's barriers)

  // ---- fixed-order reduction into an LDS image of the arena (wave order), slab ----
  float* sG = lds + g.du_oG;
  __syncthreads();
  for (int64_t e = t; e < g.slab; e += NT_) sG[e] = 0.f;
  __syncthreads();
  for (int ws = 0; ws < NW; ++ws) {
    if (ws == wv && lo8 && rok) {
      const int ib = BLK ? (nb - 1) * I : 0;  // BLK: the register rows are the last block's
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (!PAD || BLK || it0 + 16 * tt + 4 * gq + v < g.I) sG[(ib + it0 + 16 * tt + 4 * gq + v) * R + r8] += gT[tt][v];
      if constexpr (BLK)
#pragma unroll
        for (int bb = 0; bb < nb - 1; ++bb)
#pragma unroll
          for (int tt = 0; tt < NT; ++tt) {
            const du_f32x4 gt = *reinterpret_cast<const du_f32x4*>(sTB + tbn + tb_at(bb, tt));
#pragma unroll
            for (int v = 0; v < 4; ++v) sG[(bb * I + it0 + 16 * tt + 4 * gq + v) * R + r8] += gt[v];
          }
#pragma unroll
      for (int q = 0; q < NVS; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          // chunk (row 4 gq + v of the tile) -> j = 4 chunk + tile (J = 32: tile row m -> j = 4 (m & 7) + q + 2 (m >> 3))
          const int m = 4 * gq + v;
          const int j = J32 ? 4 * (m & 7) + q + 2 * (m >> 3) : 4 * (cv - n + m) + q;
          if (!PAD || j < Jr) sG[g.offP1 + j * R + r8] += gV[q][v];
        }
    }
    if (ws == wv && (DIST || wv == 0) && cok) {
#pragma unroll
      for (int k = 0; k < KR; ++k)
        if (gq + 4 * k < R) sG[g.offPC + c * R + gq + 4 * k] += dpc[k];
    }
    __syncthreads();
  }
  if (wv == 0) {
    if constexpr (DIST) {  // the owners' partials in wave order
      double s = 0.0;
      for (int w = 0; w < NW; ++w) s += sLs[w];
      lsum = s;
    } else {
      lsum = tr_wave_allreduce_d(lsum);
    }
    if (lane == 0) {
      a.dpart[2 * blockIdx.x] = lsum;
      a.dpart[2 * blockIdx.x + 1] = 0.0;
    }
  }
  float* slab = a.gpart + (int64_t)blockIdx.x * g.slab;
  for (int64_t e = t; e < g.slab; e += NT_) slab[e] = sG[e];
}

// NW waves per workgroup, 8 / NW workgroups per CU (the second bound is waves per SIMD: two,
// 256 VGPRs each), a ring of NS samples.  (J = 32 at three waves per SIMD, 168 VGPRs with every
// wave running every epilogue: 43-64 % of HBM; the one-wave epilogue at two: 53-68 %, and it does not
// fit 168; profiles/r06_mnl_j32)
template <int JT, int NW, int NS, bool PAD, bool EXACT, int NB, int RK>
__global__ __launch_bounds__(NW * TR_WAVE, 2) void k_mnl_bsp(MnlGeom g, DuArgs a, const int64_t* __restrict__ lab,
                                                               const float* __restrict__ class_w,
                                                               const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / TR_WAVE);
  bsp_body<JT, NW, NS, PAD, EXACT, NB, RK>(g, a, lab, class_w, lds, wv, lane);
}

template <int JT>
__global__ __launch_bounds__(DU_T, 2) void k_mnl_duo(MnlGeom g, DuArgs a, const int64_t* __restrict__ lab,
                                                  const float* __restrict__ class_w, const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (stop != nullptr && *stop != 0) return;
  const int lane = threadIdx.x & (TR_WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / TR_WAVE);
  duo_body<JT>(g, a, lab, class_w, lds, wv, lane);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// the split body's instantiations (J, NW, ring slots): (32 NW, 64) samples with NW = 2..8, (16 NW,
// 128) with NW = 4, 6, 8; a ring of three at NW = 5, 6; (32 NW, 32) with NW = 2..8, rings of two and three
#define TR_BSP_LIST(X) \
  X(64, 2, 2) X(64, 3, 2) X(64, 4, 2) X(64, 5, 2) X(64, 5, 3) X(64, 6, 2) X(64, 6, 3) X(64, 7, 2) \
  X(64, 8, 2) X(128, 4, 2) X(128, 6, 2) X(128, 6, 3) X(128, 8, 2)                                 \
  X(32, 2, 2) X(32, 2, 3) X(32, 3, 2) X(32, 3, 3) X(32, 4, 2) X(32, 4, 3) X(32, 5, 2) X(32, 5, 3) \
  X(32, 6, 2) X(32, 6, 3) X(32, 7, 2) X(32, 7, 3) X(32, 8, 2) X(32, 8, 3)
// ... and its row-block instantiations (J, NW, ring slots, blocks): samples of NB blocks of 32 NW x
// 64 or 16 NW x 128 rows.  (At (64, 8) only two blocks fit the LDS; (128, 8) with three and every
// four-block form spill: such samples, e.g. (384, 128), (512, 128), (768, 64), run the two-pass kernels.)
#define TR_BSP_BLK_LIST(X) \
  X(64, 8, 2, 2) X(64, 6, 2, 2) X(64, 6, 2, 3) X(128, 8, 2, 2) X(128, 6, 2, 2) X(128, 6, 2, 3)
// ... and its 16-rank instantiations (ranks 9..16; J, NW, ring slots).  (128, 6) with a ring of three
// spills; so does the padded (128, 8) form, whose samples run k_mnl_fused or the two-pass kernels.
#define TR_BSP_R16_LIST(X) \
  X(64, 2, 2) X(64, 3, 2) X(64, 4, 2) X(64, 5, 2) X(64, 5, 3) X(64, 6, 2) X(64, 6, 3) X(64, 7, 2) \
  X(64, 8, 2) X(128, 4, 2) X(128, 6, 2) X(128, 8, 2)
static bool bsp_blk_compiled(int jt, int nw, int nb) {
#define TR_BSP_BLK_HAS(J_, NW_, NS_, NB_) \
  if (jt == J_ && nw == NW_ && nb == NB_) return true;
  TR_BSP_BLK_LIST(TR_BSP_BLK_HAS)
#undef TR_BSP_BLK_HAS
  return false;
}
static const void* duo_kernel(const MnlGeom& g, bool exact) {
  if (g.bsp) {
#define TR_BSP_PTR5(J_, NW_, NS_, NB_, RK_)                                                               \
    if (exact)                                                                                            \
      return g.du_pad ? reinterpret_cast<const void*>(&k_mnl_bsp<J_, NW_, NS_, true, true, NB_, RK_>)      \
                      : reinterpret_cast<const void*>(&k_mnl_bsp<J_, NW_, NS_, false, true, NB_, RK_>);    \
    return g.du_pad ? reinterpret_cast<const void*>(&k_mnl_bsp<J_, NW_, NS_, true, false, NB_, RK_>)       \
                    : reinterpret_cast<const void*>(&k_mnl_bsp<J_, NW_, NS_, false, false, NB_, RK_>);
#define TR_BSP_PTR(J_, NW_, NS_)                                                                          \
  if (g.bs_rk == 8 && g.du_nb == 1 && g.du_jt == J_ && g.du_nw == NW_ && g.du_ns == NS_) {                 \
    TR_BSP_PTR5(J_, NW_, NS_, 1, 8)                                                                       \
  }
#define TR_BSP_BLK_PTR(J_, NW_, NS_, NB_)                                                                 \
  if (g.bs_rk == 8 && g.du_nb == NB_ && g.du_jt == J_ && g.du_nw == NW_ && g.du_ns == NS_) {               \
    TR_BSP_PTR5(J_, NW_, NS_, NB_, 8)                                                                     \
  }
#define TR_BSP_R16_PTR(J_, NW_, NS_)                                                                      \
  if (g.bs_rk == 16 && g.du_nb == 1 && g.du_jt == J_ && g.du_nw == NW_ && g.du_ns == NS_) {                \
    TR_BSP_PTR5(J_, NW_, NS_, 1, 16)                                                                      \
  }
    TR_BSP_LIST(TR_BSP_PTR)
    TR_BSP_BLK_LIST(TR_BSP_BLK_PTR)
    TR_BSP_R16_LIST(TR_BSP_R16_PTR)
#undef TR_BSP_PTR
#undef TR_BSP_BLK_PTR
#undef TR_BSP_R16_PTR
#undef TR_BSP_PTR5
    return nullptr;
  }
  return g.J == 64 ? reinterpret_cast<const void*>(&k_mnl_duo<64>) : reinterpret_cast<const void*>(&k_mnl_duo<128>);
}

// LDS carve of one duo-family workgroup with a ring of ns samples of spf floats (sets the offsets,
// returns the floats)
static int64_t duo_carve(MnlGeom* g, int nw, int64_t spf, int ns) {
  int64_t o = ns * spf;
  g->du_oZ = (int)o;
  o += 2 * 16 * 4;
  g->du_oP1 = (int)o;
  o += 8LL * (g->du_jt + 4);
  o = (o + 3) & ~(int64_t)3;
  g->bs_oU = (int)o;  // bsp: [ns][NW waves][bs_rk ranks] U partials
  o += ns * nw * (g->bs_rk == 16 ? 16 : 8);
  g->bs_oW = (int)o;  // bsp one-wave epilogue (J = 32): [ns][8] Wv, [8] double loss partials
  o += ns * 8 + 16;
  g->bs_oTB = (int)o;  // bsp row blocks: [2][nb - 1][NW][NT][128] (T, dPhi0) of the earlier blocks
  if (g->du_nb > 1) o += 2LL * (g->du_nb - 1) * nw * (g->du_jt == 128 ? 1 : 2) * 128;
  g->du_oG = g->slab <= ns * spf ? 0 : (int)o;  // the arena image aliases the drained ring
  if (g->du_oG) o += g->slab;
  return (o + 3) & ~(int64_t)3;
}

// the narrowest sample the split body takes (the 32-wide form, padded up to J = 32)
constexpr int kBspJ32Min = 24;

void mnl_duo_geom(MnlGeom* g) {
  g->duo = 0;
  g->bsp = 0;
  g->bs_exact = 0;
  g->du_nw = 4;
  g->du_wpc = 2;
  g->du_ns = 2;
  g->du_pad = 0;
  g->du_jt = g->J;
  g->du_nb = 1;
  g->bs_rk = g->R > 8 ? 16 : 8;  // the split body's rank columns
  const char* env = std::getenv("TR_MNL_DUO");
  if (env != nullptr && env[0] == '0') return;
  // (J from 28 up: padded to 64, J = 32 runs at 46-48 % of HBM against 14-37 % on the fallbacks; at
  // J = 24 and 16 the two-pass kernels are faster, 34 vs 29 % and 34 vs 25 %, tools/mnl_shapes.py)
  if (g->C > kMnlCMax || g->J % 4 != 0 || g->J < kBspJ32Min || g->J > 128) return;
  // the compiled row width: J itself (32, 64, 128) or the next one up (a padded sample).  32 for
  // samples of up to 256 rows at rank <= 8 (the 32-wide body has no row-block or 16-rank forms);
  // J = 28..32 beyond those padded to 64 as before
  const bool j32 = g->J <= 32 && g->I <= 256 && g->R <= 8;
  if (g->J < 28 && !j32) return;
  const int jt = j32 ? 32 : g->J <= 64 ? 64 : 128;
  // compiled shapes: the rank-block body takes a 32 KiB sample as (128, 64) or (64, 128) (two
  // 64-row blocks, 8 LDS-DMA groups per wave, chunk swizzle q ^ (i & 15)); the split body takes
  // those, every (32 NW, 64) sample with NW = 2..8 (one wave per 32 rows) and every (16 NW, 128)
  // sample with NW = 4, 6, 8 (one wave per 16 rows); 8 / NW workgroups per CU
  const bool s32k = g->full && g->I * g->J == 8192 && g->smask == 15;
  // (a sample whose I is not a whole number of wave rows runs padded: its rows past I read any valid
  // row of the sample and meet zero Phi0 rows)
  // (any I up to the wave-row ceiling: a sample of a few rows still runs 3.6-4x faster padded to
  // two wave rows than on the fused kernel, whose cost per sample does not fall with I)
  const bool wide = (jt <= 64 && g->I <= 256) || (jt == 128 && g->I <= 128);
  // form: the f32 rank-block body where it fits (R in 5..8: two rank blocks), the bf16-split body
  // for R <= 4 and for the other (I, 64) shapes; TR_DUO_SPLIT=1 takes the split body for R <= 8,
  // =0 the rank-block body only.  (With the non-temporal sample DMA both run at the same rate at
  // c3 — 0.339 / 0.343-0.347 ms, the sample stream bounds them — and the rank-block form is the
  // more accurate: 3.1e-7 vs 7.2e-7 normwise from fp64 at full c3 size; the reference's own op
  // sequence in fp32 at the same factors 4.0e-6.)
  const char* spl = std::getenv("TR_DUO_SPLIT");
  const bool force_split = spl != nullptr && spl[0] == '1', no_split = spl != nullptr && spl[0] == '0';
  const bool rankblock = s32k && g->nrb == 2;
  // taller samples (above 256 rows at J <= 64, 128 at J <= 128) stream through the ring in du_nb row
  // blocks of 32 NW x 64 / 16 NW x 128, NW = 8 or 6 (one workgroup per CU), the first whose rows
  // divide I and whose ring plus the earlier blocks' T / dPhi0 images fit the LDS
  int blk_nw = 0;
  if (!wide && !s32k && g->R <= 8 && !no_split) {
    for (const int c : {8, 6}) {
      const int ib = jt == 64 ? 32 * c : 16 * c;
      if (g->I % ib != 0 || g->I / ib < 2 || !bsp_blk_compiled(jt, c, g->I / ib)) continue;
      g->du_nb = g->I / ib;
      g->du_jt = jt;
      if (duo_carve(g, c, (int64_t)ib * jt, 2) * 4 <= 160 * 1024) {
        blk_nw = c;
        break;
      }
      g->du_nb = 1;
    }
  }
  const bool bsp = (s32k || wide || blk_nw) && g->R <= 16 && !no_split && (force_split || !rankblock);
  if (!bsp && !rankblock) {
    g->du_nb = 1;
    return;
  }
  const int nw = !bsp ? 4 : blk_nw ? blk_nw : jt <= 64 ? (g->I > 32 ? (g->I + 31) / 32 : 2) : (g->I > 64 ? 2 * ((g->I + 31) / 32) : 4);
  g->du_jt = bsp ? jt : g->J;
  const int wpc = 8 / nw;  // workgroups per CU: eight waves, two per SIMD
  // LDS floats per (padded) sample, or per row block
  const int64_t spf = (int64_t)(!bsp ? g->I : jt <= 64 ? 32 * nw : 16 * nw) * g->du_jt;
  // a padded sample fills at least a third of its padded shape (TR_DUO_ANYFILL=1: any fill, for the
  // tests): below that the two-pass kernels' ~2.6 TB/s on the real bytes beats the body's rate on
  // the padded ones ((16, 64): 25.8 vs 32.3 % of HBM, (24, 48) at 0.28 even, (24, 64) at 0.375 37.5 vs
  // 33.1 %; profiles/r05_mnl_fallbacks.txt)
  const char* anyfill = std::getenv("TR_DUO_ANYFILL");
  if (bsp && 3 * (int64_t)g->I * g->J < spf * g->du_nb && !(anyfill && std::atoi(anyfill) == 1)) return;
  auto carve = [&](int ns) { return duo_carve(g, nw, spf, ns); };
  // the split body at NW = 5, 6 (one workgroup per CU: 80 / 96 KiB in flight with two slots) takes
  // a ring of three samples: (160, 64) 58.9 -> 61.4 %, (192, 64) 65.4 -> 68.5 %, (96, 128) 65.8 ->
  // 69.7 % of HBM (tools/mnl_shapes.py, two runs each); at NW = 3 (two workgroups per CU) three
  // slots measured the same as two.
  // The 32-wide body (half the bytes per slot) takes a ring of three at every NW.
  const bool ring3_ok =
      bsp && g->du_nb == 1 && (jt == 32 || ((nw == 5 || nw == 6) && (jt == 64 || (nw == 6 && g->bs_rk == 8))));
  int ns = 2;
  if (ring3_ok && wpc * carve(3) * 4 <= 160 * 1024) ns = 3;
  const int64_t o = carve(ns);
  if (wpc * o * 4 > 160 * 1024) return;  // wpc workgroups per CU
  g->du_lds_floats = (int)o;
  g->du_nw = nw;
  g->du_wpc = wpc;
  g->du_ns = ns;
  g->du_pad = bsp && spf * g->du_nb != (int64_t)g->I * g->J ? 1 : 0;
  g->duo = 1;
  g->bsp = bsp ? 1 : 0;
}

// the body g describes runs without spills at du_wpc workgroups per CU (the split body in both of
// its X forms: the plan picks one per X, tr_plan_set_x_range)
static hipError_t duo_kernel_ok(const MnlGeom& g, bool* ok) {
  *ok = true;
  for (int form = 0; form < (g.bsp ? 2 : 1) && *ok; ++form) {
    const void* k = duo_kernel(g, form == 1);
    if (k == nullptr) {
      *ok = false;
      return hipSuccess;
    }
    const size_t lds = (size_t)g.du_lds_floats * 4;
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipFuncAttributes attr;
    e = hipFuncGetAttributes(&attr, k);
    if (e != hipSuccess) return e;
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, g.du_nw * TR_WAVE, lds);
    if (e != hipSuccess) return e;
    *ok = attr.localSizeBytes == 0 && nb >= g.du_wpc;  // no spills, du_wpc per CU
  }
  return hipSuccess;
}

hipError_t mnl_duo_prepare(MnlGeom* g) {
  if (!g->duo) return hipSuccess;
  bool ok = false;
  hipError_t e = duo_kernel_ok(*g, &ok);
  if (e != hipSuccess) return e;
  if (ok) return hipSuccess;
  if (g->bsp && g->du_ns == 3) {  // a ring of two instead (the three-slot instantiation spills)
    const int64_t spf = (int64_t)(g->du_jt <= 64 ? 32 : 16) * g->du_nw * g->du_jt;
    g->du_ns = 2;
    g->du_lds_floats = (int)duo_carve(g, g->du_nw, spf, 2);
    e = duo_kernel_ok(*g, &ok);
    if (e != hipSuccess) return e;
    if (ok) return hipSuccess;
  }
  if (g->bsp && g->full && g->I * g->J == 8192 && g->nrb == 2) {  // the rank-block form instead
    g->bsp = 0;
    g->du_nb = 1;
    g->du_nw = 4;
    g->du_wpc = 2;
    g->du_ns = 2;
    g->du_pad = 0;
    g->du_jt = g->J;
    g->du_lds_floats = (int)duo_carve(g, 4, 8192, 2);  // its own carve (the split body's may differ)
    e = duo_kernel_ok(*g, &ok);
    if (e != hipSuccess) return e;
    if (ok) return hipSuccess;
  }
  g->duo = 0;  // k_mnl_fused (where it fits)
  g->bsp = 0;
  g->du_nb = 1;
  g->du_nw = 4;
  g->du_wpc = 2;
  g->du_ns = 2;
  g->du_pad = 0;
  g->du_jt = g->J;
  return hipSuccess;
}

hipError_t launch_mnl_duo(const MnlGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                          const float* w, const int64_t* lab, const float* class_w, float scale, float* gpart,
                          double* dpart, int64_t rows_per_wg, int reverse, const int32_t* stop, hipStream_t st) {
  if (grid < 1 || rows_per_wg < 0 || xld % 4 != 0 || (int64_t)grid * rows_per_wg < N) return hipErrorInvalidValue;
  DuArgs a{X, N, xld, phi, w, scale, gpart, dpart, rows_per_wg, reverse};
  const size_t lds = (size_t)g.du_lds_floats * 4;
  if (g.bsp) {
#define TR_BSP_LAUNCH5(J_, NW_, NS_, NB_, RK_)                                                            \
    if (g.du_pad && g.bs_exact)                                                                           \
      hipLaunchKernelGGL((k_mnl_bsp<J_, NW_, NS_, true, true, NB_, RK_>), dim3(grid), dim3(NW_ * TR_WAVE), lds, \
                         st, g, a, lab, class_w, stop);                                                   \
    else if (g.du_pad)                                                                                    \
      hipLaunchKernelGGL((k_mnl_bsp<J_, NW_, NS_, true, false, NB_, RK_>), dim3(grid), dim3(NW_ * TR_WAVE), lds, \
                         st, g, a, lab, class_w, stop);                                                   \
    else if (g.bs_exact)                                                                                  \
      hipLaunchKernelGGL((k_mnl_bsp<J_, NW_, NS_, false, true, NB_, RK_>), dim3(grid), dim3(NW_ * TR_WAVE), lds, \
                         st, g, a, lab, class_w, stop);                                                   \
    else                                                                                                  \
      hipLaunchKernelGGL((k_mnl_bsp<J_, NW_, NS_, false, false, NB_, RK_>), dim3(grid), dim3(NW_ * TR_WAVE),     \
                         lds, st, g, a, lab, class_w, stop);                                              \
    return hipGetLastError();
#define TR_BSP_LAUNCH(J_, NW_, NS_)                                                                       \
  if (g.bs_rk == 8 && g.du_nb == 1 && g.du_jt == J_ && g.du_nw == NW_ && g.du_ns == NS_) {                 \
    TR_BSP_LAUNCH5(J_, NW_, NS_, 1, 8)                                                                    \
  }
#define TR_BSP_BLK_LAUNCH(J_, NW_, NS_, NB_)                                                              \
  if (g.bs_rk == 8 && g.du_nb == NB_ && g.du_jt == J_ && g.du_nw == NW_ && g.du_ns == NS_) {               \
    TR_BSP_LAUNCH5(J_, NW_, NS_, NB_, 8)                                                                  \
  }
#define TR_BSP_R16_LAUNCH(J_, NW_, NS_)                                                                   \
  if (g.bs_rk == 16 && g.du_nb == 1 && g.du_jt == J_ && g.du_nw == NW_ && g.du_ns == NS_) {                \
    TR_BSP_LAUNCH5(J_, NW_, NS_, 1, 16)                                                                   \
  }
    TR_BSP_LIST(TR_BSP_LAUNCH)
    TR_BSP_BLK_LIST(TR_BSP_BLK_LAUNCH)
    TR_BSP_R16_LIST(TR_BSP_R16_LAUNCH)
    return hipErrorInvalidValue;
#undef TR_BSP_LAUNCH
#undef TR_BSP_BLK_LAUNCH
#undef TR_BSP_R16_LAUNCH
#undef TR_BSP_LAUNCH5
  } else if (g.J == 64) {
    hipLaunchKernelGGL((k_mnl_duo<64>), dim3(grid), dim3(DU_T), lds, st, g, a, lab, class_w, stop);
  } else {
    hipLaunchKernelGGL((k_mnl_duo<128>), dim3(grid), dim3(DU_T), lds, st, g, a, lab, class_w, stop);
  }
  return hipGetLastError();
}

}  // namespace tr

#if TR_DUO_PROFILE
extern "C" int tr_duo_profile_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_duo_prof), sizeof(g_duo_prof));
}
#endif

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_mnl_duo() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_mnl_duo<64>));
}
}  // namespace tr
