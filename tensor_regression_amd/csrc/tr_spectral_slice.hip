// tr_spectral_slice.hip — column-slice single-pass kernel of the spectral fit model
// (spectral_tensor_regression.py stepwise_spectral_model :339-390 + lin_model :118-165, the
// fit_Adam loss at :716-717; SURVEY.md §8 row a14, BASELINE config 5).
//
// Same math as k_spec_fused (tr_spectral.hip header), different ownership.  k_spec_fused holds
// one whole sample in LDS and all eight waves walk it in lock-step: forward GEMM, a long
// epilogue through LDS, gradient GEMM, with block barriers for the LDS-DMA refill; the matrix
// cores idle through the epilogue and the barriers (39 % busy at config 5).  Here every wave
// OWNS a private column slice of every sample:
//
//   wave wv = (pair p = wv & 3, half hw = wv >> 2) owns d in [32p, 32p+32) (two 16-row d tiles,
//   interleaved: tile h holds the d with d % 2 == h) and w in [hw*W/2, (hw+1)*W/2).
//
//   forward   T_p,hw (32 d x 32 k) = X[w in half, d in pair]^T . Phi0[w in half, :] on
//             v_mfma_f32_16x16x4_f32, Phi0's B fragments of the half resident in registers;
//             column tile 0 = the spectral columns (C0, Rs*Cc <= 16), tile 1 = the lin columns
//             (A0, Rn <= 16)
//   exchange  the spectral tiles of the two halves are summed (one LDS exchange with the
//             partner wave wv ^ 4); the lin part is linear in T and needs no exchange
//   epilogue  Z / V column partials from registers -> one LDS reduction over the 8 waves ->
//             y_hat, residual, dZ, dV -> dT_n in registers, directly in the MFMA accumulator
//             layout the gradient GEMM consumes as its B operand (k step i of lane group g
//             <-> d row 4g + i of the tile)
//   gradient dPhi0[w in half, :] += X[w in half, d in pair] . dT_n[d in pair, :] into
//             accumulators that live for the whole launch (summed over the four pairs once,
//             at the end)
//
// so a wave reads only its own slice: it fills the slice by its own LDS-DMA (4-B pieces, any
// permutation of the 64 floats of a piece) and waits on its own vmcnt — no barrier for X.  The
// next sample's slice streams into the rows the gradient GEMM has finished with.  Two barriers
// per sample remain (the partner exchange and the 8-wave column reduction).  Rows d >= 128
// (D = 129 at config 5) are a VALU forward partial plus one zero-padded k step of the gradient
// GEMM.  LDS image of a slice: 64 chunks of 2 rows x 32 columns (256 B = one bank row); the
// 16-B slot of (row, 4-column quad cq) in chunk r is (cq + 8 (row & 1)) ^ swz(r & 7): the forward
// ds_read_b64 (two d tiles) and the gradient ds_read_b128 (8 consecutive d) are conflict-free.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "tr_common.h"
#include "tr_spectral.h"

#ifndef TR_SLICE_SKIP
#define TR_SLICE_SKIP 0  // timing ablation only (results invalid): 1 no LDS-DMA after the first sample,
                         // 2 no forward MFMAs, 4 no gradient MFMAs
#endif
// Kept from the round-2..5 experiments (each measured on one box against the build without it,
// DESIGN.md "Spectral kernels"; the variants that were not kept are in the git history):
//  - the second-dispatched half (waves 4-7) runs at s_setprio 1;
//  - the gradient GEMM issues the next tile's operand reads before this tile's MFMAs, and the next
//    sample's pieces of tile q + 1 at tile q (as soon as those reads have landed);
//  - the per-sample bookkeeping (dA2 / dC2 / bias / loss / y_hat, tail-row sums) on a second-half
//    wave (SL_BKW), off the first half's critical path;
//  - split kernels: the tail column's dwords go out through the sample's buffer descriptor (all 64
//    lanes, lanes past the Dt tail rows masked by an out-of-range offset) right after the wave's
//    pieces of the tiles that hold its tail rows (their 128-B lines are then on their way into L2);
//  - the epilogue's table reads carry no per-element lane masks (see tab8).
#ifndef TR_SLICE_PROFILE
#define TR_SLICE_PROFILE 0  // profiling build: per-phase cycle counts of wave 0 of workgroups 0..255
#endif

namespace tr {

#if TR_SLICE_PROFILE
__device__ unsigned long long g_slice_prof[256][8][8];  // [workgroup][wave][phase]
#define SL_MARK(ph)                                                  \
  do {                                                               \
    const unsigned long long _now = __builtin_readcyclecounter();    \
    prof[ph] += _now - prof_t;                                       \
    prof_t = _now;                                                   \
  } while (0)
#define SL_SUB_BEGIN() const unsigned long long _w0 = __builtin_readcyclecounter()
#define SL_SUB_END(ph) prof[ph] += __builtin_readcyclecounter() - _w0
#else
#define SL_MARK(ph) \
  do {              \
  } while (0)
#define SL_SUB_BEGIN() \
  do {                 \
  } while (0)
#define SL_SUB_END(ph) \
  do {                 \
  } while (0)
#endif

namespace {
typedef float sl_f4 __attribute__((ext_vector_type(4)));
typedef float sl_f2 __attribute__((ext_vector_type(2)));
constexpr int SL_NW = 8;
constexpr int SL_T = SL_NW * TR_WAVE;
constexpr int SL_ROWS = 128;            // max w rows per wave (W / 2)
constexpr int SL_SLICE = SL_ROWS * 32;  // floats of one wave's slice
constexpr int SL_STEPS = SL_ROWS / 4;   // forward k steps per wave
constexpr int SL_TILES = SL_ROWS / 16;  // gradient w tiles per wave
constexpr int SL_TAIL = 64;             // tail floats per wave (Dt <= 2 rows x <= 32 w)
constexpr int SL_BKW = 4;               // the bookkeeping wave (a second-half wave)
// fixed part of the LDS carve (floats): slices, tails, exchange, tail partials, column partials;
// compile-time in the kernel (held as run-time values they took scalar registers the sample loop
// spilled); spec_slice_geom lays the same carve out
constexpr int SL_O_TAIL = SL_NW * SL_SLICE;
constexpr int SL_O_EX = SL_O_TAIL + SL_NW * SL_TAIL;
constexpr int SL_O_TP = SL_O_EX + SL_NW * 64 * 8;
constexpr int SL_O_PART = SL_O_TP + SL_NW * 64;
constexpr int SL_O_N1 = SL_O_PART + SL_NW * 32;
static_assert(SL_O_TP % 8 == 0 && SL_O_PART % 8 == 0, "the per-wave partial rows are read as two 16-B words");

// the eight waves' partials of one slot, stored side by side: two independent 16-B reads (one
// LDS round trip, not eight dependent ones), summed in wave order from 0 like the running sums
// they replace
__device__ __forceinline__ float sl_sum8(const float* p) {
  typedef float f4_t __attribute__((ext_vector_type(4)));
  const f4_t a = *reinterpret_cast<const f4_t*>(p), b = *reinterpret_cast<const f4_t*>(p + 4);
  float s = 0.f;
  s += a[0];
  s += a[1];
  s += a[2];
  s += a[3];
  s += b[0];
  s += b[1];
  s += b[2];
  s += b[3];
  return s;
}
__device__ __forceinline__ sl_f4 sl_mfma(float a, float b, sl_f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- round-to-nearest bf16 split (SP > 0) --------------------------------------------------
// x = x1 + x2 + x3 by round-to-nearest-even bf16 conversions (v_cvt_pk_bf16_f32, two values per
// instruction): x1 = bf16(x), r = x - x1 (exact: Sterbenz), x2 = bf16(r), x3 = r - x2 (exact, at
// most 8 significant bits: exactly a bf16), for every finite |x| below the bf16 overflow
// threshold (3.39e38) and above 2^-100.  |x2| <= 2^-8 |x|, |x3| <= 2^-17 |x|, and — unlike a
// truncating split, whose pieces all carry the sign of x — the pieces' signs are independent of
// x.  The factor side (Phi0 fragments, dT) is always split in three.  The sample side X is split
// in two by default (SL_XP(SP) == 2: x1 + x2, |x - x1 - x2| < 2^-16 |x|, measured maximum 2^-17.0,
// median 2^-19.4, unbiased) and a product x.f is formed as the five cross terms x1f1, x1f2, x2f1,
// x1f3, x2f2; with TR_SLICE_XPIECES=3 (SP 3, 4) X is split in three as well and the six terms of
// weight >= 2^-17 are formed (x3f1 added), the dropped x2f3 + x3f2 + x3f3 weighing < 2^-24 |xf|
// (measured maximum 2^-24.3, median 2^-29).  Every term is an exact bf16 x bf16 product in the
// fp32 accumulator of v_mfma_f32_16x16x32_bf16 (16x the f32 MFMA rate).  At full config-5 size
// the default form's gradients lie within 3.5e-7 of fp64 (the reference's own fp32 op sequence:
// 0.6-4.2e-6; a truncating split's dropped terms are biased toward the sign of the product, and
// over config 5's sums that bias reached 8-25x the f32 MFMA form's error).
// tests/test_split_numerics.py holds these bounds, tests/test_gpu_fullsize.py the full-size errors.
typedef __bf16 sl_bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 sl_bf2 __attribute__((ext_vector_type(2)));
typedef uint32_t sl_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ sl_f4 sl_mfma_bf(sl_u4 a, sl_u4 b, sl_f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sl_bf8, a), __builtin_bit_cast(sl_bf8, b), c, 0,
                                                 0, 0);
}
// two values -> one VGPR of packed RNE bf16 (element 0 = a in the low half), v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t sl_pack_rne(float a, float b) {
  return __builtin_bit_cast(uint32_t, sl_bf2{(__bf16)a, (__bf16)b});
}
// the two halves of a packed pair back as fp32 values (the low half by a byte permute: a shift of
// the packed word lets the compiler re-convert that value alone, one more cvt per pair)
__device__ __forceinline__ float sl_lo_f32(uint32_t h) { return __uint_as_float(__builtin_amdgcn_perm(h, h, 0x01000c0cu)); }
__device__ __forceinline__ float sl_hi_f32(uint32_t h) { return __uint_as_float(h & 0xffff0000u); }
// split a (element 2m) and b (element 2m+1) into the three packed bf16 pairs of VGPR m
#ifndef TR_SLICE_SPLITMODE
#define TR_SLICE_SPLITMODE 2  // 2: x1, x2, x3 all by round-to-nearest (above); 1: x1 truncated, x2 / x3 by
                              // round-to-nearest (unbiased too, dropped terms < 2^-22 |ab|); 0: all
                              // truncated (round 3: dropped terms biased toward the sign of ab)
#endif
__device__ __forceinline__ void sl_split2(float a, float b, uint32_t& h1, uint32_t& h2, uint32_t& h3) {
  float ra, rb;
  if (TR_SLICE_SPLITMODE == 2) {
    h1 = sl_pack_rne(a, b);
    ra = a - sl_lo_f32(h1);
    rb = b - sl_hi_f32(h1);
  } else {
    const uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
    h1 = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
    ra = a - __uint_as_float(ua & 0xffff0000u);
    rb = b - __uint_as_float(ub & 0xffff0000u);
  }
  if (TR_SLICE_SPLITMODE == 0) {
    const uint32_t ura = __float_as_uint(ra), urb = __float_as_uint(rb);
    h2 = __builtin_amdgcn_perm(urb, ura, 0x07060302u);
    const float sa = ra - __uint_as_float(ura & 0xffff0000u), sb = rb - __uint_as_float(urb & 0xffff0000u);
    h3 = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
    return;
  }
  h2 = sl_pack_rne(ra, rb);
  const float sa = ra - sl_lo_f32(h2), sb = rb - sl_hi_f32(h2);
  h3 = sl_pack_rne(sa, sb);
}
__device__ __forceinline__ void sl_split_m(float a, float b, sl_u4 (&f)[3], int m) {
  uint32_t h1, h2, h3;
  sl_split2(a, b, h1, h2, h3);
  f[0][m] = h1;
  f[1][m] = h2;
  f[2][m] = h3;
}
// X side (the first operand at every call site: the sample data) in XP pieces.  XP = 2 (the
// default): x = x1 + x2 + e by two round-to-nearest bf16 conversions, |e| < 2^-16 |x| (measured
// maximum 2^-17.0, median 2^-19.4) with no
// bias (e's sign is independent of x's); five MFMAs per product of the six-term form and three
// of the packed-lin form, 6 VALU per pair of values instead of 11.  XP = 3: the three-piece split
// above, x represented exactly.  Measured at full config-5 size against an fp64 closed form
// (tests/test_gpu_fullsize.py), both forms' gradients sit within 1.7-3.5e-7 normwise, the f32
// MFMA form's within 1.1e-7 and the reference's own fp32 op sequence on the CPU within 0.6-4.2e-6.
template <int XP>
__device__ __forceinline__ void sl_splitx_m(float a, float b, sl_u4 (&f)[3], int m) {
  if constexpr (XP == 2) {
    const uint32_t h1 = sl_pack_rne(a, b);
    f[0][m] = h1;
    f[1][m] = sl_pack_rne(a - sl_lo_f32(h1), b - sl_hi_f32(h1));
  } else {
    sl_split_m(a, b, f, m);
  }
}
// c += A.B over the six cross terms of weight >= 2^-17 (A in XP pieces, B in three)
template <int XP>
__device__ __forceinline__ sl_f4 sl_mfma6(const sl_u4 (&a)[3], const sl_u4 (&b)[3], sl_f4 c) {
  if constexpr (XP == 3) c = sl_mfma_bf(a[2], b[0], c);
  c = sl_mfma_bf(a[1], b[1], c);
  c = sl_mfma_bf(a[0], b[2], c);
  c = sl_mfma_bf(a[1], b[0], c);
  c = sl_mfma_bf(a[0], b[1], c);
  c = sl_mfma_bf(a[0], b[0], c);
  return c;
}
// packed lin columns (Rn <= 8): B = [b1 | b2] (lanes 0-7 | 8-15) and [b3 | 0]; column c of the
// product is the sum of accumulator columns c and c + 8 (folded by sl_fold8): four MFMAs for
// the six cross terms (a3b2 comes along), three with a two-piece A
template <int XP>
__device__ __forceinline__ sl_f4 sl_mfma_lp(const sl_u4 (&a)[3], const sl_u4 (&b)[2], sl_f4 c) {
  if constexpr (XP == 3) c = sl_mfma_bf(a[2], b[0], c);
  c = sl_mfma_bf(a[0], b[1], c);
  c = sl_mfma_bf(a[1], b[0], c);
  c = sl_mfma_bf(a[0], b[0], c);
  return c;
}
// SP (the kernel's GEMM form): 0 f32 MFMA; 1 / 2 bf16 split with a two-piece X, lin columns
// packed (Rn <= 8) / not; 3 / 4 the same with the three-piece X
// SP 5 / 6 (signed X, the plan's choice from X's range, tr_plan_set_x_range): the forward's X in
// three pieces (T = X Phi0 cancels on signed samples, and the norms of T amplify its error) and
// the gradient's in two.  Forms 3-6 (with tail rows) form the gradient GEMM's products of each
// sample in a zero accumulator, added to the launch-long one by a VALU add: the bf16 MFMA's
// accumulation truncates small addends toward the accumulator, a sign-dependent bias over a
// workgroup's 128 samples.  Measured at full config-5 size against fp64 (worst gradient, signed X
// / |X|; gpurun_out/r06a, r06b): SP 1 2.8e-6 / 3.5e-7; forward three-piece alone 1.6e-6; SP 5
// 8.6e-7 / 9.4e-8; SP 3 with the accumulators 5.5e-7 / 8.2e-8 (without: 1.8e-6 / 3.3e-7); the
// reference's own fp32 2.4e-6 / 2.1e-6.  Kernel time at c5: SP 5 +13 %, SP 3 +20 % over SP 1;
// |X| (spectral magnitudes, bench.py c5) keeps SP 1.
#ifndef TR_SLICE_ACCUM
#define TR_SLICE_ACCUM 1  // 0: no per-sample accumulators (the negative-control build, Makefile negctl)
#endif
#define SL_LP(SP) ((SP) == 1 || (SP) == 3 || (SP) == 5)
#define SL_XP(SP) ((SP) == 3 || (SP) == 4 ? 3 : 2)   // gradient GEMM
#define SL_XPF(SP) ((SP) >= 3 ? 3 : 2)               // forward GEMM
// per-sample gradient accumulators: forms 3-6 with tail rows (without them, D <= 128, the
// accumulator temporaries push the kernel past 256 VGPRs into scratch)
#define SL_ACC(SP, DT) (TR_SLICE_ACCUM && (SP) >= 3 && (DT) > 0)
template <int CTRL>
__device__ __forceinline__ float sl_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// 16-lane row sum (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror): every lane of
// the row ends with the bitwise-identical value
__device__ __forceinline__ float sl_row_sum16(float v) {
  v += sl_dpp<0xB1>(v);
  v += sl_dpp<0x4E>(v);
  v += sl_dpp<0x141>(v);
  v += sl_dpp<0x140>(v);
  return v;
}
// xor-16 / xor-32 butterfly steps by v_permlane16/32_swap (no LDS round trip)
__device__ __forceinline__ float sl_xor16(float v) {
  const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ float sl_xor32(float v) {
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ float sl_groups_sum(float v) { return sl_xor32(sl_xor16(v)); }
// lanes i and i ^ 8 of each 16-lane row summed (row_ror:8); both end with the same value
__device__ __forceinline__ float sl_fold8(float v) { return v + sl_dpp<0x128>(v); }
// barrier that leaves LDS-DMA in flight (__syncthreads() would wait vmcnt(0))
__device__ __forceinline__ void sl_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ uint32_t sl_lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}
// sl_dma16b with soffset = tstr * q and the LDS address lds_b + lds_off formed by the statement
// itself from a base and constants (formed outside, the compiler hoisted all sixteen out of the
// sample loop into SGPRs the kernel does not have: one spill reload per piece)
__device__ __forceinline__ void sl_dma16bq(__amdgpu_buffer_rsrc_t rs, uint32_t tstr, uint32_t q, uint32_t voff,
                                           uint32_t lds_b, uint32_t lds_off) {
  uint32_t keep, so;
  asm volatile("s_mul_i32 %1, %4, %5\n\ts_mov_b32 %0, m0\n\ts_add_u32 m0, %3, %7\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %6, %1 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep), "=&s"(so)
               : "v"(voff), "s"(lds_b), "s"(tstr), "s"(q), "s"(rs), "s"(lds_off)
               : "memory", "scc");
}
// one 4-B LDS-DMA piece per lane: gsrc -> LDS byte address m0 + 4 * lane (m0 saved / restored)
__device__ __forceinline__ void sl_dma4(const float* gsrc, const float* lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(sl_lds_addr(lds_dst)))
               : "memory");
}
// one 16-B LDS-DMA piece per lane: gsrc (4-B aligned is enough) -> LDS byte address m0 + 16 * lane
__device__ __forceinline__ void sl_dma16(const float* gsrc, const float* lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(sl_lds_addr(lds_dst)))
               : "memory");
}
// one 16-B LDS-DMA piece per lane through a buffer descriptor: rsrc base + soff + voff (lane) -> LDS
// byte address m0 + 16 * lane; no per-lane 64-bit address arithmetic at the call
// (lds_b: the destination's LDS byte address, wave-uniform: formed from a 32-bit base and a
// compile-time offset, no generic-pointer cast with its null check at every piece)
// one dword per lane from buffer byte offset voff into LDS (lane L -> lds_b + 4 L); an offset past
// the descriptor's range reads 0
__device__ __forceinline__ void sl_dma4b(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_b) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(lds_b)
               : "memory");
}
__device__ __forceinline__ void sl_dma16b(__amdgpu_buffer_rsrc_t rs, uint32_t soff, uint32_t voff, uint32_t lds_b) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(lds_b), "s"(soff)
               : "memory");
}
// s_waitcnt vmcnt(n), n wave-uniform in [0, 63]
__device__ __forceinline__ void sl_wait_vm(int n) {
#define SL_VM(k) \
  case k:        \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
#define SL_VM8(b) SL_VM(b) SL_VM(b + 1) SL_VM(b + 2) SL_VM(b + 3) SL_VM(b + 4) SL_VM(b + 5) SL_VM(b + 6) SL_VM(b + 7)
  switch (n < 0 ? 0 : n) {
    SL_VM8(0) SL_VM8(8) SL_VM8(16) SL_VM8(24) SL_VM8(32) SL_VM8(40) SL_VM8(48) SL_VM8(56)
    default:
      asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  }
#undef SL_VM8
#undef SL_VM
}
// this lane's index recomputed where it is used (v_mbcnt, not a register held across the sample
// loop: at 256 VGPRs the compiler spilled the held lane index, and each reload's vmcnt(0) wait
// drained the in-flight LDS-DMA of the next sample); volatile, so it is neither hoisted nor shared
__device__ __forceinline__ int sl_lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// slot xor of chunk r (x = r & 7: bit 0 -> bit 0, bit 1 -> bit 2)
__device__ __forceinline__ int sl_swz(int x) { return (x & 1) | ((x & 2) << 1); }
}  // namespace

// SP: 0 = both GEMMs on v_mfma_f32_16x16x4_f32; 1 = bf16 split on v_mfma_f32_16x16x32_bf16 (X in
// two pieces) with the lin columns packed (Rn <= 8); 2 = the same, lin unpacked; 3 / 4 = X in three
// pieces (TR_SLICE_XPIECES=3), lin packed / unpacked
template <int CC, int DT, int SP>
__global__ __launch_bounds__(SL_T) void k_spec_slice(
    const float* __restrict__ X, int64_t N, int64_t xld, SpecGeom g, const float* __restrict__ phi,
    const float* __restrict__ Phi0, const float* __restrict__ wts, const float* __restrict__ y, float scale,
    float* __restrict__ slab, int64_t slab_stride, double* __restrict__ dpart, float* __restrict__ out,
    int64_t rows_per_wg, int reverse, const int32_t* __restrict__ stop) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (stop != nullptr && *stop != 0) return;
  const int t = threadIdx.x;
  const int lane = t & (TR_WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(t / TR_WAVE);
  const int p = wv & 3, hw = wv >> 2;
  const int i = lane & 15, gq = lane >> 4;
  const int D = g.D, K = g.K, Rn = g.Rn, Rs = g.Rs, NO = g.NO;
  const int RC = Rs * CC;
  constexpr int WH = SL_ROWS, ntl = SL_TILES;  // W = 256 (the shapes this kernel is built for)
  constexpr int Dt = DT;
  constexpr int TR = WH / 4;   // tail rows of this wave: w offsets [TR p, TR (p + 1)) of its half
  constexpr int TQ = TR / 16;  // ... = gradient tiles [TQ p, TQ (p + 1))
  constexpr int SQ = TR / 4;   // ... = forward steps [SQ p, SQ (p + 1))
  const int wbase = hw * WH;   // first w of this wave's half
  const int dbase = 32 * p;    // first d of this wave's pair

  float* slice = lds + wv * SL_SLICE;
  const uint32_t slice_b = (uint32_t)__builtin_amdgcn_readfirstlane(sl_lds_addr(slice));  // its LDS byte address
  float* sTail = lds + SL_O_TAIL + wv * SL_TAIL;  // [Dt][TR]
  const uint32_t tail_b = (uint32_t)__builtin_amdgcn_readfirstlane(sl_lds_addr(sTail));
  float* sEx = lds + SL_O_EX;                      // [8 waves][64 lanes][8]
  float* sTP = lds + SL_O_TP;                      // [2 rows][32 columns][8 waves]
  float* sPart = lds + SL_O_PART;                  // [Z 16 | V 16][8 waves]
  const int Dp = g.sl_Dp;                           // table row length (>= max(D, 128), % 4 == 0)
  float* sN1 = lds + SL_O_N1;                       // [Rn][Dp] phi(A1)^T (d contiguous: b128 reads)
  float* sC1 = sN1 + Dp * Rn;                       // [Rs][Dp] phi(C1)^T
  float* sCA = sC1 + g.sl_Dp * Rs;                  // [NO][16] w_r phi(A2)
  float* sCC = sCA + NO * 16;                       // [NO][16] phi(C2)
  float* sB = sCC + NO * 16;                        // [NO] bias
  float* sWt = sB + NO;                             // [16] w_r
  float* sAcc = sWt + 16;                           // [NO*Rn] dA2 | [NO*Rs] dC2 | [NO] dbias
  float* sTacc = sAcc + NO * (Rn + Rs + 1);         // bookkeeping wave: [Dt][dPhi(A1) 16 | dPhi(C1) 16] of rows 128+
  double* sLoss = reinterpret_cast<double*>(lds + g.sl_oLoss);  // bookkeeping wave lane 0: sum of squared errors

  for (int e = SL_O_TAIL + t; e < g.sl_lds_floats; e += SL_T) lds[e] = 0.f;
  __syncthreads();
  for (int e = t; e < D * Rn; e += SL_T) sN1[(e % Rn) * Dp + e / Rn] = phi[g.offA1 + e];
  for (int e = t; e < D * Rs; e += SL_T) sC1[(e % Rs) * Dp + e / Rs] = phi[g.offC1 + e];
  for (int e = t; e < NO * 16; e += SL_T) {
    const int o = e >> 4, r = e & 15;
    if (r < Rn) sCA[e] = wts[r] * phi[g.offA2 + o * Rn + r];
    if (r < Rs) sCC[e] = phi[g.offC2 + o * Rs + r];
  }
  for (int e = t; e < NO; e += SL_T) sB[e] = phi[g.offB + e];
  if (t < Rn) sWt[t] = wts[t];

  // B fragments: lane (i, gq) of step s holds Phi0[wbase + 4 s + gq, column]; tile 0 column i is
  // spectral column i (Phi0 column Rn + i), tile 1 column i is lin column i
  constexpr int NS = SP ? 1 : SL_STEPS;
  float bf0[NS], bf1[NS];
  // split mode: k step S covers steps 8S .. 8S+7 (element j of lane group gq <-> w = 32 S + 4 j
  // + gq of the half, the same w for A and B); bs = spectral columns, bl = lin columns
  constexpr int NSP = SP ? SL_STEPS / 8 : 1;
  constexpr int NL = SL_LP(SP) ? 2 : 3;
  sl_u4 bs[NSP][3], bl[NSP][NL];
  if constexpr (!SP) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int64_t w = wbase + 4 * s + gq;
      bf0[s] = (i < RC && w < g.W) ? Phi0[w * K + Rn + i] : 0.f;  // rows past W: padding (zero X)
      bf1[s] = (i < Rn && w < g.W) ? Phi0[w * K + i] : 0.f;
    }
  } else {
    const int cl = SL_LP(SP) ? (i & 7) : i;  // lin column this lane splits
#pragma unroll
    for (int S = 0; S < NSP; ++S)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t w0 = wbase + 4 * (8 * S + 2 * m) + gq, w1 = w0 + 4;
        const bool ok0 = w0 < g.W, ok1 = w1 < g.W;  // rows past W: padding (zero X)
        sl_split_m((i < RC && ok0) ? Phi0[w0 * K + Rn + i] : 0.f, (i < RC && ok1) ? Phi0[w1 * K + Rn + i] : 0.f, bs[S],
                   m);
        uint32_t h1, h2, h3;
        sl_split2((cl < Rn && ok0) ? Phi0[w0 * K + cl] : 0.f, (cl < Rn && ok1) ? Phi0[w1 * K + cl] : 0.f, h1, h2, h3);
        if constexpr (SL_LP(SP)) {
          bl[S][0][m] = i < 8 ? h1 : h2;
          bl[S][1][m] = i < 8 ? h3 : 0u;
        } else {
          bl[S][0][m] = h1;
          bl[S][1][m] = h2;
          bl[S][NL - 1][m] = h3;
        }
      }
  }
  sl_f4 gacc[SL_TILES][2];
#pragma unroll
  for (int q = 0; q < SL_TILES; ++q) {
    gacc[q][0] = sl_f4{0.f, 0.f, 0.f, 0.f};
    gacc[q][1] = sl_f4{0.f, 0.f, 0.f, 0.f};
  }
  float an1[2][4], as1[4];  // dPhi(A1) partial (both d tiles), dPhi(C1) (own tile h = hw)
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    an1[0][v] = an1[1][v] = 0.f;
    as1[v] = 0.f;
  }
  const float bm = (float)((Rn > 0) + (Rs > 0));  // the bias is added by both terms (Q10)

  // per-lane LDS offsets (floats) of the forward operand (step s: + 128 s, period 4 in the
  // swizzle) and of the two gradient operand reads (tile q: + 512 q); formed from a fresh lane
  // index at the phase that uses them (held across the sample loop they took registers the
  // split GEMMs need)
  auto fo_of = [](int L, int s) {
    const int i = L & 15, gq = L >> 4, r = 2 * s + (gq >> 1);
    return 64 * (gq >> 1) + 4 * (((i >> 1) + 8 * (gq & 1)) ^ sl_swz(r)) + 2 * (i & 1);
  };
  auto bo_of = [](int L, int c) {
    const int i = L & 15, gq = L >> 4;
    return 64 * (i >> 1) + 4 * ((2 * gq + c + 8 * (i & 1)) ^ sl_swz(i >> 1));
  };

  const int64_t n0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t n1 = n0 + rows_per_wg < N ? n0 + rows_per_wg : N;
  const int64_t nr = n1 > n0 ? n1 - n0 : 0;
  auto sample_of = [&](int64_t k) -> int64_t { return reverse ? (n1 - 1 - k) : (n0 + k); };

  // LDS-DMA of gradient tile q (rows 16q..16q+15 = chunks 8q..8q+7) of this wave's slice of
  // sample n: two 16-B-per-lane pieces of 4 chunks; lane L fills slot L%16 of chunk 4c4 + L/16,
  // i.e. row 2r + (slot'>>3), columns 4 (slot' & 7) .. +3 with slot' = (L%16) ^ swz(r & 7).
  // (global_load_lds_dwordx4 takes 4-B aligned sources; one dword piece per lane costs the
  // memory pipeline as much as a dwordx4 one: ~3 vs ~6.8 TB/s chip-wide, tools/ldsdma_probe.hip.)
  // The per-lane offsets are recomputed from an opaque copy of the lane index at every call:
  // hoisted out of the sample loop they would hold 16 address registers.
  // The lane part of a piece's source is the same for every tile and sample: two byte offsets
  // (c4 = 0, 1) held for the launch; the sample base goes into a buffer descriptor (SGPRs) and
  // the tile's row offset into soffset, so a piece costs no per-lane address arithmetic.
  auto dvo_of = [&](int L, int c4) {
    const int lsl = L & 15, lc = L >> 4;
    const int x = 4 * c4 + lc;  // chunk within the tile (= r & 7)
    const int sp = lsl ^ sl_swz(x);
    int d = dbase + 4 * (sp & 7);
    d = d < D ? d : 0;  // a column quad past D (D < 128): any valid quad, times zero factor rows; a
                        // quad straddling D reads the next row's first values (zeros past the
                        // sample, the descriptor's range), times zero rows as well
    return (uint32_t)(((2 * x + (sp >> 3)) * D + d) * 4);
  };
  uint32_t dvo[2];  // (set by the phase that issues pieces)
  auto set_dvo = [&]() {
    const int L = sl_lane_now();
    dvo[0] = dvo_of(L, 0);
    dvo[1] = dvo_of(L, 1);
  };
  // the descriptor starts at this wave's half of the sample (row wbase); tile q's rows are at
  // soffset q * tstr, formed inside the piece's statement (hoisted out of the sample loop, the
  // eight tile offsets took SGPRs the kernel does not have: one spill reload per piece)
  // (W < 256: the rows past W read zeros, the descriptor's range; a half wholly past W has none)
  const uint32_t hbytes = (uint32_t)((g.W > wbase ? g.W - wbase : 0) * D * 4), tstr = (uint32_t)(64 * D);
  auto rsrc_of = [&](int64_t n) {
    const uint64_t a = (uint64_t)(uintptr_t)(X + n * xld + (int64_t)wbase * D);
    const uint64_t au = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)au, (short)0, (int)hbytes, 0x00020000);
  };
  auto dma_piece_r = [&](__amdgpu_buffer_rsrc_t rs, int q, int c4) {  // chunks 8q + 4c4 .. +3
    sl_dma16bq(rs, tstr, (uint32_t)q, dvo[c4], slice_b, 256u * (uint32_t)(8 * q + 4 * c4));
  };
  auto dma_piece = [&](int64_t n, int q, int c4) { dma_piece_r(rsrc_of(n), q, c4); };
  auto dma_tile = [&](int64_t n, int q) {
    dma_piece(n, q, 0);
    dma_piece(n, q, 1);
  };
  auto dma_tail = [&](int64_t n) {
    const int ln = sl_lane_now();  // the per-lane source is formed at the call (no live address pair)
    if (SP) {
      // through the sample's descriptor, all 64 lanes: lane -> (row 128 + lane / TR, w offset
      // lane % TR) as below; lanes with lane / TR >= Dt take an out-of-range offset (no request:
      // each active lane's dword is a line of its own in the memory pipeline)
      const int tr = ln / TR, wo = ln - tr * TR;
      const uint32_t off = (uint32_t)(((TR * p + wo) * D + 128 + tr) * 4);
      sl_dma4b(rsrc_of(n), tr >= Dt ? 0xFFFFFF00u : off, tail_b);
    } else if (ln < Dt * TR) {  // lane -> (row 128 + lane / TR, w offset lane % TR)
      const int tr = ln / TR, wo = ln - tr * TR;
      const int64_t w = wbase + TR * p + wo;
      sl_dma4(X + n * xld + (w < g.W ? w : 0) * D + 128 + tr, sTail);  // (rows past W: any valid row, times zero)
    }
  };
  // split kernels: wave p's tail goes out right after its pieces of tile qt = TQ p + TQ - 1 (the
  // tiles holding its tail rows, whose 128-B lines the pair waves 0 / 3 fetch at the same stage;
  // the forward's wait for tile q + 1 counts the tail only while q + 1 <= qt); the f32 form issues
  // it first (waiting for tile 0 also retires it: it reads the tail inside the loop)
  constexpr bool TAIL_LAST = SP;
  constexpr int NTL = (TAIL_LAST && Dt > 0) ? 1 : 0;  // tail pieces issued after tile pieces
  const int qt = !TAIL_LAST ? SL_TILES - 1 : TQ * p + TQ - 1;
  auto dma_sample = [&](int64_t n) {
    if (Dt > 0 && !TAIL_LAST) dma_tail(n);
#pragma unroll
    for (int q = 0; q < SL_TILES; ++q) {
      dma_tile(n, q);
      if (Dt > 0 && TAIL_LAST && q == qt) dma_tail(n);
    }
  };

  __builtin_amdgcn_s_waitcnt(0);  // retire the prologue's loads (the loop's waits are counted)
  __syncthreads();
  set_dvo();
  if (nr > 0) dma_sample(sample_of(0));
  if (hw == 1) __builtin_amdgcn_s_setprio(1);
#if TR_SLICE_PROFILE
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long prof_t = __builtin_readcyclecounter();
#endif

#pragma unroll 1
  for (int64_t k = 0; k < nr; ++k) {
    const int64_t n = sample_of(k);
    const bool has_next = k + 1 < nr && !((TR_SLICE_SKIP & 1) && k > 0);
    const int64_t nn = has_next ? sample_of(k + 1) : n;

    // ---- forward: T (tile jt, d tile h) over this wave's half ---------------------------
    sl_f4 T00 = {0.f, 0.f, 0.f, 0.f}, T01 = T00, T10 = T00, T11 = T00;
    // tail rows d = 128 + tr: VALU partial over this wave's tail steps [SQ p, SQ (p + 1)) inside
    // the forward loop (bf0 / bf1 of the step are in hand), reduced over lane groups after it
    float ta[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    sl_f4 Tts = {0.f, 0.f, 0.f, 0.f}, Ttl = Tts;  // split mode: tail rows (row tr = lane group 0, reg tr)
    {
      sl_f2 xa[4], xb[4];
      sl_u4 xf[2][3];  // split mode: the k step's A fragments of d tiles 0 / 1
      int fo[4];
      {
        const int L = sl_lane_now();
#pragma unroll
        for (int s = 0; s < 4; ++s) fo[s] = fo_of(L, s);
      }
      {
        SL_SUB_BEGIN();
        sl_wait_vm((ntl - 1) * 2 + NTL);
        SL_SUB_END(1);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = *reinterpret_cast<const sl_f2*>(slice + 128 * s + fo[s]);
#pragma unroll
      for (int q = 0; q < SL_TILES; ++q) {
        if (q + 1 < ntl) {
          {
            SL_SUB_BEGIN();
            sl_wait_vm((ntl - 2 - q) * 2 + (q + 1 <= qt ? NTL : 0));
            SL_SUB_END(1);
          }
#pragma unroll
          for (int s = 0; s < 4; ++s)
            xb[s] = *reinterpret_cast<const sl_f2*>(slice + 128 * (4 * (q + 1) + s) + fo[s]);
        }
        if constexpr (!SP) {
#pragma unroll
          for (int s = 0; s < 4 && !(TR_SLICE_SKIP & 2); ++s) {
            T00 = sl_mfma(xa[s].x, bf0[4 * q + s], T00);
            T01 = sl_mfma(xa[s].y, bf0[4 * q + s], T01);
            T10 = sl_mfma(xa[s].x, bf1[4 * q + s], T10);
            T11 = sl_mfma(xa[s].y, bf1[4 * q + s], T11);
          }
        } else {
          // tile q holds elements 4 (q & 1) .. +3 of k step q / 2: VGPRs 2 (q & 1), 2 (q & 1) + 1
#pragma unroll
          for (int mm = 0; mm < 2; ++mm) {
            sl_splitx_m<SL_XPF(SP)>(xa[2 * mm].x, xa[2 * mm + 1].x, xf[0], 2 * (q & 1) + mm);
            sl_splitx_m<SL_XPF(SP)>(xa[2 * mm].y, xa[2 * mm + 1].y, xf[1], 2 * (q & 1) + mm);
          }
          if ((q & 1) && !(TR_SLICE_SKIP & 2)) {
            const int S = q >> 1;
            T00 = sl_mfma6<SL_XPF(SP)>(xf[0], bs[S], T00);
            T01 = sl_mfma6<SL_XPF(SP)>(xf[1], bs[S], T01);
            if constexpr (SL_LP(SP)) {
              T10 = sl_mfma_lp<SL_XPF(SP)>(xf[0], bl[S], T10);
              T11 = sl_mfma_lp<SL_XPF(SP)>(xf[1], bl[S], T11);
            } else {
              T10 = sl_mfma6<SL_XPF(SP)>(xf[0], bl[S], T10);
              T11 = sl_mfma6<SL_XPF(SP)>(xf[1], bl[S], T11);
            }
          }
        }
        if constexpr (!SP) {
          if (Dt > 0 && q / TQ == p) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int wo = 4 * (4 * q + s - SQ * p) + gq;
#pragma unroll
              for (int tr = 0; tr < Dt; ++tr) {
                const float xt = sTail[tr * TR + wo];
                ta[tr][0] = fmaf(xt, bf0[4 * q + s], ta[tr][0]);
                ta[tr][1] = fmaf(xt, bf1[4 * q + s], ta[tr][1]);
              }
            }
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) xa[s] = xb[s];
      }
    }
    // y of the first two outputs by scalar loads issued here: their latency hides under the
    // exchange, barrier A and the column partials (issued inside the output loop it was exposed;
    // issued before the forward, an SMEM load in flight turns its counted LDS waits into lgkmcnt(0))
    const float y0 = y[n * NO], y1 = NO > 1 ? y[n * NO + 1] : 0.f;
    // lane-dependent indices of the epilogue from an opaque copy of the lane index: every LDS
    // address below is then formed here (a few VALU ops) instead of living across the loop
    // (held through the GEMMs, the split kernels spilled them to scratch: a vmcnt(0) reload each)
    const int lk = sl_lane_now();
    const int i = lk & 15, gq = lk >> 4;
    const int rs = i / CC;
    const bool rs_ok = rs < Rs;
    const bool vlane = rs_ok && (i % CC) == 0;
    if constexpr (SL_LP(SP)) {  // packed lin columns: column c = accumulator columns c + (c ^ 8)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        T10[v] = sl_fold8(T10[v]);
        T11[v] = sl_fold8(T11[v]);
      }
    }
    if constexpr (SP) {
      if (Dt > 0) {
        // tail rows d = 128 + tr over this wave's tail k step (S = p): A row i = tail row i
        // (rows >= Dt zero), element j <-> w offset 4 j + gq of the wave's 32 tail w (after the
        // loop: nothing of the forward is live; one case per static S)
        sl_u4 tf[3];
        if (NTL) sl_wait_vm(0);  // the tail (issued after the tiles) has landed
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const float x0 = i < Dt ? sTail[i * TR + 8 * m + gq] : 0.f;
          const float x1 = i < Dt ? sTail[i * TR + 8 * m + 4 + gq] : 0.f;
          sl_splitx_m<SL_XPF(SP)>(x0, x1, tf, m);
        }
        auto tail_step = [&](const sl_u4(&b_s)[3], const sl_u4(&b_l)[NL]) {
          Tts = sl_mfma6<SL_XPF(SP)>(tf, b_s, Tts);
          if constexpr (SL_LP(SP))
            Ttl = sl_mfma_lp<SL_XPF(SP)>(tf, b_l, Ttl);
          else
            Ttl = sl_mfma6<SL_XPF(SP)>(tf, b_l, Ttl);
        };
        switch (p) {
          case 0: tail_step(bs[0], bl[0]); break;
          case 1: tail_step(bs[1], bl[1]); break;
          case 2: tail_step(bs[2], bl[2]); break;
          default: tail_step(bs[3], bl[3]); break;
        }
      }
    }
    if (Dt > 0) {
#pragma unroll
      for (int tr = 0; tr < Dt; ++tr) {
        if constexpr (SP) {
          ta[tr][0] = Tts[tr];
          ta[tr][1] = SL_LP(SP) ? sl_fold8(Ttl[tr]) : Ttl[tr];
        } else {
          ta[tr][0] = sl_groups_sum(ta[tr][0]);
          ta[tr][1] = sl_groups_sum(ta[tr][1]);
        }
        if (gq == 0) {
          sTP[(tr * 32 + i) * SL_NW + wv] = ta[tr][0];
          sTP[(tr * 32 + 16 + i) * SL_NW + wv] = ta[tr][1];
        }
      }
    }
    SL_MARK(0);
    // ---- exchange the spectral tiles with the partner half ---------------------------------
    *reinterpret_cast<sl_f4*>(sEx + (wv * TR_WAVE + lk) * 8) = T00;
    *reinterpret_cast<sl_f4*>(sEx + (wv * TR_WAVE + lk) * 8 + 4) = T01;
    SL_MARK(2);
    sl_barrier();
    SL_MARK(3);
    {
      const float* pe = sEx + ((wv ^ 4) * TR_WAVE + lk) * 8;
      T00 += *reinterpret_cast<const sl_f4*>(pe);  // two-term sums commute: both halves hold
      T01 += *reinterpret_cast<const sl_f4*>(pe + 4);  // the bitwise-identical full tile
    }
    // full tail row values: lane (i, gq < Dt) holds T[128 + gq][spectral i] / [lin i]
    float tt0 = 0.f, tt1 = 0.f;
    if (Dt > 0 && gq < Dt) {
      tt0 = sl_sum8(sTP + (gq * 32 + i) * SL_NW);
      tt1 = sl_sum8(sTP + (gq * 32 + 16 + i) * SL_NW);
    }

    // y of this sample, lane o (n_out <= 64); read by readlane after barrier B

    // ---- column partials: Z (lin, both d tiles, this half's partial T) and V (spectral, own d
    // tile h = hw, full T) -- nothing but the two sums stays live across barrier B -------------
    auto norm_of = [&](float x) {  // || T[d, spectral group of this lk] ||
      float sq = x * x;
      if (CC >= 2) sq += sl_dpp<0xB1>(sq);
      if (CC >= 4) sq += sl_dpp<0x4E>(sq);
      return __builtin_amdgcn_sqrtf(sq);
    };
    // table offsets from an opaque copy of the lane index: recomputed here (a few VALU ops)
    // instead of living across the sample loop as spilled registers
    const int lo = sl_lane_now();
    const int ie = lo & 15, ge = lo >> 4, rse = ie / CC;
    // phi(A1)[d, ie] / phi(C1)[d, ie / CC] of this lane's 8 rows d = dbase + 8 ge + 2v + h: two
    // ds_read_b128 each, element 2v + h
    const int n1o = (ie < Rn ? ie : 0) * Dp + dbase + 8 * ge, c1o = (rse < Rs ? rse : 0) * Dp + dbase + 8 * ge;
    // (no per-element lane masks; a lane past Rn / Rs reads table row 0, finite,
    // and meets zero factors: T columns past Rn are zero, and dz / dv are zeroed there, so only
    // the lin column partial needs one mask — the packed form's lanes 8-15 hold folded columns)
    auto tab8 = [&](const float* tb, int off, float (&o)[2][4]) {
      const sl_f4 lo = *reinterpret_cast<const sl_f4*>(tb + off), hi = *reinterpret_cast<const sl_f4*>(tb + off + 4);
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float x = v < 2 ? lo[2 * v + h] : hi[2 * (v - 2) + h];
          o[h][v] = x;
        }
    };
    float zp = 0.f, vp = 0.f;
    {
      float n1[2][4], c1[2][4];
      tab8(sN1, n1o, n1);
      tab8(sC1, c1o, c1);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int v = 0; v < 4; ++v) zp = fmaf(n1[h][v], h == 0 ? T10[v] : T11[v], zp);
#pragma unroll
      for (int v = 0; v < 4; ++v)
        vp = fmaf(hw == 0 ? c1[0][v] : c1[1][v], norm_of(hw == 0 ? T00[v] : T01[v]), vp);
    }
    vp = vlane ? vp : 0.f;
    zp = i < Rn ? zp : 0.f;
    const float Mt = norm_of(tt0);
    const int dtl = 128 + gq;  // tail row of this lk group (valid when gq < Dt)
    const float n1t = (Dt > 0 && gq < Dt && i < Rn) ? sN1[i * Dp + dtl] : 0.f;
    const float c1t = (Dt > 0 && gq < Dt && rs_ok) ? sC1[rs * Dp + dtl] : 0.f;
    zp = sl_groups_sum(zp);
    vp = sl_groups_sum(vp);
    if (wv == SL_BKW && Dt > 0) {  // the bookkeeping wave adds the tail rows' terms
      float zt = n1t * tt1;
      float vt = vlane ? c1t * Mt : 0.f;
      zp += sl_groups_sum(zt);
      vp += sl_groups_sum(vt);
    }
    if (gq == 0) {
      sPart[i * SL_NW + wv] = zp;
      if (vlane) sPart[(16 + rs) * SL_NW + wv] = vp;
    }
    SL_MARK(4);
    sl_barrier();
    SL_MARK(5);

    // ---- Z / V, y_hat, residual, dZ / dV (every wave, identical order) ----------------------
    float n1[2][4], c1[2][4];  // (issued first: their latency hides under the sums below)
    tab8(sN1, n1o, n1);
    tab8(sC1, c1o, c1);
    const float zi = sl_sum8(sPart + i * SL_NW), vi = sl_sum8(sPart + (16 + i) * SL_NW);
    float dz = 0.f, dv = 0.f;
    // output o with target yo: y_hat, residual, its dZ / dV terms, the bookkeeping wave's sums
    auto out_step = [&](int o, float yo) {
      const float ca = sCA[o * 16 + i], cc = sCC[o * 16 + i];
      const float pl = sl_row_sum16(ca * zi);
      const float ps = sl_row_sum16(cc * vi);
      const float b = sB[o];
      const float yh = (Rn > 0 ? pl + b : 0.f) + (Rs > 0 ? ps + b : 0.f);
      const float e = yh - yo;
      const float rv = e * scale;
      dz = fmaf(rv, ca, dz);
      dv = fmaf(rv, sCC[o * 16 + rs], dv);
      if (wv == SL_BKW && lk < 16) {
        if (i < Rn) sAcc[o * Rn + i] += sWt[i] * rv * zi;
        if (i < Rs) sAcc[NO * Rn + o * Rs + i] += rv * vi;
        if (lk == 0) {
          sAcc[NO * (Rn + Rs) + o] += bm * rv;
          *sLoss += (double)e * (double)e;
          if (out != nullptr) out[n * NO + o] = yh;
        }
      }
    };
    // y by scalar loads (a vector load's compiler-inserted vmcnt(0) would drain the in-flight
    // LDS-DMA); one or two outputs straight-line (their table reads and row sums overlap), more in
    // a loop
    if (NO == 2) {
      out_step(0, y0);
      out_step(1, y1);
    } else if (NO == 1) {
      out_step(0, y0);
    } else {
#pragma unroll 2
      for (int o = 0; o < NO; ++o) out_step(o, o == 0 ? y0 : (o == 1 ? y1 : y[n * NO + o]));
    }
    dz = i < Rn ? dz : 0.f;
    dv = rs_ok ? dv : 0.f;

    // ---- dT (in place, accumulator layout = gradient B operand) and dPhi(A1) / dPhi(C1) -----
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float m0 = norm_of(T00[v]), m1 = norm_of(T01[v]);
      const float c10 = c1[0][v], c11 = c1[1][v];
      an1[0][v] = fmaf(dz, T10[v], an1[0][v]);
      an1[1][v] = fmaf(dz, T11[v], an1[1][v]);
      as1[v] = fmaf(dv, hw == 0 ? m0 : m1, as1[v]);
      T10[v] = dz * n1[0][v];
      T11[v] = dz * n1[1][v];
      const float q0 = m0 > 0.f ? dv * c10 * __builtin_amdgcn_rcpf(m0) : 0.f;
      const float q1 = m1 > 0.f ? dv * c11 * __builtin_amdgcn_rcpf(m1) : 0.f;
      T00[v] = q0 * T00[v];
      T01[v] = q1 * T01[v];
    }
    float dTt0 = 0.f, dTt1 = 0.f;  // tail rows: B operand of the zero-padded gradient k step
    if (Dt > 0) {
      dTt1 = dz * n1t;
      dTt0 = Mt > 0.f ? dv * c1t * __builtin_amdgcn_rcpf(Mt) * tt0 : 0.f;
      if (wv == SL_BKW && gq < Dt) {
        if (i < Rn) sTacc[gq * 32 + i] = fmaf(dz, tt1, sTacc[gq * 32 + i]);
        if (vlane) sTacc[gq * 32 + 16 + rs] = fmaf(dv, Mt, sTacc[gq * 32 + 16 + rs]);
      }
    }

    SL_MARK(6);
    // ---- gradient: dPhi0[w in half, :] += X[w, d in pair] dT[d in pair, :] ------------------
    {
      // tail operands of tiles TQ p, TQ p + 1 (then the tail rows are free for the next sample)
      float at[TQ];
#pragma unroll
      for (int u = 0; u < TQ; ++u) at[u] = (Dt > 0 && gq < Dt) ? sTail[gq * TR + 16 * u + i] : 0.f;
      set_dvo();
      int bo0, bo1;
      {
        const int L = sl_lane_now();
        bo0 = bo_of(L, 0);
        bo1 = bo_of(L, 1);
      }
      if (has_next && Dt > 0 && !TAIL_LAST) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        dma_tail(nn);
      }
      // split mode: B fragments of dT (element 2v + h of lane group g = d row 8g + 2v + h of the
      // pair: spectral T0h[v], lin T1h[v])
      sl_u4 ds[3], dl[NL];
      if constexpr (SP) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          sl_split_m(T00[v], T01[v], ds, v);
          uint32_t h1, h2, h3;
          sl_split2(T10[v], T11[v], h1, h2, h3);
          if constexpr (SL_LP(SP)) {  // lanes 8-15 take the second part of column i - 8
            const uint32_t h2r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)h2, 0x128, 0xF, 0xF, false);
            dl[0][v] = i < 8 ? h1 : h2r;
            dl[1][v] = i < 8 ? h3 : 0u;
          } else {
            dl[0][v] = h1;
            dl[1][v] = h2;
            dl[NL - 1][v] = h3;
          }
        }
      }
      // the next tile's operand reads go out before this tile's MFMAs
      sl_f4 pa = *reinterpret_cast<const sl_f4*>(slice + bo0);
      sl_f4 pb = *reinterpret_cast<const sl_f4*>(slice + bo1);
#pragma unroll
      for (int q = 0; q < SL_TILES; ++q) {
        if (q < ntl) {
          const sl_f4 va = pa, vb = pb;
          if (q + 1 < ntl) {
            pa = *reinterpret_cast<const sl_f4*>(slice + 512 * (q + 1) + bo0);
            pb = *reinterpret_cast<const sl_f4*>(slice + 512 * (q + 1) + bo1);
          }
          // the tile's two LDS-DMA pieces of the next sample go out between its MFMAs (after
          // the reads landed), not back to back: bursts stall on the memory issue queue
          if constexpr (!SP) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const sl_f4& src = v < 2 ? va : vb;
              const float a0 = src[2 * (v & 1) + 0], a1 = src[2 * (v & 1) + 1];
              if (!(TR_SLICE_SKIP & 4)) {
                gacc[q][0] = sl_mfma(a0, T00[v], gacc[q][0]);
                gacc[q][1] = sl_mfma(a0, T10[v], gacc[q][1]);
                gacc[q][0] = sl_mfma(a1, T01[v], gacc[q][0]);
                gacc[q][1] = sl_mfma(a1, T11[v], gacc[q][1]);
              }
              if (has_next && (v & 1)) {
                if (v == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tile q's reads landed
                // (the next tile's two reads may still be in flight: waited too)
                dma_piece(nn, q, v >> 1);
              }
            }
          } else {
            // A fragments: element 2v + h = X[w, d of (v, h)] (the order dT is held in)
            sl_u4 af[3];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const sl_f4& src = v < 2 ? va : vb;
              sl_splitx_m<SL_XP(SP)>(src[2 * (v & 1) + 0], src[2 * (v & 1) + 1], af, v);
            }
            // the reads of tile q and q + 1 have landed at this wait: the next sample's pieces of
            // tile q + 1 go out now, a tile earlier (tile 0's at q = 0); the issue order (tiles in
            // order, the tail after tile qt) is the forward's count
            if (has_next) {
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
              if (q == 0) {
                dma_piece(nn, 0, 0);
                dma_piece(nn, 0, 1);
                if (TAIL_LAST && Dt > 0 && qt == 0) dma_tail(nn);
              }
              if (q + 1 < ntl) dma_piece(nn, q + 1, 0);
            }
            if (!(TR_SLICE_SKIP & 4)) {
              if constexpr (SL_ACC(SP, DT))
                gacc[q][0] += sl_mfma6<SL_XP(SP)>(af, ds, sl_f4{0.f, 0.f, 0.f, 0.f});
              else
                gacc[q][0] = sl_mfma6<SL_XP(SP)>(af, ds, gacc[q][0]);
            }
            if (has_next && q + 1 < ntl) {
              dma_piece(nn, q + 1, 1);
              if (TAIL_LAST && Dt > 0 && q + 1 == qt) dma_tail(nn);
            }
            if (!(TR_SLICE_SKIP & 4)) {
              const sl_f4 c1 = SL_ACC(SP, DT) ? sl_f4{0.f, 0.f, 0.f, 0.f} : gacc[q][1];
              sl_f4 r1;
              if constexpr (SL_LP(SP))
                r1 = sl_mfma_lp<SL_XP(SP)>(af, dl, c1);
              else
                r1 = sl_mfma6<SL_XP(SP)>(af, dl, c1);
              gacc[q][1] = SL_ACC(SP, DT) ? gacc[q][1] + r1 : r1;
            }
          }
          if (Dt > 0 && q / TQ == p) {
            gacc[q][0] = sl_mfma(at[q % TQ], dTt0, gacc[q][0]);
            gacc[q][1] = sl_mfma(at[q % TQ], dTt1, gacc[q][1]);
          }
        }
      }
    }
    SL_MARK(7);
  }

#if TR_SLICE_PROFILE
  if (lane == 0 && blockIdx.x < 256)
    for (int q = 0; q < 8; ++q) g_slice_prof[blockIdx.x][wv][q] = prof[q];
#endif
  // ---- per-workgroup slab (arena layout, phi space) -------------------------------------------
  // lane-dependent indices formed afresh from an opaque lane index (held across the sample loop
  // from the prologue, two of them were spilled to scratch: the launch then needed scratch memory)
  const int lp = sl_lane_now();
  const int tp = wv * TR_WAVE + lp, ip = lp & 15, gqp = lp >> 4, rsp = ip / CC;
  const bool vlp = rsp < Rs && (ip % CC) == 0;
  __syncthreads();  // (no LDS-DMA in flight: the last sample issued none)
  if constexpr (SL_LP(SP)) {  // packed lin columns
#pragma unroll
    for (int q = 0; q < SL_TILES; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) gacc[q][1][v] = sl_fold8(gacc[q][1][v]);
  }
#pragma unroll
  for (int q = 0; q < SL_TILES; ++q)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) *reinterpret_cast<sl_f4*>(slice + ((q * 2 + jt) * TR_WAVE + lp) * 4) = gacc[q][jt];
  *reinterpret_cast<sl_f4*>(sEx + (wv * TR_WAVE + lp) * 8) = sl_f4{an1[0][0], an1[0][1], an1[0][2], an1[0][3]};
  *reinterpret_cast<sl_f4*>(sEx + (wv * TR_WAVE + lp) * 8 + 4) = sl_f4{an1[1][0], an1[1][1], an1[1][2], an1[1][3]};
  __syncthreads();
  float* sl = slab + (int64_t)blockIdx.x * slab_stride;
  // dPhi0 (A0 and C0 columns): the four pairs' partials in pair order
  for (int e = tp; e < g.W * 32; e += SL_T) {
    const int w = e >> 5, jc = e & 31;
    const int h2 = w / WH, wl = w - h2 * WH;
    const int q = wl >> 4, gg = (wl & 15) >> 2, reg = wl & 3, jt = jc >> 4, ii = jc & 15;
    const int idx = ((q * 2 + jt) * TR_WAVE + 16 * gg + ii) * 4 + reg;
    float s = 0.f;
#pragma unroll
    for (int p2 = 0; p2 < 4; ++p2) s += lds[(p2 + 4 * h2) * SL_SLICE + idx];
    if (jt == 0) {
      if (ii < RC) sl[g.offC0 + (int64_t)w * RC + ii] = s;
    } else if (ii < Rn) {
      sl[g.offA0 + (int64_t)w * Rn + ii] = s;
    }
  }
  // dPhi(A1) rows d < 128: the two halves' partials; dPhi(C1): the owner lane's own sum
  const int Dm = D < 128 ? D : 128;
  for (int e = tp; e < Dm * Rn; e += SL_T) {
    const int d = e / Rn, r = e - d * Rn;
    const int p2 = d >> 5, c = d & 31, gg = c >> 3, v = (c & 7) >> 1, h = c & 1;
    const int li = 16 * gg + r;
    sl[g.offA1 + e] = sEx[(p2 * TR_WAVE + li) * 8 + 4 * h + v] + sEx[((p2 + 4) * TR_WAVE + li) * 8 + 4 * h + v];
  }
  if (vlp) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int d = dbase + 8 * gqp + 2 * v + hw;
      if (d < D) sl[g.offC1 + (int64_t)d * Rs + rsp] = as1[v];
    }
  }
  if (wv == 0 && Dt > 0 && gqp < Dt) {
    if (ip < Rn) sl[g.offA1 + (int64_t)(128 + gqp) * Rn + ip] = sTacc[gqp * 32 + ip];
    if (vlp) sl[g.offC1 + (int64_t)(128 + gqp) * Rs + rsp] = sTacc[gqp * 32 + 16 + rsp];
  }
  for (int e = tp; e < NO * Rn; e += SL_T) sl[g.offA2 + e] = sAcc[e];
  for (int e = tp; e < NO * Rs; e += SL_T) sl[g.offC2 + e] = sAcc[NO * Rn + e];
  for (int e = tp; e < NO; e += SL_T) sl[g.offB + e] = sAcc[NO * (Rn + Rs) + e];
  if (tp == 0) {
    dpart[2 * blockIdx.x] = *sLoss;
    dpart[2 * blockIdx.x + 1] = 0.0;
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
void spec_slice_geom(SpecGeom* g) {
  g->sl = 0;
  const char* env = std::getenv("TR_SPEC_SLICE");
  if (env != nullptr && env[0] == '0') return;
  const char* gen = std::getenv("TR_SPEC_GENERIC");  // forcing the generic path forces it for training too
  if (gen != nullptr && gen[0] == '1') return;
  if (g->Rn < 1 || g->Rn > 16 || g->Rs < 1 || g->Rs * g->Cc > 16) return;
  if (!(g->Cc == 1 || g->Cc == 2 || g->Cc == 4)) return;
  // any W <= 256: rows past W read zeros (the descriptor's range) and meet zero Phi0 rows; even
  // at W = 32 the padded kernel beats the lock-step k_spec_fused (tools/spec_shapes.py: W = 200
  // 0.60 vs 1.64 ms, W = 128, D = 129 0.84 vs 1.68, W = 64 1.61 vs 3.13, W = 32 3.15 vs 6.07 ms per
  // step at 2 GiB of X)
  if (g->W < 1 || g->W > 2 * SL_ROWS) return;
  // any D <= 130: columns past D (a partial last quad, whole padded pairs) meet zero phi(A1) /
  // phi(C1) rows.  Below D = 128 the kernel still runs all four pairs, and yet it beats the
  // lock-step k_spec_fused at every D measured (tools/spec_shapes.py, W = 256: D = 96 0.57 vs
  // 2.27 ms, D = 65 0.74 vs 1.97, D = 33 1.35 vs 3.38, D = 9 4.76 vs 7.03 ms per fit_Adam step at
  // 2 GiB of X)
  if (g->D < 1 || g->D > 130) return;
  const int Dt = g->D > 128 ? g->D - 128 : 0;
  if (g->NO > 64) return;
  g->slDt = Dt;
  // GEMMs on the bf16 matrix cores through split operands: X in two pieces (default) or three
  // (TR_SLICE_XPIECES=3); TR_SLICE_SPLIT=0 keeps the f32 MFMA form
  const char* spl = std::getenv("TR_SLICE_SPLIT");
  const char* xpc = std::getenv("TR_SLICE_XPIECES");
  const int x3 = (xpc != nullptr && xpc[0] == '3') ? 2 : 0;
  g->slSp = (spl != nullptr && spl[0] == '0') ? 0 : (g->Rn <= 8 ? 1 : 2) + x3;
  g->sl_Dp = ((g->D > 128 ? g->D : 128) + 3) & ~3;
  g->sl_oTail = SL_O_TAIL;
  g->sl_oEx = SL_O_EX;
  g->sl_oTP = SL_O_TP;
  g->sl_oPart = SL_O_PART;
  g->sl_oN1 = SL_O_N1;
  const int64_t small = (int64_t)g->sl_Dp * (g->Rn + g->Rs) + (int64_t)g->NO * 33 + 16 +
                        (int64_t)g->NO * (g->Rn + g->Rs + 1) + 2 * 32;
  g->sl_oLoss = (int)(g->sl_oN1 + ((small + 3) & ~(int64_t)3));  // 16-B aligned double
  const int64_t tot = g->sl_oLoss + 4;
  if (tot * 4 > 160 * 1024) return;
  g->sl_lds_floats = (int)tot;
  g->sl = 1;
}

template <int DT, int SP>
static const void* slice_kernel_dt(int cc) {  // (cc: 1, 2 or 4)
  if (cc == 1) return reinterpret_cast<const void*>(&k_spec_slice<1, DT, SP>);
  if (cc == 2) return reinterpret_cast<const void*>(&k_spec_slice<2, DT, SP>);
  return reinterpret_cast<const void*>(&k_spec_slice<4, DT, SP>);
}
template <int SP>
static const void* slice_kernel_sp(int cc, int dt) {
  return dt == 0 ? slice_kernel_dt<0, SP>(cc) : (dt == 1 ? slice_kernel_dt<1, SP>(cc) : slice_kernel_dt<2, SP>(cc));
}
static const void* slice_kernel(int cc, int dt, int sp) {
  switch (sp) {
    case 0: return slice_kernel_sp<0>(cc, dt);
    case 1: return slice_kernel_sp<1>(cc, dt);
    case 2: return slice_kernel_sp<2>(cc, dt);
    case 3: return slice_kernel_sp<3>(cc, dt);
    case 4: return slice_kernel_sp<4>(cc, dt);
    case 5: return slice_kernel_sp<5>(cc, dt);
    default: return slice_kernel_sp<6>(cc, dt);
  }
}

static hipError_t slice_runs(const SpecGeom& g, int sp, bool* ok) {
  const void* k = slice_kernel(g.Cc, g.slDt, sp);
  hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g.sl_lds_floats * 4);
  if (e != hipSuccess) return e;
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, SL_T, (size_t)g.sl_lds_floats * 4);
  if (e != hipSuccess) return e;
  *ok = per_cu >= 1;
  return hipSuccess;
}

int spec_slice_signed_sp(const SpecGeom& g) { return g.slSpBase + (g.slDt == 0 ? 2 : 4); }

hipError_t spec_slice_prepare(SpecGeom* g) {
  g->slSpBase = g->slSp;
  g->slSigned = 0;
  if (!g->sl) return hipSuccess;
  bool ok = false;
  hipError_t e = slice_runs(*g, g->slSp, &ok);
  if (e != hipSuccess) return e;
  if (!ok) {
    g->sl = 0;  // falls back to k_spec_fused
    return hipSuccess;
  }
  // the signed-X form of a two-piece split (tr_plan_set_x_range picks it per X): SP + 4; without
  // tail rows (D <= 128) that instantiation spills, and the three-piece form (SP + 2) runs instead
  if (g->slSp == 1 || g->slSp == 2) {
    e = slice_runs(*g, spec_slice_signed_sp(*g), &ok);
    if (e != hipSuccess) return e;
    g->slSigned = ok ? 1 : 0;
  }
  return hipSuccess;
}

hipError_t launch_spec_slice(const SpecGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                             const float* Phi0, const float* wts, const float* y, float scale, float* slab,
                             int64_t slab_stride, double* dpart, float* out, int64_t rows_per_wg, int reverse,
                             const int32_t* stop, hipStream_t st) {
  const size_t lb = (size_t)g.sl_lds_floats * 4;
  const void* k = slice_kernel(g.Cc, g.slDt, g.slSp);
  void* args[] = {(void*)&X,    (void*)&N,     (void*)&xld,         (void*)&g,     (void*)&phi,
                  (void*)&Phi0, (void*)&wts,   (void*)&y,           (void*)&scale, (void*)&slab,
                  (void*)&slab_stride, (void*)&dpart, (void*)&out, (void*)&rows_per_wg, (void*)&reverse,
                  (void*)&stop};
  return hipLaunchKernel(k, dim3(grid), dim3(SL_T), args, lb, st);
}

#if TR_SLICE_PROFILE
}  // namespace tr
extern "C" int tr_slice_profile_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tr::g_slice_prof), sizeof(tr::g_slice_prof));
}
namespace tr {
#endif
}  // namespace tr

namespace tr {
// this translation unit's code object, loaded when the first plan is created (tr_api.hip:
// preload_code_objects) instead of at the first launch of one of its kernels
hipError_t touch_code_object_spectral_slice() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_spec_slice<2, 1, 1>));
}
}  // namespace tr
