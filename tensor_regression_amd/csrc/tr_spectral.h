// tr_spectral.h — host/device interface of the spectral-model kernels
// (spectral_tensor_regression.py: lin_model 118-165, spectral_model 168-220,
// stepwise_latents_model 284-336, stepwise_spectral_model 339-390).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace tr {

enum { SPEC_TRAIN = 0, SPEC_PRED = 1, SPEC_LATENT = 2 };

// Geometry of one spectral model shape, passed to the kernels by value.
//
// X is (N, W, D) sample-major.  Parameters (the reference's Bcp_n + Bcp_c + [bias], in that
// order, each factor row-major):
//   A0 (W, Rn, 1) | A1 (D, Rn, 1) | A2 (NO, Rn, 1) | C0 (W, Rs, Cc) | C1 (D, Rs, 1) | C2 (NO, Rs, 1) | bias (NO)
// The two W-side factors are contracted in ONE GEMM per sample:
//   T_n (D x K) = X_n^T (D x W) . Phi0 (W x K),   Phi0 = [phi(A0) | phi(C0) flattened (r, c)],
//   K = Rn + Rs*Cc,
// on v_mfma_f32_16x16x4_f32 with X_n staged in LDS (row stride S, odd => conflict-free MFMA
// operand reads in both GEMM orientations) and Phi0's B fragments resident in registers.
struct SpecGeom {
  int W, D, NO, Rn, Rs, Cc, K, KT;  // KT = ceil(K / 16) column tiles
  int S;                            // LDS row stride of X_n (= D: lane-linear LDS-DMA image)
  int KS;                           // LDS row stride of the T / dT scratch (16*KT + 1)
  int Wrows;                        // LDS rows of the X_n region (16*ceil(W/16), pad rows zero)
  int nDF, Dtail;                   // full 16-row d tiles, remaining d rows
  int WS;                           // forward k steps (32 per 128-row block of w)
  int DS;                           // gradient-GEMM k steps over d (64-block walk)
  int nWT;                          // 16-row w tiles of the gradient GEMM
  int vec;                          // X_n staged by 16-B LDS-DMA pieces (W*D % 4 == 0), else 4-B
  int64_t WD;                       // W*D (floats per sample)
  int64_t offA0, offA1, offA2, offC0, offC1, offC2, offB, nparams;
  int nonneg[3];
  // LDS carve (floats)
  int oT, oTail, oRed, oSm, oAcc, oPhi, lds_floats;
  // generic path (tr_spectral_gen.hip) for shapes outside the fused kernel's envelope
  int gen;  // 1: T_n staged through HBM by k_specg_fwd / k_specg_epi / k_specg_bwd
  int gKP;  // K padded to 16 (row stride of the T / dT staging buffer)
  // column-slice training kernel (tr_spectral_slice.hip) for the shapes it covers (config 5)
  int sl;                       // 1: SPEC_TRAIN runs k_spec_slice
  int slSp;                     // its GEMMs: 0 f32 MFMA; bf16 split with X in two pieces: 1 lin packed, 2 not; X in three: 3, 4;
                                // signed X (forward X in three pieces, per-sample gradient accumulators): 5, 6
  int slSpBase, slSigned;       // the plan's form for non-negative X, and whether its signed-X form (+4) runs
  int slDt, sl_Dp;              // rows d >= 128 (<= 2), rows of the phi(A1) / phi(C1) tables
  int sl_oTail, sl_oEx, sl_oTP, sl_oPart, sl_oN1, sl_oLoss, sl_lds_floats;  // LDS carve (floats)
};

// Fills g; returns false (with a reason) when the shape is outside the kernels' envelope.
bool spec_geom_init(SpecGeom* g, int64_t W, int64_t D, int64_t NO, int Rn, int Rs, int Cc, const int32_t* nonneg,
                    std::string* why);
// Whether the fused kernel for this geometry fits (LDS, registers) on the device.
hipError_t spec_prepare(const SpecGeom& g, int mode, int* ok);

// phi / dphi of every parameter (softplus where flagged; bias copied, dphi = 1) and the
// concatenated W-side matrix Phi0 (W x K).
hipError_t launch_spec_prep(const SpecGeom& g, const float* params, float beta, float thr, float* phi,
                            float* dphi, float* Phi0, const int32_t* stop, hipStream_t st);
// The fused single-pass kernel (one workgroup per CU, contiguous sample ranges).
//   SPEC_TRAIN : per-workgroup gradient slabs (arena layout, phi-space) + (sse, 0) in dpart;
//                `out` (optional) receives the fit-model y_hat (N x NO)
//   SPEC_PRED  : out (N x NO) = lin_model + spectral_model (the reference's predict)
//   SPEC_LATENT: out (N x Rn) = stepwise_latents_model
hipError_t launch_spec_fused(int mode, const SpecGeom& g, int grid, const float* X, int64_t N, int64_t xld,
                             const float* phi,
                             const float* Phi0, const float* wts, const float* y, float scale, float* slab,
                             int64_t slab_stride, double* dpart, float* out, int64_t rows_per_wg, int reverse,
                             const int32_t* stop, hipStream_t st);
// generic path: dynamic-LDS attribute of the epilogue kernel; T is a (N x D x gKP) staging buffer;
// SPEC_TRAIN writes one arena-layout slab (phi space) + (sse, 0) per chunk of ceil(N / nchunks)
// samples, i.e. ceil(N / ceil(N / nchunks)) slabs
size_t specg_epi_lds_bytes(const SpecGeom& g);
hipError_t specg_prepare(const SpecGeom& g);
hipError_t launch_specg(int mode, const SpecGeom& g, int nchunks, const float* X, int64_t N, int64_t xld,
                        const float* phi, const float* Phi0, const float* wts, const float* y, float scale,
                        float* T, float* slab, int64_t slab_stride, double* dpart, float* out,
                        const int32_t* stop, hipStream_t st);
// column-slice kernel: eligibility + LDS carve (sets g->sl), occupancy check (may clear g->sl),
// launch (SPEC_TRAIN only; same outputs as launch_spec_fused)
void spec_slice_geom(SpecGeom* g);
hipError_t spec_slice_prepare(SpecGeom* g);
int spec_slice_signed_sp(const SpecGeom& g);  // the slice kernel form for signed X (tr_plan_set_x_range)
hipError_t launch_spec_slice(const SpecGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                             const float* Phi0, const float* wts, const float* y, float scale, float* slab,
                             int64_t slab_stride, double* dpart, float* out, int64_t rows_per_wg, int reverse,
                             const int32_t* stop, hipStream_t st);
// grad[e] = G[e] * dphi[e]  (softplus chain of the reduced phi-space gradient)
hipError_t launch_spec_chain(int64_t n, const float* G, const float* dphi, float* grad, const int32_t* stop,
                             hipStream_t st);

}  // namespace tr
