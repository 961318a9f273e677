// tr_kernels.h — host-side launch interface of the gfx950 kernels (internal, not the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tr_common.h"

namespace tr {

// MODE_MNL_LOGITS: raw logits Z of one class tile (wide-class path, C > 16: the softmax / CE
// epilogue then runs in k_softmax_rows over the whole row of C logits)
enum { MODE_LIN_TRAIN = 0, MODE_LIN_PRED = 1, MODE_MNL_TRAIN = 2, MODE_MNL_PRED = 3, MODE_MNL_LOGITS = 4 };

// Scalars of one k_update launch (Adam constants precomputed on the host in fp64 exactly
// as torch/optim/adam.py does with python floats, then rounded to fp32 like torch's scalar
// arguments).
struct UpdateArgs {
  int mode;            // 0 = Adam step, 1 = finalize only (LBFGS closure)
  int amsgrad;
  float lambda_l2;
  float one_minus_b1;  // lerp weight
  float beta2;
  float one_minus_b2;
  float eps;
  float weight_decay;
  float step_size;     // lr / (1 - b1^t)
  float bc2_sqrt;      // sqrt(1 - b2^t)
  int64_t hist_base;
  int64_t iter;
  int64_t patience;
  double tol;
  int nan_stop;        // spectral fit_Adam: stop (not converged) on a NaN loss while iter <= patience
};

// Next-iteration factor preparation folded into an Adam step (k_update, tr_plan_set_prepare_next):
// mode 1 = phi / dphi (k_prep_factors' output; what the factored multinomial pass reads).
struct PrepArgs {
  int mode;
  float beta, thr;
  float* phi;
  float* dphi;
};

// Launch helpers (all asynchronous on `st`).  Return hipError_t of the launch.
// `xld` is X's row stride in floats (P for a dense X; may differ for strided / windowed views,
// the P floats of each row being contiguous).
hipError_t launch_prep_factors(const FactorSet& fs, const float* params, float beta, float thr,
                               float* phi, float* dphi, const int32_t* stop, hipStream_t st);
// softplus + dense B (one launch when the factors fit LDS, else prep + build)
hipError_t launch_build_dense(const FactorSet& fs, const float* params, float beta, float thr, float* phi,
                              float* dphi, const float* w, float* dense, const int32_t* stop, hipStream_t st);
bool linear_fused_supported(int T, int CH);
hipError_t launch_linear_fused(int T, int CH, int grid, const float* X, int64_t N, int64_t P, int64_t xld,
                               const float* B, const float* bias, const float* y, float scale,
                               float* gpart, double* dpart, float* yhat, int64_t rows_per_wg,
                               int reverse, const int32_t* stop, hipStream_t st);
hipError_t prepare_linear_fused(int T, int CH, size_t lds_bytes, int* wg_per_cu);
// single pass for rows of P <= 128 floats, G = 64 / PQ rows per wave (PQ = linear_packed_pq(P))
int linear_packed_pq(int64_t P);
hipError_t launch_linear_packed(int PQ, int grid, const float* X, int64_t N, int64_t P, int64_t xld, const float* B,
                                const float* bias, const float* y, float scale, float* gpart, double* dpart,
                                int64_t rows_per_wg, int reverse, const int32_t* stop, hipStream_t st);
hipError_t prepare_linear_packed(int PQ, int* wg_per_cu);
// single pass for P beyond one CU's LDS (tr_cluster.hip): clusters of S workgroups, member s
// owning feature slice [s*slice(CH), (s+1)*slice(CH)), exchanging per-row partial dots
int linear_cluster_num_ch(void);
int linear_cluster_ch(int k);
int64_t linear_cluster_slice(int CH);
size_t linear_cluster_lds(int CH);
hipError_t prepare_linear_cluster(int CH, int* wg_per_cu);
hipError_t launch_linear_cluster(int CH, int S, int ncl, const float* X, int64_t N, int64_t P, int64_t xld,
                                 const float* B, const float* bias, const float* y, float scale, float* gpart,
                                 double* dpart, int64_t rows_per_cl, int reverse, uint32_t tag0,
                                 unsigned long long* gran, uint32_t* err, const int32_t* stop, hipStream_t st);
int rows_rb(int C);
int cols_cw(int C);
hipError_t launch_x_range(const float* X, int64_t N, int64_t P, int64_t xld, double* out, int nblocks, hipStream_t st);
bool rows_supported(int C);
hipError_t launch_rows(int C, int mode, int W, const float* X, int64_t N, int64_t P, int64_t xld,
                       const float* Bt, const float* bias, const void* target, const float* class_w,
                       float scale, float* out, double* dpart, float* yhat, const int32_t* stop,
                       hipStream_t st);
int64_t rows_num_waves(int C, int64_t N);
bool rows_mfma_supported(int C, int64_t P);
int64_t rows_mfma_num_waves(int64_t N, int64_t P);
hipError_t launch_rows_mfma(int mode, const float* X, int64_t N, int64_t P, int64_t xld, const float* Bt, int C,
                            const int64_t* lab, const float* class_w, float scale, float* out, double* dpart,
                            const int32_t* stop, hipStream_t st);
hipError_t launch_cols(int C, int W, int64_t nstripes, int64_t nchunks, const float* X, int64_t N,
                       int64_t P, int64_t xld, const float* V, int64_t rows_per_chunk, float* gpart, int reverse,
                       const int32_t* stop, hipStream_t st);
// wide-class multinomial path (any C; C > 16 splits into class tiles of 16):
//   logits Z (N x C) = X . B by class tile (MFMA when mfma != 0, else VALU), then
//   k_softmax_rows: double softmax + weighted CE + dZ in place (train) or the probabilities (pred),
//   then the column reduction X^T dZ by class tile into the (slab, class, feature) partials
int wide_class_tile(void);
hipError_t launch_mnl_logits(int C, int mfma, int W, const float* X, int64_t N, int64_t P, int64_t xld,
                             const float* Bt, float* Z, const int32_t* stop, hipStream_t st);
int64_t softmax_rows_num_waves(int64_t N);
hipError_t launch_softmax_rows(int mode, int C, float* Z, int64_t N, const int64_t* lab, const float* class_w,
                               float scale, float* out, double* dpart, const int32_t* stop, hipStream_t st);
hipError_t launch_cols_wide(int C, int W, int64_t nstripes, int64_t nchunks, const float* X, int64_t N, int64_t P,
                            int64_t xld, const float* V, int64_t rows_per_chunk, float* gpart, int reverse,
                            const int32_t* stop, hipStream_t st);
hipError_t launch_reduce_slabs(int W, const float* part, int64_t nslabs, int64_t ncols, float* out,
                               const double* dpart, int64_t nd, double loss_scale, float* loss_slot,
                               float* bias_slot, const int32_t* stop, hipStream_t st,
                               const float* chain_dphi = nullptr, float* chain_out = nullptr, int64_t nchain = 0,
                               const uint32_t* err = nullptr);
hipError_t launch_mttkrp(const FactorSet& fs, const float* phi, const float* dphi, const float* w,
                         const float* G, float* grad, const int32_t* stop, hipStream_t st, float* part = nullptr,
                         int64_t part_cap = 0);
hipError_t launch_update(const FactorSet& fs, int n_bias, float* params, const float* grad,
                         const UpdateArgs& ua, float* m, float* v, float* vmax, float* grad_total_out,
                         float* loss_out, double* loss_hist, int32_t* stop, hipStream_t st,
                         const PrepArgs* prep = nullptr);
// the plateau test alone (fit_Adam's stop rule, standard…py:467-470) on the fp64 loss history
hipError_t launch_converge(const double* loss_hist, int64_t hist_base, int64_t iter, int64_t patience, double tol,
                           int32_t* stop, hipStream_t st);
// whether k_update can prepare the next iteration in this mode for this factor set
bool update_prepare_mode_ok(const FactorSet& fs, int mode);
// MTTKRP of a two-factor model, one wave per factor row (tr_update.hip); launch_mttkrp uses it
bool mttkrp2_supported(const FactorSet& fs);
bool mttkrp3_supported(const FactorSet& fs, int64_t part_cap);
hipError_t launch_mttkrp3(const FactorSet& fs, const float* phi, const float* dphi, const float* w, const float* G,
                          float* grad, float* part, int64_t part_cap, const int32_t* stop, hipStream_t st);
hipError_t launch_mttkrp2(const FactorSet& fs, const float* phi, const float* dphi, const float* w, const float* G,
                          float* grad, const int32_t* stop, hipStream_t st);

}  // namespace tr
