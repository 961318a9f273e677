// tr_fp64.h — float64 linear CP model (CP_linear_regression(dtype=torch.float64)): launch helpers
// of tr_fp64.hip, all asynchronous on `st`.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tr_kernels.h"

namespace tr {

struct Update64 {
  int mode;  // 0 = Adam step, 1 = finalize only (LBFGS closure)
  int amsgrad;
  double lambda_l2, one_minus_b1, beta2, one_minus_b2, eps, weight_decay, step_size, bc2_sqrt;
  int64_t hist_base, iter;
};

hipError_t launch64_prep_dense(const FactorSet& fs, const double* params, double beta, double thr, double* phi,
                               double* dphi, const double* w, double* dense, const int32_t* stop, hipStream_t st);
int64_t rows64_num_waves(int64_t N);
// pred: out = y_hat; else out = residual * scale, yhat (optional) = y_hat, dpart = (sse, sum r) per wave
hipError_t launch64_rows(int pred, const double* X, int64_t N, int64_t P, int64_t xld, const double* B,
                         const double* bias, const double* y, double scale, double* out, double* yhat, double* dpart,
                         const int32_t* stop, hipStream_t st);
hipError_t launch64_cols(const double* X, int64_t N, int64_t P, int64_t xld, const double* r, int64_t nchunks,
                         double* gpart, const int32_t* stop, hipStream_t st);
hipError_t launch64_reduce(const double* part, int64_t nslabs, int64_t P, double* G, const double* dpart, int64_t nd,
                           double loss_scale, double* loss_slot, double* bias_slot, const int32_t* stop,
                           hipStream_t st);
hipError_t launch64_mttkrp(const FactorSet& fs, const double* phi, const double* dphi, const double* w,
                           const double* G, double* grad, const int32_t* stop, hipStream_t st);
hipError_t launch64_update(const FactorSet& fs, int n_bias, double* params, const double* grad, const Update64& ua,
                           double* m, double* v, double* vmax, double* grad_total_out, double* loss_out,
                           double* loss_hist, int32_t* stop, hipStream_t st);

}  // namespace tr
