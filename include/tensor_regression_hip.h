/*
 * tensor_regression_hip.h — C ABI of the MI355X (gfx950) CP tensor-regression hot path.
 *
 * This is the drop-in boundary for the reference's forward/gradient loop
 * (kimerein/tensor_regression).  The reference has no FFI layer of its own: its hot path
 * is the pure-Python/torch sequence
 *
 *     lin_model / model  ->  loss_fn + lambda_L2 * L2_penalty  ->  loss.backward()
 *                        ->  optimizer.step()  ->  loss_running.append(loss.item())
 *
 * in standard_tensor_regression.py:458-470 (CP_linear_regression.fit_Adam) and
 * multinomial_tensor_regression.py:453-465 (CP_logistic_regression.fit_Adam).  Each entry
 * point below replaces one contiguous piece of that sequence; the Python package
 * `tensor_regression_amd` binds them with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - Every pointer argument is DEVICE memory on the plan's device unless stated otherwise;
 *     the library never frees memory it did not allocate.
 *   - fp32 (the reference's multinomial and spectral classes are fp32-only,
 *     multinomial_tensor_regression.py:255; the standard class defaults to fp32, :206), plus a
 *     float64 linear model through the *_f64 entry points (CP_linear_regression(dtype=
 *     torch.float64), standard_tensor_regression.py:206).
 *   - X is sample-major and C-contiguous: X[n, i_1, ..., i_K], i.e. an (N x P) row-major
 *     matrix with P = prod(dims).
 *   - Parameter arena: the Kruskal factor list `Bcp` packed back to back in the reference's
 *     list order, each factor (I_f x R) row-major, followed by the scalar bias for the
 *     linear model: [A_1 | A_2 | ... | A_F | (bias)].  tr_plan_factor_offset() gives the
 *     offsets; tr_plan_num_params() the total.
 *   - Gradient arena: same layout as the parameter arena plus TWO trailing slots: the data
 *     loss, then the device status (0.0 = the pass succeeded; nonzero = a kernel of the pass
 *     failed, see tr_plan_status), i.e. tr_plan_num_grads() = tr_plan_num_params() + 2.
 *     Both slots survive the cross-shard sum meaningfully.  Data-term gradients
 *     are already normalised by the GLOBAL sample count (linear) or class-weight total
 *     (multinomial), so the element-wise sum of the arenas of disjoint sample shards is the
 *     full-data gradient — one all-reduce(sum) per iteration is the only exchange.
 *   - `stream` is a hipStream_t passed as void*; all calls are asynchronous on it.
 *   - Return value: 0 on success, < 0 invalid argument (TR_E_*), > 0 a hipError_t.
 *     tr_last_error() returns a thread-local message for the last failure.
 *   - `stop_flag` (int32 device scalar, may be NULL): when non-zero every kernel of the
 *     iteration returns immediately.  tr_adam_step sets it when the reference's plateau
 *     test fires (standard_tensor_regression.py:467-470), which lets the host enqueue many
 *     iterations without a per-iteration host synchronisation.
 */
#ifndef TENSOR_REGRESSION_HIP_H
#define TENSOR_REGRESSION_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TR_ABI_VERSION 8

#define TR_MODEL_LINEAR 0      /* CP_linear_regression: y_hat = <X, [[w; Phi]]> + bias, MSE */
#define TR_MODEL_MULTINOMIAL 1 /* CP_logistic_regression: softmax(<X, [[w; Phi]]>), CE(weight) */
#define TR_MODEL_SPECTRAL 2    /* spectral CP_linear_regression: lin_model + stepwise_spectral_model, MSE */

#define TR_MAX_FACTORS 8

/* *stop_flag written by tr_adam_step when the gradient arena's status slot is set: the step was
 * NOT applied, parameters and Adam state are those after iteration `iter - 1`.
 * Value = TR_STOP_DEVICE_ERROR - iter (plateau stops are > 0, spectral NaN stops > -2^30). */
#define TR_STOP_DEVICE_ERROR (-(1 << 30))

#define TR_E_ARG (-1)      /* invalid argument (shape/size/pointer) */
#define TR_E_UNSUPPORTED (-2)
#define TR_E_NOMEM (-3)

typedef struct tr_plan tr_plan;

/* Library ABI version (TR_ABI_VERSION). */
int tr_abi_version(void);

/* SHA-256 (hex) of the sources the library was compiled from (the .hip and .h files of csrc,
 * in byte order of their names, then this header); the Python loader refuses a library whose id
 * does not match the sources next to it. */
const char* tr_build_id(void);

/* Thread-local message describing the most recent failure ("" if none). */
const char* tr_last_error(void);

/*
 * Create a plan for one model shape on `device` and allocate its workspace.
 * Replaces the shape bookkeeping of CP_linear_regression.__init__
 * (standard_tensor_regression.py:204-303) / CP_logistic_regression.__init__
 * (multinomial_tensor_regression.py:212-286).
 *   model          TR_MODEL_LINEAR or TR_MODEL_MULTINOMIAL
 *   n_feature_modes K = X.ndim - 1 (1 .. TR_MAX_FACTORS-1)
 *   feature_dims   host array of K dims (I_1 .. I_K)
 *   n_classes      multinomial: C (the extra factor has C rows); linear: ignored (use 1)
 *   rank           R (1 .. 1024)
 *   max_rows       largest sample count later passed to tr_loss_grad (sizes the workspace)
 *   non_negative   host array, one flag per factor (K linear / K+1 multinomial): softplus
 *                  is applied to flagged factors (non_neg_fn, standard…py:53-85)
 *   softplus_beta / softplus_threshold   torch.nn.functional.softplus kwargs
 */
int tr_plan_create(tr_plan** out, int device, int model, int n_feature_modes,
                   const int64_t* feature_dims, int n_classes, int rank, int64_t max_rows,
                   const int32_t* non_negative, float softplus_beta, float softplus_threshold);

int tr_plan_destroy(tr_plan* plan);

int64_t tr_plan_num_params(const tr_plan* plan); /* factors (+ bias) */
int64_t tr_plan_num_grads(const tr_plan* plan);  /* num_params + 2 (data-loss + status slots) */
int64_t tr_plan_factor_offset(const tr_plan* plan, int factor);
int64_t tr_plan_workspace_bytes(const tr_plan* plan);
/* Human-readable description of the kernel strategy chosen for this plan (host string). */
const char* tr_plan_describe(const tr_plan* plan);

/*
 * Row stride of X for the following tr_forward / tr_loss_grad / tr_spectral_latents calls:
 * sample n starts at X + n*stride floats and its P floats are contiguous (stride 0 = P, the
 * dense default).  A stride < P expresses the reference's windowed samples
 * (util.py:67-114, WindowedDataset: sample n = rows [n + w0, n + w1) of an untiled (T, F...)
 * series) without materialising them: stride = F, P = window * F.  The vector (16-byte) kernel
 * paths need stride % 4 == 0 and a 16-byte aligned X; otherwise the plan switches to its scalar
 * paths, and a misaligned X on a vector plan is rejected with TR_E_ARG.
 */
int tr_plan_set_x_stride(tr_plan* plan, int64_t stride);

/*
 * Range statistics of a sample-major X (n_rows rows of P floats at row stride xld; xld = 0: P;
 * rows may overlap): workgroup b of nblocks (1..1024) writes out[b] = max |x|,
 * out[nblocks + b] = the smallest mean x^2 of a row that is not all zero (+inf if none) and
 * out[2 nblocks + b] = min x (doubles) over its rows, asynchronously on `stream`; the caller
 * reduces the 3 * nblocks values (max, min, min).  One streaming read of X.  No reference
 * counterpart: it guards the split kernels' number formats (tr_plan_set_x_range).
 */
int tr_x_range(const float* X, int64_t n_rows, int64_t P, int64_t xld, double* out, int nblocks, void* stream);

/*
 * X's range for the plan's next tr_loss_grad calls (max |x|, the smallest mean x^2 of a nonzero
 * sample, and min x, e.g. from tr_x_range).
 *  - The multinomial factored pass in its bf16-split form represents X as a bf16 piece plus an f16
 *    residual, within 2^-20 |x| + 2^-25 of x — per sample normwise 2^-20 + 2^-25 / rms(sample) —
 *    while every nonzero sample's rms >= 2^-5 and max |x| < 2^23; outside that range (or for a
 *    non-finite value) the plan runs its exact form (three bf16 pieces, x represented exactly,
 *    ~15-20 % slower).
 *  - The spectral column-slice kernel in its split form takes X in two bf16 pieces; on signed X
 *    (min x < 0: the forward T = X Phi0 cancels) the plan runs its signed form (the forward's X in
 *    three pieces and per-sample gradient accumulators, ~13 % slower).
 * Re-set after every tr_plan_set_x_stride call (which resets the plan to its default form).
 * Plans of other kernels ignore it.  The Python layer calls both once per X (Plan._x_form).
 */
int tr_plan_set_x_range(tr_plan* plan, double max_abs, double min_row_mean_sq, double min_x);

/*
 * The multinomial factored pass's shape decision for two-mode samples (I, J), rank R, C classes,
 * without a device (ABI 8): out[0] = 1 if the two-workgroups-per-CU family (k_mnl_duo / k_mnl_bsp)
 * takes the shape, [1] = 1 for its bf16-split body (0: the rank-block body), [2] waves per
 * workgroup, [3] workgroups per CU, [4] ring slots, [5] 1 if padded, [6] compiled row width (32,
 * 64 or 128), [7] row blocks per sample, [8] rank columns (8 or 16), [9] LDS bytes per workgroup,
 * [10] 1 if k_mnl_fused fits the shape.  A plan may still fall back (a spilling instantiation, found at plan
 * creation from the code object).  Reads the same environment switches as tr_plan_create.  n_out:
 * entries to write (at most 11).  Returns TR_E_UNSUPPORTED when no factored kernel fits at all.
 */
int tr_mnl_geometry(int64_t I, int64_t J, int R, int C, int32_t* out, int n_out);

/*
 * Device status of the plan's kernels since the last call (synchronises the device).
 * *status = 0: healthy.  Bit 0: a cross-workgroup exchange of the single-pass kernel for wide
 * rows (P beyond one CU's LDS) gave up waiting for a partner workgroup — it happens only when
 * the GPU is shared with another kernel so the cluster was not co-resident (the plan launches at
 * most one workgroup per CU, so an unshared GPU always holds the whole grid); that call's
 * gradient and loss are NaN and the gradient arena's status slot is set.  No reference
 * counterpart (the reference has no device kernels).
 */
int tr_plan_status(tr_plan* plan, int32_t* status);

/*
 * Recover from a device-side failure (status bit set / TR_STOP_DEVICE_ERROR): clears the status
 * and switches the plan to its two-pass path, which has no cross-workgroup dependence.  The fit
 * loop then resumes at the failed iteration from the untouched parameters and Adam state.
 */
int tr_plan_recover(tr_plan* plan);

/*
 * Forward model only (predict path).
 * Replaces lin_model (standard…py:87-130) — out[n] = <X_n, B> + bias — and model
 * (multinomial…py:148-187) — out[n, c] = softmax_c(<X_n, B_c>) — where
 * B = cp_to_tensor((weights, non_neg_fn(Bcp))).
 *   out: n_rows floats (linear) or n_rows x C floats row-major (multinomial).
 */
int tr_forward(tr_plan* plan, const float* X, int64_t n_rows, const float* params,
               const float* weights, float* out, void* stream);

/*
 * Data-term loss and gradient of one sample shard (forward + loss + backward).
 * Replaces the forward, loss_fn and loss.backward() of one fit_Adam iteration
 * (standard…py:460-462; multinomial…py:455-457) — WITHOUT the L2 term, which
 * tr_adam_step / tr_finalize_grad add once after the cross-shard sum.
 *   target      linear: float y[n_rows]; multinomial: int64 labels[n_rows] in [0, C)
 *   class_weight multinomial: float[C] CrossEntropyLoss weights; linear: NULL
 *   norm        linear: global N (MSELoss mean); multinomial: global sum_n cw[y_n]
 *   grad_out    tr_plan_num_grads() floats, overwritten: data gradient of every parameter
 *               (+ bias) and the data loss in the last slot.
 *   yhat_out    optional (may be NULL): linear model output per row (n_rows floats).
 */
int tr_loss_grad(tr_plan* plan, const float* X, int64_t n_rows, const void* target,
                 const float* class_weight, double norm, const float* params,
                 const float* weights, float* grad_out, float* yhat_out,
                 const int32_t* stop_flag, void* stream);

/*
 * L2 term + total loss only (no parameter update) — the closure value/gradient that
 * torch.optim.LBFGS needs in fit() (standard…py:368-373, multinomial…py:357-362).
 *   grad_total_out  num_params floats: data gradient + lambda * d(sum_k ||A_k||_F)/dA
 *   loss_out        1 float: data loss + lambda * sum_k ||A_k||_F (L2_penalty, standard…py:180-196)
 */
int tr_finalize_grad(tr_plan* plan, const float* params, const float* grad,
                     float lambda_l2, float* grad_total_out, float* loss_out, void* stream);

/*
 * One torch.optim.Adam / AMSGrad step on the whole parameter arena, preceded by the L2
 * term and followed by the reference's bookkeeping:
 *   loss_hist[hist_base + iter] = data loss + lambda * L2_penalty   (loss_running.append)
 *   if iter > patience and sum(|diff(loss_hist[iter - patience : hist_base + iter + 1])|) < tol:
 *       *stop_flag = iter + 1                                      (standard…py:467-470)
 * Adam math follows torch/optim/adam.py _single_tensor_adam (torch 2.10):
 *   g += wd * p; m = lerp(m, g, 1 - b1); v = v * b2 + (1 - b2) g^2;
 *   vmax = max(vmax, v) if amsgrad; denom = sqrt(v or vmax) / sqrt(1 - b2^t) + eps;
 *   p -= lr / (1 - b1^t) * m / denom.
 *   step        1-based Adam step t for this iteration
 *   loss_hist   fp64 device array (the reference's loss_running as python floats)
 *   max_exp_avg_sq  may be NULL when amsgrad == 0
 */
int tr_adam_step(tr_plan* plan, float* params, const float* grad, float* exp_avg,
                 float* exp_avg_sq, float* max_exp_avg_sq, float lambda_l2, double lr,
                 double beta1, double beta2, double eps, double weight_decay, int amsgrad,
                 int64_t step, double* loss_hist, int64_t hist_base, int64_t iter,
                 int64_t patience, double tol, int32_t* stop_flag, void* stream);

/*
 * Fold the NEXT iteration's factor preparation into tr_adam_step: with enable = 1, on a plan
 * that takes the factored multinomial single pass, every tr_adam_step also computes
 * softplus(A_k) and its derivative from the parameters it has just written, and the following
 * tr_loss_grad on the SAME params pointer skips its own preparation launch.  Valid as long as
 * the parameters change only through tr_adam_step between those calls (the fit_Adam loop);
 * results are bitwise identical to enable = 0.  Other plans ignore the setting.
 */
int tr_plan_set_prepare_next(tr_plan* plan, int enable);

/*
 * float64 linear model: CP_linear_regression(..., dtype=torch.float64) (standard…py:206; the
 * reference's KAT-1, demo_TensorRegression.ipynb, is an fp64 LBFGS fit).  Same arenas and
 * semantics as the fp32 entry points above with double buffers (X, y, params, weights, grad,
 * Adam state, outputs); the plan computes in double (two passes over X on the VALU).  A float64
 * plan accepts only the _f64 entry points, a float32 plan only the float ones (TR_E_ARG).
 */
int tr_plan_create_f64(tr_plan** out, int device, int n_feature_modes, const int64_t* feature_dims, int rank,
                       int64_t max_rows, const int32_t* non_negative, double softplus_beta,
                       double softplus_threshold);
int tr_forward_f64(tr_plan* plan, const double* X, int64_t n_rows, const double* params, const double* weights,
                   double* out, void* stream);
int tr_loss_grad_f64(tr_plan* plan, const double* X, int64_t n_rows, const double* y, double norm,
                     const double* params, const double* weights, double* grad_out, double* yhat_out,
                     const int32_t* stop_flag, void* stream);
int tr_finalize_grad_f64(tr_plan* plan, const double* params, const double* grad, double lambda_l2,
                         double* grad_total_out, double* loss_out, void* stream);
int tr_adam_step_f64(tr_plan* plan, double* params, const double* grad, double* exp_avg, double* exp_avg_sq,
                     double* max_exp_avg_sq, double lambda_l2, double lr, double beta1, double beta2, double eps,
                     double weight_decay, int amsgrad, int64_t step, double* loss_hist, int64_t hist_base,
                     int64_t iter, int64_t patience, double tol, int32_t* stop_flag, void* stream);

/*
 * Spectral model plan (spectral_tensor_regression.CP_linear_regression, spectral…py:424-539;
 * fit model lin_model :118-165 + stepwise_spectral_model :339-390; predict model
 * lin_model + spectral_model :168-220).  X is (N, n_w, n_d) fp32, y is (N, n_out) fp32.
 *   n_complex      = n_complex_dim + 1 (third dim of Bcp_c[0])
 *   non_negative   host int32[3]: flags of the (w, d, out) factors, shared by Bcp_n and Bcp_c
 * Parameter arena (reference order Bcp_n + Bcp_c + [bias], each row-major):
 *   A0 (n_w, Rn) | A1 (n_d, Rn) | A2 (n_out, Rn) | C0 (n_w, Rs, n_complex) | C1 (n_d, Rs) |
 *   C2 (n_out, Rs) | bias (n_out)
 * tr_plan_factor_offset(plan, f) gives f = 0..5 and the bias offset for f = 6.
 * With such a plan:
 *   tr_loss_grad   target = y (N x n_out floats), norm = global N * n_out (MSELoss mean),
 *                  class_weight = NULL, yhat_out (optional) = fit-model y_hat (N x n_out)
 *   tr_forward     out (N x n_out) = the reference's predict() model (spectral…py:959-960);
 *                  weights = all rank_normal + rank_spectral weights
 *   tr_adam_step   also applies the spectral NaN stop (spectral…py:738-741): when the loss
 *                  is NaN and iter <= patience, *stop_flag = -(iter + 1) (stopped, not converged)
 * Envelope (tr_plan_create_spectral returns TR_E_UNSUPPORTED outside it, with the reason in
 * tr_last_error()):  K = rank_normal + rank_spectral * n_complex <= 256, n_w <= 2^24,
 * n_d, n_out <= 2^16, and one sample's epilogue — n_d * (K + 1) + (n_d + n_out) *
 * (rank_normal + rank_spectral) floats (+ scratch) — within the 160 KiB LDS of a CU.  Inside it
 * the plan picks (tr_plan_describe):
 *   slice-1pass-mfma   training at n_w = 256, 97 <= n_d <= 130 (n_d >= 128 or n_d % 4 == 0),
 *                      1 <= Rn <= 16, Rs * n_complex <= 16 with n_complex in {1, 2, 4},
 *                      n_out <= 64 (and its LDS fits): column-slice single pass (config 5);
 *                      described as slice-1pass-mfma-bf16split when its GEMMs run on the bf16
 *                      matrix cores through split operands (the default): factor-side operands in
 *                      three round-to-nearest bf16 pieces (exact), the sample data in two
 *                      (|x - x1 - x2| < 2^-16 |x|, measured 2^-17, unbiased), fp32 accumulation.  At full config-5
 *                      size its gradients lie within 3.5e-7 normwise of an fp64 closed form (the
 *                      f32 MFMA form 1.1e-7, the reference's own fp32 op sequence 0.6-4.2e-6);
 *                      results are not bitwise those of the f32 MFMA form.  Environment, read at
 *                      plan creation: TR_SLICE_XPIECES=3 takes the sample data in three pieces too
 *                      (exact; slower), TR_SLICE_SPLIT=0 the f32 MFMA form
 *   fused-1pass-mfma   K <= 32, n_w, n_d, n_out <= 256 and the whole sample + scratch in LDS:
 *                      single pass; also every tr_forward / tr_spectral_latents of such a plan
 *   generic-3kernel-mfma  any other shape in the envelope: T_n staged through HBM (three kernels)
 */
int tr_plan_create_spectral(tr_plan** out, int device, int64_t n_w, int64_t n_d, int64_t n_out,
                            int rank_normal, int rank_spectral, int n_complex, int64_t max_rows,
                            const int32_t* non_negative, float softplus_beta, float softplus_threshold);

/*
 * stepwise_latents_model (spectral…py:284-336) — out (N x rank_normal) =
 * einsum('tdr,drs->tr', einsum('twd,wrs->tdr', X, phi(A0)), phi(A1)); used by predict_latents.
 */
int tr_spectral_latents(tr_plan* plan, const float* X, int64_t n_rows, const float* params, float* out,
                        void* stream);

/*
 * Per-kernel device timing (measurement support; no reference counterpart).
 * `enable` is a bit mask over TR_KERNEL_* kinds (1 << kind; -1 = all): every launch of a
 * selected kind is bracketed by hipEvents on the caller's stream (no host synchronisation).  tr_plan_read_timing synchronises the recorded events and returns,
 * per kernel kind (TR_KERNEL_*), the summed elapsed milliseconds and the number of launches,
 * then clears the record.  tr_plan_set_timing_every(plan, n) brackets only the n-th, 2n-th, ...
 * launch of each selected kind (n >= 1, default 1; tr_plan_set_timing restarts the count), for
 * runs that must disturb the stream even less.  The events are timing-only (no system-scope
 * fence when recorded).
 */
#define TR_KERNEL_STREAM_FUSED 0 /* single-pass X stream (linear) */
#define TR_KERNEL_STREAM_ROWS 1  /* two-pass forward X stream */
#define TR_KERNEL_STREAM_COLS 2  /* two-pass backward X stream */
#define TR_KERNEL_REDUCE 3       /* slab reduction */
#define TR_KERNEL_MTTKRP 4       /* factor gradients */
#define TR_KERNEL_PREP 5         /* softplus + dense B */
#define TR_KERNEL_UPDATE 6       /* L2 + Adam + plateau test */
#define TR_KERNEL_NKINDS 7
int tr_plan_set_timing(tr_plan* plan, int enable);
int tr_plan_set_timing_every(tr_plan* plan, int every);
int tr_plan_read_timing(tr_plan* plan, double* total_ms /* [TR_KERNEL_NKINDS] */,
                        int64_t* launches /* [TR_KERNEL_NKINDS] */);

#ifdef __cplusplus
}
#endif

#endif /* TENSOR_REGRESSION_HIP_H */
