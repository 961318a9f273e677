"""Spectral CP tensor regression on MI355X — drop-in for the reference's
`spectral_tensor_regression.py` (kimerein/tensor_regression).

Same module functions and `CP_linear_regression` class (same arguments, defaults, attributes,
factor layouts Bcp_n (I, Rn, 1) and Bcp_c (W, Rs, n_complex_dim+1), (D, Rs, 1), (n_out, Rs, 1),
`loss_running` semantics), with the fit/predict hot path on gfx950, each sample of X read from
HBM once per iteration.  Kernel envelope (the plan picks the first that covers the shape):
  * training with X.shape[1] <= 256, X.shape[2] <= 130 (config 5: 256 x 129), rank_normal <= 16,
    rank_spectral * (n_complex_dim + 1) <= 16,
    n_complex_dim + 1 in {1, 2, 4}, n_out <= 64 — runs the column-slice single pass
    k_spec_slice (csrc/tr_spectral_slice.hip: bf16 split GEMMs on the matrix cores);
  * other shapes with K = rank_normal + rank_spectral * (n_complex_dim + 1) <= 32,
    X.shape[1], X.shape[2], n_out <= 256 and the whole sample in a CU's 160 KiB LDS (and every
    predict / predict_latents call of such shapes) run the whole-sample single pass k_spec_fused
    (csrc/tr_spectral.hip);
  * the rest, up to K <= 256 with one sample's epilogue (X.shape[2] * (K + 1) +
    (X.shape[2] + n_out) * (rank_normal + rank_spectral) floats) in a CU's LDS, the three-kernel
    path (csrc/tr_spectral_gen.hip).  Outside that the plan raises ValueError.

Reference semantics kept as they are: the fit model is
lin_model + stepwise_spectral_model (norm BEFORE the d/out contractions) while predict uses
lin_model + spectral_model (norm AFTER the full contraction); the bias is added by both terms;
the spectral fit_Adam / fit stop on a NaN loss.

Deliberate differences: tensors run on a HIP device, fp32 only; a y with n_out == 1 is
rejected (the reference broadcasts (N,) + (N,1) to (N,N), Q10).
"""
import numpy as np
import torch

from . import _engine, _lib
from ._engine import SpectralPlan, adam_hparams, as_device_f32, run_adam_fit

__all__ = ["make_BcpInit", "non_neg_fn", "edge_clamp", "lin_model", "spectral_model", "stepwise_linear_model",
           "stepwise_latents_model", "stepwise_spectral_model", "L2_penalty", "CP_linear_regression"]


####################################
######## Helper functions ##########
####################################

def make_BcpInit(B_dims, rank, non_negative, complex_dims=None, scale=1, device='cpu', dtype=torch.float32):
    """Initial Kruskal factors (I, rank, complex_dim) (spectral…py:17-60): orthogonal init with
    gain `scale` on the CPU generator (seed-identical to the reference), non-negative factors
    shifted by two standard deviations and halved when the first factor has more than one row."""
    if complex_dims is None:
        complex_dims = list([1] * len(B_dims))
    Bcp_init = [torch.nn.init.orthogonal_(torch.empty(B_dims[ii], rank, complex_dims[ii], dtype=dtype),
                                          gain=scale).to(device) for ii in range(len(B_dims))]
    Bcp_init = [(Bcp_init[ii] + torch.std(Bcp_init[ii]) * 2 * non_negative[ii]) / (non_negative[ii] + 1)
                if Bcp_init[0].shape[0] > 1 else Bcp_init[ii] for ii in range(len(Bcp_init))]
    return Bcp_init


def non_neg_fn(B_cp, non_negative, softplus_kwargs=None):
    """Yield softplus(A_k) for flagged factors, A_k otherwise (spectral…py:62-94)."""
    if softplus_kwargs is None:
        softplus_kwargs = {'beta': 50, 'threshold': 1}
    for ii in range(len(B_cp)):
        if non_negative[ii]:
            yield torch.nn.functional.softplus(B_cp[ii], **softplus_kwargs)
        else:
            yield B_cp[ii]


def edge_clamp(B_cp, edge_idx, clamp_val=0, device='cpu', dtype=torch.float32):
    """Zero (clamp_val) rows `edge_idx` of the first factor (spectral…py:97-115)."""
    eIdxBool = torch.ones(B_cp[0].shape[0], dtype=dtype, device=device)
    eIdxBool[edge_idx] = clamp_val
    return [B_cp[0] * eIdxBool[:, None, None], B_cp[1], B_cp[2]]


def L2_penalty(B_cp):
    """sum_k ||B_k||_F of the raw factors, not squared (spectral…py:393-417)."""
    ii = 0
    for comp in B_cp:
        ii += torch.sqrt(torch.sum(comp ** 2))
    return ii


_plan_cache = {}


def _plan(shape, n_out, rank_normal, rank_spectral, n_complex, rows, non_negative, softplus_kwargs, device):
    beta, thr = _engine.softplus_params(softplus_kwargs)
    key = (int(shape[0]), int(shape[1]), int(n_out), int(rank_normal), int(rank_spectral), int(n_complex),
           tuple(bool(non_negative[f]) for f in range(3)), beta, thr, _engine.device_index(device))
    p = _plan_cache.get(key)
    if p is None or p.max_rows < rows:
        p = SpectralPlan(shape[0], shape[1], n_out, rank_normal, rank_spectral, n_complex, rows, non_negative,
                         softplus_kwargs, device)
        _plan_cache[key] = p
    return p


def _check_X(X, name):
    if not isinstance(X, torch.Tensor) or X.device.type != "cuda":
        raise ValueError(f"{name}: X must be a torch tensor on a HIP device (device='cuda')")
    if X.ndim != 3:
        raise ValueError(f"{name}: X must be 3-D (N, W, D) (the reference's einsum 'twd', spectral…py:387)")


def _zero_factors(shapes, dev):
    return [torch.zeros(s, dtype=torch.float32, device=dev) for s in shapes]


def _module_forward(X, Bcp_n, Bcp_c, weights, rank_normal, non_negative, bias, softplus_kwargs, what):
    """Runs the predict kernel with one side of the model empty (rank 0 => that term is absent)."""
    dev = X.device
    Xd = _engine.as_device_rows(X, dev.index)
    W, D = int(X.shape[1]), int(X.shape[2])
    bias = torch.as_tensor(bias, dtype=torch.float32).to(dev).reshape(-1)
    n_out = int((Bcp_n or Bcp_c)[2].shape[0])
    if bias.numel() == 1 and n_out > 1:
        bias = bias.expand(n_out)
    Rn = int(Bcp_n[0].shape[1]) if Bcp_n else 0
    Rs = int(Bcp_c[0].shape[1]) if Bcp_c else 0
    Cc = int(Bcp_c[0].shape[2]) if Bcp_c else 1
    plan = _plan((W, D), n_out, Rn, Rs, Cc, Xd.shape[0], list(non_negative), softplus_kwargs, dev)
    Bn = Bcp_n if Bcp_n else _zero_factors([(W, 0, 1), (D, 0, 1), (n_out, 0, 1)], dev)
    Bc = Bcp_c if Bcp_c else _zero_factors([(W, 0, Cc), (D, 0, 1), (n_out, 0, 1)], dev)
    arena = plan.pack([torch.as_tensor(A).to(dev) for A in Bn], [torch.as_tensor(A).to(dev) for A in Bc], bias)
    w = torch.as_tensor(weights, dtype=torch.float32).to(dev).reshape(-1)
    w_full = torch.cat([w, torch.ones(Rs, device=dev)]) if what == "lin" else torch.cat([torch.ones(Rn, device=dev), w])
    return plan, Xd, arena, w_full.contiguous()


def lin_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """inner(X, cp_to_tensor((weights, non_neg_fn(Bcp[:, :, 0]))), n_modes=2).squeeze() + bias
    (spectral…py:118-165) on the gfx950 predict kernel.  X (N, W, D) on a HIP device; returns
    (N, n_out) fp32 (no autograd graph)."""
    _check_X(X, "lin_model")
    if Bcp[0].shape[1] == 0:
        return torch.zeros(1).to(X.device)
    plan, Xd, arena, w = _module_forward(X, list(Bcp), None, weights, int(Bcp[0].shape[1]), non_negative, bias,
                                         softplus_kwargs, "lin")
    return plan.forward(Xd, arena, w).squeeze()


def spectral_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """norm_c(inner(X, cp_to_tensor((weights, [Bcp[0][:, :, c], Bcp[1][:, :, 0], ...])))) + bias
    (spectral…py:168-220) — the reference's predict-time spectral term."""
    _check_X(X, "spectral_model")
    if Bcp[0].shape[1] == 0:
        return torch.zeros(1).to(X.device)
    plan, Xd, arena, w = _module_forward(X, None, list(Bcp), weights, 0, non_negative, bias, softplus_kwargs,
                                         "spec")
    return plan.forward(Xd, arena, w)


def stepwise_latents_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """einsum('tdr,drs->tr', einsum('twd,wrs->tdr', X, phi(Bcp[0])), phi(Bcp[1])) (spectral…py:284-336)."""
    _check_X(X, "stepwise_latents_model")
    if Bcp[0].shape[1] == 0:
        return torch.zeros(1).to(X.device)
    n_out = int(Bcp[2].shape[0]) if len(Bcp) > 2 else 2
    Bn = list(Bcp) if len(Bcp) > 2 else list(Bcp) + [torch.zeros(n_out, Bcp[0].shape[1], 1)]
    plan, Xd, arena, _ = _module_forward(X, Bn, None, torch.ones(int(Bcp[0].shape[1])), int(Bcp[0].shape[1]),
                                         non_negative, torch.zeros(n_out), softplus_kwargs, "lin")
    return plan.latents(Xd, arena)


def stepwise_linear_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """The reference's stepwise form of the linear term (spectral…py:223-281) returns
    einsum('tdr,drs->tr', ...) — the rank latents, not y_hat; kept as that."""
    return stepwise_latents_model(X, Bcp, weights, non_negative, bias, softplus_kwargs)


def stepwise_spectral_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """einsum('tr,nrs->tn', einsum('tdr,drs->tr', ||einsum('twd,wrc->tdrc')||_c, phi(Bcp[1])), phi(Bcp[2]))
    + bias (spectral…py:339-390) — the fit-time spectral term (weights unused, as in the reference)."""
    _check_X(X, "stepwise_spectral_model")
    if Bcp[0].shape[1] == 0:
        return torch.zeros(1).to(X.device)
    plan, Xd, arena, w = _module_forward(X, None, list(Bcp), torch.ones(int(Bcp[0].shape[1])), 0, non_negative,
                                         bias, softplus_kwargs, "spec")
    n_out = plan.dims[2]
    N = Xd.shape[0]
    y0 = torch.zeros((N, n_out), dtype=torch.float32, device=Xd.device)
    grad = torch.zeros(plan.num_grads, dtype=torch.float32, device=Xd.device)
    yhat = torch.empty((N, n_out), dtype=torch.float32, device=Xd.device)
    plan.loss_grad(Xd, y0, None, float(N * n_out), arena, w, grad, yhat=yhat)
    return yhat


class _VerbosePrinter:
    """verbose==2 per-iteration print of the reference (spectral…py:728-732), fit-model y_hat."""

    def __init__(self, plan, X, y, weights, norm):
        self.plan, self.X, self.y, self.w, self.norm = plan, X, y, weights, norm
        self.var_y = torch.var(y).item()
        self.grad = torch.zeros(plan.num_grads, dtype=torch.float32, device=X.device)
        self.yhat = torch.empty_like(y)

    def before_step(self, arena):
        self.plan.loss_grad(self.X, self.y, None, self.norm, arena, self.w, self.grad, yhat=self.yhat)

    def after_step(self, ii, loss):
        ratio = torch.var(self.yhat).item() / self.var_y
        print(f'Iteration: {ii}, Loss: {loss}  ;  Variance ratio (y_hat / y_true): {ratio}')


####################################
########### Main class #############
####################################

class CP_linear_regression():
    def __init__(self,
                 X_shape,
                 y_shape,
                 dtype=torch.float32,
                 rank_normal=1,
                 rank_spectral=1,
                 non_negative=False,
                 weights=None,
                 Bcp_init=None,
                 Bcp_init_scale=1,
                 n_complex_dim=0,
                 bias_init=0,
                 device='cpu',
                 softplus_kwargs=None):
        """Spectral CP regression (spectral_tensor_regression.py:425-539; same arguments and
        attributes; `bias_init` is accepted and unused, as in the reference)."""
        self.dtype = dtype
        if weights is None:
            self.weights = torch.ones((rank_normal + rank_spectral), dtype=self.dtype, requires_grad=False,
                                      device=device)
        else:
            self.weights = torch.tensor(weights, dtype=self.dtype, requires_grad=False, device=device)
        if softplus_kwargs is None:
            self.softplus_kwargs = {'beta': 50, 'threshold': 1}
        else:
            self.softplus_kwargs = softplus_kwargs
        self.rank_normal = rank_normal
        self.rank_spectral = rank_spectral
        self.rank = rank_normal + rank_spectral
        self.device = device
        if non_negative is True:
            self.non_negative = [True] * (len(X_shape))
        elif non_negative is False:
            self.non_negative = [False] * (len(X_shape))
        else:
            self.non_negative = non_negative
        self.bias = torch.zeros(y_shape[1:], dtype=self.dtype, requires_grad=True, device=device)
        self.y_shape = y_shape
        B_dims = list(X_shape[1:]) + list(y_shape[1:])
        complex_dims = list([n_complex_dim + 1] + [1] * (len(B_dims) - 1))
        if Bcp_init is None:
            self.Bcp_n = make_BcpInit(B_dims, self.rank_normal, self.non_negative, complex_dims=None,
                                      scale=Bcp_init_scale, device=self.device, dtype=self.dtype)
            self.Bcp_c = make_BcpInit(B_dims, self.rank_spectral, self.non_negative, complex_dims=complex_dims,
                                      scale=Bcp_init_scale, device=self.device, dtype=self.dtype)
            for ii in range(len(B_dims)):
                self.Bcp_n[ii].requires_grad = True
                self.Bcp_c[ii].requires_grad = True
        else:
            self.Bcp_n = Bcp_init[0]
            self.Bcp_c = Bcp_init[1]
        self.loss_running = []
        self._plan = None

    # ---- plumbing --------------------------------------------------------------------------
    def _shape(self):
        W, D, O = (int(self.Bcp_n[k].shape[0]) for k in range(3))
        return W, D, O, int(self.Bcp_n[0].shape[1]), int(self.Bcp_c[0].shape[1]), int(self.Bcp_c[0].shape[2])

    def _get_plan(self, X, rows):
        from .util import HostStream
        if isinstance(X, HostStream):
            rows = min(rows, X.chunk_rows)
        W, D, O, Rn, Rs, Cc = self._shape()
        if len(X.shape) != 3 or (int(X.shape[1]), int(X.shape[2])) != (W, D):
            raise ValueError(f"X must be (N, {W}, {D}) for these factors; got {tuple(X.shape)}")
        p = self._plan
        dev = _engine.device_index(X.device if isinstance(X, torch.Tensor) else f"cuda:{X.dev_index}")
        if (p is None or p.max_rows < rows or p.dims != (W, D, O)
                or (p.rank_normal, p.rank_spectral, p.n_complex) != (Rn, Rs, Cc) or p.dev != dev
                or p.nonlin != _engine.nonlin_key(self.non_negative, self.softplus_kwargs, 3)):
            p = SpectralPlan(W, D, O, Rn, Rs, Cc, rows, self.non_negative, self.softplus_kwargs, f"cuda:{dev}")
            self._plan = p
        return p

    def _inputs(self, X, y):
        if self.dtype != torch.float32:
            raise NotImplementedError(f"the gfx950 kernels compute in fp32; this model was built with "
                                      f"dtype={self.dtype}")
        from .util import HostStream
        if isinstance(X, HostStream):
            dev = X.dev_index
        else:
            dev = _engine.compute_device(X, self.device)
            X = _engine.as_device_rows(X, dev)
        y = torch.as_tensor(y)
        O = int(self.Bcp_n[2].shape[0])
        if y.ndim != 2 or y.shape[0] != X.shape[0] or y.shape[1] != O:
            raise ValueError(f"y must be (N, n_out) = ({X.shape[0]}, {O}); got {tuple(y.shape)}")
        if O == 1:
            raise NotImplementedError(
                "n_out == 1: the reference broadcasts lin_model's (N,) against the spectral term's (N, 1) "
                "into an (N, N) loss (SURVEY.md App. B-Q10); not reproduced by the gfx950 path")
        y = as_device_f32(y, dev)
        return X, y, dev

    def _arena(self, plan):
        return plan.pack(self.Bcp_n, self.Bcp_c, self.bias)

    def _weights(self, dev):
        return self.weights.to(f"cuda:{dev}", torch.float32).contiguous()

    def _set_grads(self, plan, gtot):
        views = plan.factor_views(gtot)
        for A, g in zip(list(self.Bcp_n) + list(self.Bcp_c), views):
            A.grad = g.to(A.device).clone()
        self.bias.grad = gtot[plan.offsets[6]:].to(self.bias.device).clone().view(self.bias.shape)

    # ---- fitting -----------------------------------------------------------------------------
    def fit(self, X, y, lambda_L2=0.01, max_iter=1000, tol=1e-5, patience=10, verbose=False,
            running_loss_logging_interval=10, LBFGS_kwargs=None):
        """LBFGS fit (spectral_tensor_regression.py:541-649): torch.optim.LBFGS drives the
        parameters, every closure evaluation is one gfx950 pass; logs the TOTAL loss (with L2)."""
        if LBFGS_kwargs is None:
            raise TypeError("torch.optim.lbfgs.LBFGS() argument after ** must be a mapping, not NoneType")
        X, y, dev = self._inputs(X, y)
        from .util import HostStream
        if isinstance(X, HostStream):
            raise NotImplementedError("the LBFGS fit needs X resident on the device (use fit_Adam for a HostStream)")
        N, O = X.shape[0], y.shape[1]
        plan = self._get_plan(X, N)
        optimizer = torch.optim.LBFGS(list(self.Bcp_n) + list(self.Bcp_c) + [self.bias], **LBFGS_kwargs)
        w = self._weights(dev)
        opts = dict(dtype=torch.float32, device=f"cuda:{dev}")
        grad = torch.zeros(plan.num_grads, **opts)
        gtot = torch.zeros(plan.num_params, **opts)
        loss_out = torch.zeros(1, **opts)
        norm = float(N * O)

        def total_loss(with_grads):
            arena = self._arena(plan)
            plan.loss_grad(X, y, None, norm, arena, w, grad)
            plan.finalize_grad(arena, grad, lambda_L2, gtot, loss_out)
            if with_grads:
                self._set_grads(plan, gtot)
            return loss_out[0].clone()

        def closure():
            optimizer.zero_grad()
            return total_loss(True)

        convergence_reached = False
        for ii in range(max_iter):
            if ii % running_loss_logging_interval == 0:
                self.loss_running.append(total_loss(False).item())
                if verbose == 2:
                    print(f'Iteration: {ii}, Loss: {self.loss_running[-1]}')
            if len(self.loss_running) > patience:
                if np.sum(np.abs(np.diff(self.loss_running[-patience + 1:]))) < tol:
                    convergence_reached = True
                    break
            elif np.isnan(self.loss_running[-1]):
                convergence_reached = False
                print('Loss is NaN. Stopping.')
                break
            optimizer.step(closure)
        if (verbose is True) or (verbose >= 1):
            print('Convergence reached' if convergence_reached else
                  'Reached maximum number of iterations without convergence')
        return convergence_reached

    def fit_Adam(self, X, y, lambda_L2=0.01, max_iter=1000, tol=1e-5, patience=10, verbose=False,
                 plotting_interval=100, Adam_kwargs=None, process_group=None):
        """Adam fit (spectral_tensor_regression.py:652-743), device resident on gfx950.

        process_group: optional torch.distributed group; X / y are then this rank's sample shard
        and the per-iteration gradient arena is summed with one all-reduce.
        """
        hp = adam_hparams(Adam_kwargs)
        from .util import HostStream

        def prepare():
            Xd, yd, dev = self._inputs(X, y)
            if verbose in (2, 3) and isinstance(Xd, HostStream):
                raise NotImplementedError("verbose=2/3 (per-iteration y_hat variance) is not offered for a HostStream X")
            return Xd, yd, dev, self._get_plan(Xd, Xd.shape[0])
        # under a process group one collective settles the start (_engine.fit_start): a rank-local
        # failure raises on every rank, the arena sizes agree, and the global sample count
        if process_group is None:
            X, y, dev, plan = prepare()
            n_global = float(X.shape[0])
        else:
            (X, y, dev, plan), n_global = _engine.fit_start(process_group, prepare, lambda o: o[0].shape[0],
                                                            lambda o: o[3].num_params)
        norm = n_global * y.shape[1]
        arena = self._arena(plan)
        w = self._weights(dev)
        vcb = _VerbosePrinter(plan, X, y, w, norm) if verbose in (2, 3) else None
        convergence_reached, _ = run_adam_fit(plan, X, y, None, norm, arena, w, lambda_L2, max_iter, tol, patience,
                                              hp, self.loss_running, verbose_cb=vcb, process_group=process_group,
                                              arena_checked=True)
        plan.unpack_into(arena, self.Bcp_n, self.Bcp_c, self.bias)
        if plan.last_stop < 0:
            print('Loss is NaN. Stopping.')
        if (verbose is True) or (verbose >= 1):
            print('Convergence reached' if convergence_reached else
                  'Reached maximum number of iterations without convergence')
        return convergence_reached

    ####################################
    ############ POST-HOC ##############
    ####################################

    def _factors_for(self, Bcp, device):
        if Bcp is None:
            return self.Bcp_n, self.Bcp_c
        Bcp_n, Bcp_c = list(Bcp[0]), list(Bcp[1])
        conv = (lambda a: torch.tensor(a, dtype=torch.float32, requires_grad=False).to(device)) \
            if isinstance(Bcp[0][0], torch.Tensor) is False else (lambda a: a.to(device))
        return [conv(a) for a in Bcp_n], [conv(a) for a in Bcp_c]

    def predict(self, X, Bcp=None, device=None, plot_pref=False):
        """lin_model + spectral_model (spectral_tensor_regression.py:895-963) as a CPU torch tensor."""
        if device is None:
            device = self.device
        if isinstance(X, torch.Tensor) is False:
            X = torch.tensor(X, dtype=torch.float32, requires_grad=False)
        Bcp_n, Bcp_c = self._factors_for(Bcp, device)
        dev = _engine.compute_device(X, device)
        Xd = _engine.as_device_rows(X, dev)
        plan = self._get_plan(Xd, Xd.shape[0])
        arena = plan.pack(Bcp_n, Bcp_c, self.bias)
        y_hat = plan.forward(Xd, arena, self._weights(dev))
        return y_hat.squeeze().cpu().detach() if y_hat.shape[0] == 1 else y_hat.cpu().detach()

    def predict_latents(self, X, Bcp=None, device=None, plot_pref=False):
        """stepwise_latents_model of the normal factors (spectral…py:966-1031), numpy (N, rank_normal)."""
        if device is None:
            device = self.device
        if isinstance(X, torch.Tensor) is False:
            X = torch.tensor(X, dtype=torch.float32, requires_grad=False)
        Bcp_n, Bcp_c = self._factors_for(Bcp, device)
        dev = _engine.compute_device(X, device)
        Xd = _engine.as_device_rows(X, dev)
        if int(Bcp_n[0].shape[1]) == 0:
            return torch.zeros(1).numpy()
        plan = self._get_plan(Xd, Xd.shape[0])
        arena = plan.pack(Bcp_n, Bcp_c, self.bias)
        return plan.latents(Xd, arena).cpu().numpy()

    def return_Bcp_final(self):
        """softplus-applied (Bcp_n, Bcp_c) as numpy lists (spectral…py:1034-1050)."""
        Bcp_n = list(non_neg_fn(self.Bcp_n, self.non_negative, softplus_kwargs=self.softplus_kwargs))
        Bcp_c = list(non_neg_fn(self.Bcp_c, self.non_negative, softplus_kwargs=self.softplus_kwargs))
        Bcp_n_nonNeg = [Bcp_n[ii].detach().cpu().numpy() for ii in range(len(Bcp_n))]
        Bcp_c_nonNeg = [Bcp_c[ii].detach().cpu().numpy() for ii in range(len(Bcp_c))]
        return Bcp_n_nonNeg, Bcp_c_nonNeg

    def detach_Bcp(self):
        Bcp_n_detached = [Bcp.detach().cpu().numpy() for Bcp in self.Bcp_n]
        Bcp_c_detached = [Bcp.detach().cpu().numpy() for Bcp in self.Bcp_c]
        return Bcp_n_detached, Bcp_c_detached

    def get_params(self):
        return {
            'weights': self.weights.detach().cpu().numpy(),
            'Bcp_n': self.detach_Bcp()[0],
            'Bcp_c': self.detach_Bcp()[1],
            'non_negative': self.non_negative,
            'softplus_kwargs': self.softplus_kwargs,
            'rank': self.rank,
            'device': self.device,
            'loss_running': self.loss_running}

    def set_params(self, params):
        """As the reference (spectral…py:1080-1090), which assigns params['Bcp'] to self.Bcp."""
        self.weights = params['weights']
        self.Bcp = params['Bcp']
        self.non_negative = params['non_negative']
        self.softplus_kwargs = params['softplus_kwargs']
        self.rank = params['rank']
        self.device = params['device']
        self.loss_running = params['loss_running']
        self._plan = None

    def display_params(self):
        print('weights:', self.weights)
        print('Bcp_n:', self.Bcp_n)
        print('Bcp_c:', self.Bcp_c)
        print('non_negative:', self.non_negative)
        print('softplus_kwargs:', self.softplus_kwargs)
        print('rank:', self.rank)
        print('device:', self.device)
        print('loss_running:', self.loss_running)

    def plot_outputs(self):
        import matplotlib.pyplot as plt
        plt.figure()
        plt.plot(self.loss_running)
        plt.xlabel('logged iteration')
        plt.ylabel('loss')
        plt.title('loss')
        Bcp_n_final, Bcp_c_final = self.return_Bcp_final()
        if self.rank_normal > 0:
            fig_n, axs = plt.subplots(len(Bcp_n_final))
            for ii, val in enumerate(Bcp_n_final):
                axs[ii].set_title(f'factor {ii + 1}')
                axs[ii].plot(val.squeeze())
            fig_n.suptitle('Bcp_n components')
        if self.rank_spectral > 0:
            fig_c, axs = plt.subplots(len(Bcp_c_final[1:]) + Bcp_c_final[0].shape[1])
            for jj in range(Bcp_c_final[0].shape[1]):
                axs[jj].plot(Bcp_c_final[0][:, jj, :].squeeze())
            for ii, val in enumerate(Bcp_c_final[1:]):
                axs[Bcp_c_final[0].shape[1] + ii].set_title(f'factor {ii + 2}')
                axs[Bcp_c_final[0].shape[1] + ii].plot(val.squeeze())
            fig_c.suptitle('Bcp_c components')
