"""CP linear tensor regression on MI355X — drop-in for the reference's
`standard_tensor_regression.py` (kimerein/tensor_regression).

Same module functions and `CP_linear_regression` class, same argument names, defaults,
Kruskal-factor list layout and `loss_running` semantics.  What changes is underneath:
the hot path — softplus + cp_to_tensor + inner(X, B) + MSELoss + backward + Adam
(standard_tensor_regression.py:458-470) — runs as gfx950 HIP kernels through the C ABI
(`include/tensor_regression_hip.h`), X is streamed from HBM once per iteration, and there is
no torch.autograd on that path.

Differences from the reference (all deliberate):
  * tensors must live on a HIP device (`device='cuda'`); the kernels compute in the model's
    dtype, float32 or float64 (dtype=torch.float64: a float64 two-pass path, csrc/tr_fp64.hip);
  * `lin_model` returns a non-differentiable tensor (the fit loops compute gradients in HIP);
  * a 2-D `y` is rejected (the reference silently broadcasts (N,) - (N,1) to (N,N), quirk Q11);
  * `fit_Adam` takes an optional `process_group` to fit sample shards over torch.distributed.
"""
import numpy as np
import torch

from . import _engine, _lib
from ._engine import Plan, as_device_f32, adam_hparams, run_adam_fit

__all__ = ["make_BcpInit", "non_neg_fn", "lin_model", "stepwise_model", "L2_penalty",
           "CP_linear_regression"]


####################################
######## Helper functions ##########
####################################

def make_BcpInit(B_dims, rank, non_negative, scale=1, device='cpu', dtype=torch.float32):
    """Initial Kruskal factors (standard_tensor_regression.py:18-51).

    Orthogonal init with gain `scale`, drawn on the CPU generator exactly like the reference
    (so the same torch seed gives the same factors), then non-negative factors shifted by two
    standard deviations and halved — only when the first factor has more than one row
    (reference quirk Q6).
    """
    Bcp_init = [torch.nn.init.orthogonal_(torch.empty(B_dims[ii], rank, dtype=dtype), gain=scale).to(device)
                for ii in range(len(B_dims))]
    if Bcp_init[0].shape[0] > 1:
        Bcp_init = [(Bcp_init[ii] + torch.std(Bcp_init[ii]) * 2 * non_negative[ii]) / (non_negative[ii] + 1)
                    for ii in range(len(Bcp_init))]
    return Bcp_init


def non_neg_fn(B_cp, non_negative, softplus_kwargs=None):
    """Yield softplus(A_k) for flagged factors, A_k otherwise (standard…py:53-85)."""
    if softplus_kwargs is None:
        softplus_kwargs = {'beta': 50, 'threshold': 1}
    for ii in range(len(B_cp)):
        if non_negative[ii]:
            yield torch.nn.functional.softplus(B_cp[ii], **softplus_kwargs)
        else:
            yield B_cp[ii]


_plan_cache = {}


def _plan_for(model, feature_dims, n_classes, rank, rows, non_negative, softplus_kwargs, device,
              dtype=torch.float32):
    nf = len(feature_dims) + (1 if model == _lib.TR_MODEL_MULTINOMIAL else 0)
    beta, thr = _engine.softplus_params(softplus_kwargs)
    key = (model, tuple(int(d) for d in feature_dims), int(n_classes), int(rank),
           tuple(bool(non_negative[f]) for f in range(nf)), beta, thr, _engine.device_index(device), dtype)
    p = _plan_cache.get(key)
    if p is None or p.max_rows < rows:
        p = Plan(model, feature_dims, n_classes, rank, rows, non_negative, softplus_kwargs, device, dtype=dtype)
        _plan_cache[key] = p
    return p


def lin_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """y_hat = inner(X, cp_to_tensor((weights, non_neg_fn(Bcp)))[..., None], n_modes=len(Bcp)) + bias

    (standard_tensor_regression.py:87-130), computed by the gfx950 forward kernel.
    X: (N, I_1..I_K) on a HIP device; returns (N,) fp32 (no autograd graph).
    """
    if not isinstance(X, torch.Tensor) or X.device.type != "cuda":
        raise ValueError("lin_model: X must be a torch tensor on a HIP device (device='cuda')")
    K = len(Bcp)
    if list(X.shape[1:]) != [int(A.shape[0]) for A in Bcp] or X.ndim != K + 1:
        raise ValueError(f"Incorrect shapes for inner product along {K} common modes. "
                         f"tensor_1.shape={list(X.shape)}, factors={[tuple(A.shape) for A in Bcp]}")
    rank = int(Bcp[0].shape[1])
    dev = X.device
    dtype = X.dtype
    for A in Bcp:  # inner(X, B) is one matmul in the reference: operands of one dtype
        if torch.as_tensor(A).dtype != dtype:
            raise RuntimeError(f"expected m1 and m2 to have the same dtype, but got: {dtype} != "
                               f"{torch.as_tensor(A).dtype}")
    Xd = _engine.as_device_rows(X, dev.index, dtype)
    plan = _plan_for(_lib.TR_MODEL_LINEAR, X.shape[1:], 1, rank, 1, non_negative, softplus_kwargs, dev, dtype)
    arena = plan.pack([torch.as_tensor(A).to(dev) for A in Bcp], torch.as_tensor(bias).to(dev))
    w = torch.as_tensor(weights, dtype=dtype).to(dev).contiguous()
    return plan.forward(Xd, arena, w)


def stepwise_model(X, Bcp, weights, non_negative, bias, softplus_kwargs=None):
    """einsum form of lin_model for 3-D X (standard…py:133-177): the reference ignores
    `weights` here, i.e. it is lin_model with unit weights."""
    if Bcp[0].shape[1] == 0:
        return torch.zeros(1).to(X.device)
    rank = int(Bcp[0].shape[1])
    return lin_model(X, Bcp, torch.ones(rank, device=X.device), non_negative, bias, softplus_kwargs)


def L2_penalty(B_cp):
    """sum_k ||A_k||_F of the raw factors, not squared (standard…py:180-196)."""
    ii = 0
    for comp in B_cp:
        ii += torch.sqrt(torch.sum(comp ** 2))
    return ii


class _VerbosePrinter:
    """verbose==2 per-iteration print of the reference (standard…py:465-466)."""

    def __init__(self, plan, X, y, weights):
        self.plan, self.X, self.weights = plan, X, weights
        self.var_y = torch.var(y).item()
        self.yhat = None

    def before_step(self, arena):
        self.yhat = self.plan.forward(self.X, arena, self.weights)

    def after_step(self, ii, loss):
        ratio = torch.var(self.yhat).item() / self.var_y
        print(f'Iteration: {ii}, Loss: {loss}  ;  Variance ratio (y_hat / y_true): {ratio}')


####################################
########### Main class #############
####################################

class CP_linear_regression():
    def __init__(self,
                 X_shape,
                 dtype=torch.float32,
                 rank=5,
                 non_negative=False,
                 weights=None,
                 Bcp_init=None,
                 Bcp_init_scale=1,
                 bias_init=0,
                 device='cpu',
                 softplus_kwargs=None):
        """CP linear regression y = <X, [[weights; softplus?(Bcp)]]> + bias
        (standard_tensor_regression.py:204-303; same arguments and attributes)."""
        self.dtype = dtype
        if weights is None:
            self.weights = torch.ones((rank), dtype=self.dtype, requires_grad=False, device=device)
        else:
            self.weights = torch.tensor(weights, dtype=self.dtype, requires_grad=False, device=device)
        if softplus_kwargs is None:
            self.softplus_kwargs = {'beta': 50, 'threshold': 1}
        else:
            self.softplus_kwargs = softplus_kwargs
        self.rank = rank
        self.device = device
        if non_negative is True:
            self.non_negative = [True] * (len(X_shape))
        elif non_negative is False:
            self.non_negative = [False] * (len(X_shape))
        else:
            self.non_negative = non_negative
        self.bias = torch.tensor([bias_init], dtype=self.dtype, requires_grad=True, device=device)
        B_dims = list(X_shape[1:])
        if Bcp_init is None:
            self.Bcp = make_BcpInit(B_dims, self.rank, self.non_negative, scale=Bcp_init_scale,
                                    device=self.device, dtype=self.dtype)
            for ii in range(len(B_dims)):
                self.Bcp[ii].requires_grad = True
        else:
            self.Bcp = Bcp_init
        self.loss_running = []
        self._plan = None

    # ---- plumbing --------------------------------------------------------------------------
    def _check_dtype(self):
        if self.dtype not in (torch.float32, torch.float64):
            raise NotImplementedError(f"the gfx950 kernels compute in float32 or float64; this model was built "
                                      f"with dtype={self.dtype}")

    def _get_plan(self, X, rows):
        from .util import HostStream
        if isinstance(X, HostStream):
            rows = min(rows, X.chunk_rows)
        dims = [int(A.shape[0]) for A in self.Bcp]
        if list(X.shape[1:]) != dims:
            raise ValueError(f"Incorrect shapes for inner product along {len(dims)} common modes. "
                             f"tensor_1.shape={list(X.shape)}, factors={[tuple(A.shape) for A in self.Bcp]}")
        p = self._plan
        dev = _engine.device_index(X.device if isinstance(X, torch.Tensor) else f"cuda:{X.dev_index}")
        if (p is None or p.max_rows < rows or p.feature_dims != dims or p.rank != int(self.Bcp[0].shape[1])
                or p.dev != dev or p.dtype != self.dtype
                or p.nonlin != _engine.nonlin_key(self.non_negative, self.softplus_kwargs, len(dims))):
            p = Plan(_lib.TR_MODEL_LINEAR, dims, 1, int(self.Bcp[0].shape[1]), rows, self.non_negative,
                     self.softplus_kwargs, f"cuda:{dev}", dtype=self.dtype)
            self._plan = p
        return p

    def _inputs(self, X, y):
        self._check_dtype()
        from .util import HostStream
        if isinstance(X, HostStream):  # out-of-core: X streams from host memory every iteration
            if self.dtype != torch.float32:
                raise NotImplementedError("HostStream streams float32 samples; this model is float64")
            dev = X.dev_index
            y = torch.as_tensor(y)
            if y.ndim != 1 or y.shape[0] != len(X):
                raise ValueError(f"y must be 1-D with len(y) == len(X); got y.shape={tuple(y.shape)}")
            return X, as_device_f32(y, dev), dev
        dev = _engine.compute_device(X, self.device)
        X = _engine.as_device_rows(X, dev, self.dtype)
        y = torch.as_tensor(y)
        if y.ndim != 1 or y.shape[0] != X.shape[0]:
            raise ValueError(f"y must be 1-D with len(y) == X.shape[0]; got y.shape={tuple(y.shape)}, "
                             f"X.shape[0]={X.shape[0]}")
        y = as_device_f32(y, dev, self.dtype)
        return X, y, dev

    # ---- fitting -----------------------------------------------------------------------------
    def fit(self, X, y, lambda_L2=0.01, max_iter=1000, tol=1e-5, patience=10, verbose=False,
            running_loss_logging_interval=10, LBFGS_kwargs=None):
        """LBFGS fit (standard_tensor_regression.py:305-398).  torch.optim.LBFGS drives the
        parameters; every closure evaluation is one gfx950 loss+gradient pass."""
        if LBFGS_kwargs is None:
            raise TypeError("torch.optim.lbfgs.LBFGS() argument after ** must be a mapping, not NoneType")
        X, y, dev = self._inputs(X, y)
        from .util import HostStream
        if isinstance(X, HostStream):
            raise NotImplementedError("the LBFGS fit needs X resident on the device (use fit_Adam for a HostStream)")
        N = X.shape[0]
        plan = self._get_plan(X, N)
        params = self.Bcp + [self.bias]
        optimizer = torch.optim.LBFGS(params, **LBFGS_kwargs)
        w = self.weights.to(f"cuda:{dev}", self.dtype).contiguous()
        opts = dict(dtype=self.dtype, device=f"cuda:{dev}")
        grad = torch.zeros(plan.num_grads, **opts)
        gtot = torch.zeros(plan.num_params, **opts)
        loss_out = torch.zeros(1, **opts)

        def closure():
            optimizer.zero_grad()
            arena = plan.pack(self.Bcp, self.bias)
            plan.loss_grad_checked(X, y, None, float(N), arena, w, grad)
            plan.finalize_grad(arena, grad, lambda_L2, gtot, loss_out)
            views = plan.factor_views(gtot)
            for A, g in zip(self.Bcp, views):
                A.grad = g.to(A.device).clone()
            self.bias.grad = gtot[plan.offsets[-1]:].to(self.bias.device).clone().view(self.bias.shape)
            return loss_out[0].clone()

        convergence_reached = False
        for ii in range(max_iter):
            if ii % running_loss_logging_interval == 0:
                arena = plan.pack(self.Bcp, self.bias)
                y_hat = plan.forward(X, arena, w)
                self.loss_running.append(torch.mean((y_hat - y) ** 2).item())
                if verbose == 2:
                    print(f'Iteration: {ii}, Loss: {self.loss_running[-1]}  ;  Variance ratio (y_hat / y_true): '
                          f'{torch.var(y_hat).item() / torch.var(y).item()}')
            if ii > patience:
                if np.sum(np.abs(np.diff(self.loss_running[ii - patience:]))) < tol:
                    convergence_reached = True
                    break
            optimizer.step(closure)
        plan.check_status()
        if (verbose is True) or (verbose >= 1):
            print('Convergence reached' if convergence_reached else
                  'Reached maximum number of iterations without convergence')
        return convergence_reached

    def fit_Adam(self, X, y, lambda_L2=0.01, max_iter=1000, tol=1e-5, patience=10, verbose=False,
                 Adam_kwargs=None, process_group=None):
        """Adam fit (standard_tensor_regression.py:400-476), device resident on gfx950.

        X: a device tensor (samples may be a strided / windowed view, util.windowed_view) or a
        util.HostStream (host-resident X streamed through HBM in chunks every iteration).
        process_group: optional torch.distributed group; X / y are then this rank's sample
        shard and the per-iteration gradient arena is summed with one all-reduce.
        """
        hp = adam_hparams(Adam_kwargs)
        from .util import HostStream

        def prepare():
            Xd, yd, dev = self._inputs(X, y)
            if verbose == 2 and isinstance(Xd, HostStream):
                raise NotImplementedError("verbose=2 (per-iteration y_hat variance) is not offered for a HostStream X")
            return Xd, yd, dev, self._get_plan(Xd, Xd.shape[0])
        # under a process group one collective settles the start (_engine.fit_start): a rank-local
        # failure raises on every rank, the arena sizes agree, and the global sample count
        if process_group is None:
            X, y, dev, plan = prepare()
            n_global = float(X.shape[0])
        else:
            (X, y, dev, plan), n_global = _engine.fit_start(process_group, prepare, lambda o: o[0].shape[0],
                                                            lambda o: o[3].num_params)
        arena = plan.pack(self.Bcp, self.bias)
        w = self.weights.to(f"cuda:{dev}", self.dtype).contiguous()
        vcb = _VerbosePrinter(plan, X, y, w) if verbose == 2 else None
        convergence_reached, _ = run_adam_fit(plan, X, y, None, n_global, arena, w, lambda_L2, max_iter, tol,
                                              patience, hp, self.loss_running, verbose_cb=vcb,
                                              process_group=process_group, arena_checked=True)
        plan.unpack_into(arena, self.Bcp, self.bias)
        if (verbose is True) or (verbose >= 1):
            print('Convergence reached' if convergence_reached else
                  'Reached maximum number of iterations without convergence')
        return convergence_reached

    ####################################
    ############ POST-HOC ##############
    ####################################

    def predict(self, X, Bcp=None, device=None, plot_pref=False):
        """y_hat as numpy (standard_tensor_regression.py:628-687); inputs are cast to fp32
        like the reference (quirk Q12)."""
        if device is None:
            device = self.device
        if isinstance(X, torch.Tensor) is False:
            X = torch.tensor(X, dtype=torch.float32, requires_grad=False).to(device)
        elif X.device != torch.device(device):
            X = X.to(device)
        if Bcp is None:
            Bcp = self.Bcp
        elif isinstance(Bcp[0], torch.Tensor) is False:
            for ii in range(len(Bcp)):
                Bcp[ii] = torch.tensor(Bcp[ii], dtype=torch.float32, requires_grad=False).to(device)
        elif Bcp[0].device != torch.device(device):
            for ii in range(len(Bcp)):
                Bcp[ii] = Bcp[ii].to(device)
        y_hat = lin_model(X, Bcp, self.weights, self.non_negative, self.bias,
                          softplus_kwargs=self.softplus_kwargs).detach().cpu().numpy()
        return y_hat

    def return_Bcp_final(self):
        """softplus-applied factors as numpy (standard…py:690-703)."""
        Bcp = list(non_neg_fn(self.Bcp, self.non_negative, softplus_kwargs=self.softplus_kwargs))
        return [Bcp[ii].detach().cpu().numpy() for ii in range(len(Bcp))]

    def detach_Bcp(self):
        return [Bcp.detach().cpu().numpy() for Bcp in self.Bcp]

    def get_params(self):
        return {
            'weights': self.weights.detach().cpu().numpy(),
            'Bcp': self.detach_Bcp(),
            'non_negative': self.non_negative,
            'softplus_kwargs': self.softplus_kwargs,
            'rank': self.rank,
            'device': self.device,
            'loss_running': self.loss_running}

    def set_params(self, params):
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
        print('Bcp:', self.Bcp)
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
        Bcp_final = self.return_Bcp_final()
        fig, axs = plt.subplots(len(Bcp_final))
        for ii, val in enumerate(Bcp_final):
            axs[ii].set_title(f'factor {ii}')
            axs[ii].plot(val)
        fig.suptitle('components')
