"""CP multinomial logistic tensor regression on MI355X — drop-in for the reference's
`multinomial_tensor_regression.py` (kimerein/tensor_regression).

Same helpers, `model`, `CP_logistic_regression` class and semantics — including the
reference's double softmax (the model returns probabilities and CrossEntropyLoss applies
log-softmax to them again, multinomial_tensor_regression.py:180-187 + :448-450) — with the
hot path (factor prep, X·B over all classes, softmax, weighted CE, X^T·dZ, MTTKRP, Adam)
running as gfx950 HIP kernels through the C ABI.
"""
import numpy as np
import torch

from . import _engine, _lib
from ._engine import Plan, as_device_f32, adam_hparams, run_adam_fit
from .standard_tensor_regression import _plan_for, L2_penalty  # noqa: F401  (L2_penalty re-exported)

__all__ = ["squeeze_integers", "confusion_matrix", "idx_to_oneHot", "make_BcpInit", "non_neg_fn", "model",
           "L2_penalty", "CP_logistic_regression"]


####################################
######## Useful functions ##########
####################################

def squeeze_integers(intVec):
    """Relabel integers to consecutive ids from 0 (multinomial…py:18-37)."""
    intVec = np.asarray(intVec)
    uniques = np.unique(intVec)
    return np.searchsorted(uniques, intVec)


def confusion_matrix(y_hat, y_true):
    """Column-normalised confusion matrix (multinomial…py:45-65)."""
    n_classes = np.max(y_true) + 1
    if y_hat.ndim == 1:
        y_hat = idx_to_oneHot(y_hat, n_classes)
    cmat = y_hat.T @ idx_to_oneHot(y_true, n_classes)
    return cmat / np.sum(cmat, axis=0)[None, :]


def idx_to_oneHot(arr, n_classes=None):
    """(multinomial…py:67-86)"""
    if n_classes is None:
        n_classes = np.max(arr) + 1
    oneHot = np.zeros((arr.size, n_classes))
    oneHot[np.arange(arr.size), arr] = 1
    return oneHot


def make_BcpInit(B_dims, rank, non_negative, scale=1, device='cpu'):
    """Uniform init rand*scale - (1-nn)*scale/2, requires_grad (multinomial…py:88-114)."""
    Bcp_init = [(torch.rand((B_dims[ii], rank)) * scale - (1 - non_negative[ii]) * (scale / 2)).to(device)
                for ii in range(len(B_dims))]
    for ii in range(len(B_dims)):
        Bcp_init[ii].requires_grad = True
    return Bcp_init


def non_neg_fn(B_cp, non_negative, softplus_kwargs=None):
    """(multinomial…py:116-146)"""
    if softplus_kwargs is None:
        softplus_kwargs = {'beta': 50, 'threshold': 1}
    for ii in range(len(B_cp)):
        if non_negative[ii]:
            yield torch.nn.functional.softplus(B_cp[ii], **softplus_kwargs)
        else:
            yield B_cp[ii]


def model(X, Bcp, weights, non_negative, softplus_kwargs=None):
    """softmax(inner(X, cp_to_tensor((weights, non_neg_fn(Bcp))), n_modes=len(Bcp)-1), dim=1)
    (multinomial_tensor_regression.py:148-187) on the gfx950 forward kernel; returns (N, C)."""
    if not isinstance(X, torch.Tensor) or X.device.type != "cuda":
        raise ValueError("model: X must be a torch tensor on a HIP device (device='cuda')")
    K = len(Bcp) - 1
    if X.ndim != K + 1 or list(X.shape[1:]) != [int(A.shape[0]) for A in Bcp[:-1]]:
        raise ValueError(f"Incorrect shapes for inner product along {K} common modes. "
                         f"tensor_1.shape={list(X.shape)}, factors={[tuple(A.shape) for A in Bcp]}")
    dev = X.device
    C, rank = int(Bcp[-1].shape[0]), int(Bcp[0].shape[1])
    plan = _plan_for(_lib.TR_MODEL_MULTINOMIAL, X.shape[1:], C, rank, 1, non_negative, softplus_kwargs, dev)
    arena = plan.pack([torch.as_tensor(A).to(dev) for A in Bcp])
    w = torch.as_tensor(weights, dtype=torch.float32).to(dev).contiguous()
    return plan.forward(_engine.as_device_rows(X, dev.index), arena, w)


####################################
########### Main class #############
####################################

class CP_logistic_regression():
    def __init__(self, X, y, rank=5, non_negative=False, weights=None, Bcp_init=None, Bcp_init_scale=1,
                 device='cpu', softplus_kwargs=None):
        """(multinomial_tensor_regression.py:212-286; same arguments and attributes).  X may also
        be a util.HostStream (host-resident X streamed through HBM every iteration; fit_Adam and
        predict only)."""
        from .util import HostStream
        self.X = X if isinstance(X, HostStream) else torch.as_tensor(X, dtype=torch.float32).to(device)
        self.y = torch.as_tensor(y, dtype=torch.long).to(device)
        if weights is None:
            self.weights = torch.ones((rank), device=device)
        else:
            self.weights = torch.tensor(weights)
        if softplus_kwargs is None:
            self.softplus_kwargs = {'beta': 50, 'threshold': 1}
        else:
            self.softplus_kwargs = softplus_kwargs
        self.rank = rank
        self.device = device
        if non_negative is True:
            self.non_negative = [True] * (self.X.ndim)
        elif non_negative is False:
            self.non_negative = [False] * (self.X.ndim)
        else:
            self.non_negative = non_negative
        self.n_classes = len(torch.unique(self.y))
        B_dims = np.concatenate((np.array(self.X.shape[1:]), [self.n_classes]))
        # a class factor drawn here from the LOCAL labels may be widened to the global class set
        # by a sharded fit_Adam (_sync_class_set); one passed in by the caller is never resized
        self._class_factor_auto = Bcp_init is None
        self._Bcp_init_scale = Bcp_init_scale
        if Bcp_init is None:
            self.Bcp = make_BcpInit(B_dims, self.rank, self.non_negative, scale=Bcp_init_scale, device=self.device)
        else:
            self.Bcp = Bcp_init
        self.loss_running = []
        self._plan = None
        self._dev_cache = None

    def return_self(self):
        return self.Bcp

    # ---- plumbing ------------------------------------------------------------------------------
    def _device_data(self):
        from .util import HostStream
        hs = isinstance(self.X, HostStream)
        dev = self.X.dev_index if hs else _engine.compute_device(self.X, self.device)
        c = self._dev_cache
        if c is None or c[0] != dev or c[1] is not self.X or c[2] is not self.y:
            Xd = self.X if hs else _engine.as_device_rows(self.X, dev)
            yd = self.y.to(f"cuda:{dev}", torch.long).contiguous()
            C = int(self.Bcp[-1].shape[0])
            ymin, ymax = int(yd.min().item()), int(yd.max().item())
            if ymin < 0 or ymax >= C:
                raise IndexError(f"Target {ymax if ymax >= C else ymin} is out of bounds.")
            self._dev_cache = (dev, self.X, self.y, Xd, yd)
        return self._dev_cache[0], self._dev_cache[3], self._dev_cache[4]

    def _get_plan(self, Xd, rows):
        from .util import HostStream
        if isinstance(Xd, HostStream):
            rows = min(rows, Xd.chunk_rows)
        dims = [int(A.shape[0]) for A in self.Bcp[:-1]]
        if list(Xd.shape[1:]) != dims:
            raise ValueError(f"Incorrect shapes for inner product along {len(dims)} common modes. "
                             f"tensor_1.shape={list(Xd.shape)}, factors={[tuple(A.shape) for A in self.Bcp]}")
        C, R = int(self.Bcp[-1].shape[0]), int(self.Bcp[0].shape[1])
        p = self._plan
        if (p is None or p.max_rows < rows or p.feature_dims != dims or p.n_classes != C or p.rank != R
                or p.dev != _engine.device_index(Xd.device)
                or p.nonlin != _engine.nonlin_key(self.non_negative, self.softplus_kwargs, len(dims) + 1)):
            p = Plan(_lib.TR_MODEL_MULTINOMIAL, dims, C, R, rows, self.non_negative, self.softplus_kwargs,
                     Xd.device)
            self._plan = p
        return p

    def _sync_class_set(self, process_group):
        """The class set of a sample-sharded fit is the union of every rank's labels.

        The reference takes n_classes = len(unique(y)) from the data it is given
        (multinomial_tensor_regression.py:279-280) and CrossEntropyLoss then requires every label
        to be < n_classes.  A rank's shard may miss classes, so under a process group the count is
        taken from all ranks' labels (MAX all-reduce of the label range, then of a presence
        bitmap), and every rank raises the reference's own error when the union is not
        0..C-1 — the same error a single process on the concatenated data would raise.  A class
        factor this model drew from its local labels is widened to the global count (the new rows
        drawn like make_BcpInit's); the fit then starts every rank from group rank 0's parameters
        (sync_replicas).  A caller's Bcp_init keeps its shape, and must cover the labels."""
        import torch.distributed as dist
        cdev = _engine.collective_device(process_group)
        y = torch.as_tensor(self.y).reshape(-1).to(cdev, torch.long)
        n = y.numel()
        # label range and every rank's sample count in one MAX all-reduce (the counts in per-rank
        # slots, -1 elsewhere)
        world, me = dist.get_world_size(process_group), dist.get_rank(process_group)
        rng = torch.full((2 + world,), -1, dtype=torch.int64)
        rng[0], rng[1], rng[2 + me] = (int(y.max()) if n else -1), (-int(y.min()) if n else 0), n
        rng = rng.to(cdev)
        dist.all_reduce(rng, op=dist.ReduceOp.MAX, group=process_group)
        r = rng.tolist()
        ymax, ymin, n_all = r[0], -r[1], sum(r[2:])
        if n_all == 0:
            raise ValueError("the sharded multinomial fit got no samples on any rank")
        if ymin < 0:
            raise IndexError(f"Target {ymin} is out of bounds.")
        if ymax >= n_all:  # fewer samples than label values: the union cannot be 0..ymax
            raise IndexError(f"Target {ymax} is out of bounds.")
        present = torch.zeros(ymax + 1, dtype=torch.int32, device=cdev)
        if n:
            present[y] = 1
        dist.all_reduce(present, op=dist.ReduceOp.MAX, group=process_group)
        C = int(present.sum())
        if self._class_factor_auto:
            if C != ymax + 1:  # reference: n_classes = C < ymax + 1 -> label ymax out of bounds
                raise IndexError(f"Target {ymax} is out of bounds.")
            A = self.Bcp[-1]
            if int(A.shape[0]) != C:
                extra = (torch.rand((C - int(A.shape[0]), self.rank)) * self._Bcp_init_scale
                         - (1 - self.non_negative[-1]) * (self._Bcp_init_scale / 2)).to(A.device)
                with torch.no_grad():
                    self.Bcp[-1] = torch.cat([A.detach(), extra.to(A.dtype)], dim=0).requires_grad_(True)
                self._plan = None
                self._dev_cache = None
                self._cw_cache = None
            self.n_classes = C
        Cm = int(self.Bcp[-1].shape[0])
        _engine.check_uniform(Cm, process_group, "the number of classes (class-factor rows)", cdev)
        if ymax >= Cm:
            raise IndexError(f"Target {ymax} is out of bounds.")

    def _class_weights(self, weights, dev, yd):
        """The class weights on the device and this rank's CE normaliser sum_n w[y_n].  Both are
        kept for the next fit on the same labels and weights (the normaliser costs a reduction
        over the labels and a host synchronisation)."""
        cwh = torch.as_tensor(weights, dtype=torch.float32).detach().cpu()
        C = int(self.Bcp[-1].shape[0])
        if cwh.ndim != 1 or cwh.numel() != C:
            raise RuntimeError(f"weight tensor should be defined either for all {C} classes or no classes "
                               f"but got weight tensor of shape: {list(cwh.shape)}")
        key = (yd, yd._version, dev, cwh.numpy().tobytes())
        c = getattr(self, "_cw_cache", None)
        if c is not None and c[0] is key[0] and c[1:4] == key[1:]:
            return c[4], c[5]
        cw = cwh.to(f"cuda:{dev}").contiguous()
        W = float(cw.double()[yd].sum().item())
        self._cw_cache = key + (cw, W)
        return cw, W

    # ---- fitting -------------------------------------------------------------------------------
    def fit(self, lambda_L2=0.01, max_iter=1000, tol=1e-5, patience=10, weights=None, verbose=False,
            running_loss_logging_interval=10, LBFGS_kwargs=None):
        """LBFGS fit (multinomial_tensor_regression.py:291-387); closures evaluated on gfx950."""
        if LBFGS_kwargs is None:
            raise TypeError("torch.optim.lbfgs.LBFGS() argument after ** must be a mapping, not NoneType")
        dev, Xd, yd = self._device_data()
        if not isinstance(Xd, torch.Tensor):
            raise NotImplementedError("the LBFGS fit needs X resident on the device (use fit_Adam for a HostStream)")
        plan = self._get_plan(Xd, Xd.shape[0])
        cw, W = self._class_weights(weights, dev, yd)
        optimizer = torch.optim.LBFGS(self.Bcp, **LBFGS_kwargs)
        w = self.weights.to(f"cuda:{dev}", torch.float32).contiguous()
        opts = dict(dtype=torch.float32, device=f"cuda:{dev}")
        grad = torch.zeros(plan.num_grads, **opts)
        gtot = torch.zeros(plan.num_params, **opts)
        loss_out = torch.zeros(1, **opts)

        def closure():
            optimizer.zero_grad()
            arena = plan.pack(self.Bcp)
            plan.loss_grad(Xd, yd, cw, W, arena, w, grad)
            plan.finalize_grad(arena, grad, lambda_L2, gtot, loss_out)
            for A, g in zip(self.Bcp, plan.factor_views(gtot)):
                A.grad = g.to(A.device).clone()
            return loss_out[0].clone()

        convergence_reached = False
        for ii in range(max_iter):
            if ii % running_loss_logging_interval == 0:
                arena = plan.pack(self.Bcp)
                plan.loss_grad(Xd, yd, cw, W, arena, w, grad)  # data loss only (reference :372)
                self.loss_running.append(float(grad[plan.num_params].item()))
                if verbose == 2:
                    print(f'Iteration: {ii}, Loss: {self.loss_running[-1]}')
            if ii > patience:
                if np.sum(np.abs(np.diff(self.loss_running[ii - patience:]))) < tol:
                    convergence_reached = True
                    break
            optimizer.step(closure)
        if (verbose is True) or (verbose >= 1):
            print('Convergence reached' if convergence_reached else
                  'Reached maximum number of iterations without convergence')
        return convergence_reached

    def fit_Adam(self, lambda_L2=0.01, max_iter=1000, tol=1e-5, patience=10, weights=None, verbose=False,
                 Adam_kwargs=None, process_group=None):
        """Adam fit (multinomial_tensor_regression.py:389-471), device resident on gfx950.

        process_group: optional torch.distributed group; self.X / self.y are then this rank's
        sample shard (the CE normaliser sum_n w[y_n] is all-reduced once)."""
        hp = adam_hparams(Adam_kwargs)

        def prepare():
            dev, Xd, yd = self._device_data()
            plan = self._get_plan(Xd, Xd.shape[0])
            cw, W = self._class_weights(weights, dev, yd)
            return dev, Xd, yd, plan, cw, W
        if process_group is None:
            dev, Xd, yd, plan, cw, W = prepare()
        else:
            # collectives first, then the rank-local checks with a collective verdict: a failure on
            # one rank raises on every rank instead of leaving the others in a later all-reduce
            self._sync_class_set(process_group)
            (dev, Xd, yd, plan, cw, _), W = _engine.fit_start(process_group, prepare, lambda o: o[5],
                                                              lambda o: o[3].num_params)
        arena = plan.pack(self.Bcp)
        w = self.weights.to(f"cuda:{dev}", torch.float32).contiguous()
        vcb = _Verbose() if verbose == 2 else None
        convergence_reached, _ = run_adam_fit(plan, Xd, yd, cw, W, arena, w, lambda_L2, max_iter, tol, patience,
                                              hp, self.loss_running, verbose_cb=vcb, process_group=process_group,
                                              arena_checked=True)
        plan.unpack_into(arena, self.Bcp)
        if (verbose is True) or (verbose >= 1):
            print('Convergence reached' if convergence_reached else
                  'Reached maximum number of iterations without convergence')
        return convergence_reached

    def predict(self, X=None, y_true=None, Bcp=None, device=None):
        """(probabilities, argmax) as numpy (multinomial…py:474-545); the 'logit' the reference
        returns is the softmax output (quirk Q2)."""
        from .util import HostStream
        if device is None:
            device = self.device
        if X is None:
            X = self.X
        if isinstance(X, HostStream):  # chunk by chunk through the same forward kernel
            Bd = [torch.as_tensor(A).to(f"cuda:{X.dev_index}") for A in (self.Bcp if Bcp is None else Bcp)]
            logit = torch.cat([model(Xc, Bd, self.weights, self.non_negative, softplus_kwargs=self.softplus_kwargs)
                               for _, _, Xc in X.chunks()]).detach().cpu().numpy()
            return logit, np.argmax(logit, axis=1)
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
        dev = _engine.compute_device(X, device)
        Xd = _engine.as_device_rows(X, dev)
        logit = model(Xd, [torch.as_tensor(A).to(f"cuda:{dev}") for A in Bcp], self.weights, self.non_negative,
                      softplus_kwargs=self.softplus_kwargs).detach().cpu().numpy()
        pred = np.argmax(logit, axis=1)
        return logit, pred

    def return_Bcp_final(self):
        Bcp = list(non_neg_fn(self.Bcp, self.non_negative, softplus_kwargs=self.softplus_kwargs))
        return [Bcp[ii].detach().cpu().numpy() for ii in range(len(Bcp))]

    def make_confusion_matrix(self, prob_or_pred='pred', prob=None, pred=None, y_true=None):
        """(multinomial…py:562-597)"""
        if (prob is None) and (pred is None):
            prob, pred = self.predict()
        if y_true is None:
            y_true = self.y.detach().cpu().numpy()
        if prob_or_pred == 'pred':
            cm = confusion_matrix(pred, y_true)
        elif prob_or_pred == 'prob':
            cm = confusion_matrix(prob, y_true)
        acc = np.sum(np.diag(cm)) / np.sum(cm)
        return cm, acc

    def detach_Bcp(self):
        return [Bcp.detach().cpu().numpy() for Bcp in self.Bcp]

    def get_params(self):
        # the reference reads a nonexistent self.bias here (quirk Q4); the working subset is returned
        X = self.X.X if not isinstance(self.X, torch.Tensor) else self.X  # HostStream: its host tensor
        return {'X': X.detach().cpu().numpy(),
                'y': self.y.detach().cpu().numpy(),
                'weights': self.weights.detach().cpu().numpy(),
                'Bcp': self.detach_Bcp(),
                'non_negative': self.non_negative,
                'softplus_kwargs': self.softplus_kwargs,
                'rank': self.rank,
                'device': self.device,
                'loss_running': self.loss_running}

    def set_params(self, params):
        self.X = params['X']
        self.y = params['y']
        self.weights = params['weights']
        self.Bcp = params['Bcp']
        if 'bias' in params:
            self.bias = params['bias']
        self.non_negative = params['non_negative']
        self.softplus_kwargs = params['softplus_kwargs']
        self.rank = params['rank']
        self.device = params['device']
        self.loss_running = params['loss_running']
        self._plan = None
        self._dev_cache = None
        self._cw_cache = None

    def display_params(self):
        print('X:', self.X.shape)
        print('y:', self.y.shape)
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
        logit, pred = self.predict()
        fig, axs = plt.subplots(2)
        axs[0].imshow(idx_to_oneHot(pred, self.n_classes), aspect='auto', interpolation='none')
        axs[1].imshow(idx_to_oneHot(self.y.detach().cpu().numpy(), self.n_classes), aspect='auto',
                      interpolation='none')
        axs[1].set_xlabel('class')
        fig.suptitle('predictions')
        cm, acc = self.make_confusion_matrix(prob_or_pred='pred')
        fig = plt.figure()
        plt.imshow(cm)
        plt.ylabel('true class')
        plt.xlabel('predicted class')
        plt.title('confusion matrix (predictions)')
        Bcp_final = self.return_Bcp_final()
        fig, axs = plt.subplots(len(Bcp_final))
        for ii, val in enumerate(Bcp_final):
            axs[ii].set_title(f'factor {ii}')
            axs[ii].plot(val)
        fig.suptitle('components')


class _Verbose:
    """verbose==2 print of the multinomial fit_Adam (multinomial…py:460-461)."""

    def before_step(self, arena):
        pass

    def after_step(self, ii, loss):
        print(f'Iteration: {ii}, Loss: {loss}')
