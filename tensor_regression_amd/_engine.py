"""Host-side engine: one gfx950 plan per model shape, the packed parameter arena and the
device-resident fit loop shared by CP_linear_regression and CP_logistic_regression.

Everything on the hot path goes through the C ABI (include/tensor_regression_hip.h); torch is
used only for device memory, the current HIP stream and torch.distributed.  The reference's
per-iteration `loss.item()` host sync (standard_tensor_regression.py:464) is replaced by a
device loss history plus a device stop flag (the plateau test of :467-470 runs on the GPU), so
the host enqueues `sync_every` iterations between synchronisations.
"""
import atexit
import ctypes
import math
import os
import sys
import weakref

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

_DEFAULT_SOFTPLUS = {"beta": 50, "threshold": 1}
# fit_Adam: fold the next iteration's factor preparation into each Adam step (tests toggle it)
_PREPARE_NEXT = os.environ.get("TR_NO_PREPARE_NEXT", "0") in ("", "0")
# a pass that failed on the device (wide-row cluster exchange timed out: GPU shared): "fallback"
# resumes the fit on the two-pass path from the untouched state; "raise" raises RuntimeError
_ON_DEVICE_ERROR = os.environ.get("TR_ON_DEVICE_ERROR", "fallback")
# torch.optim.Adam defaults (torch/optim/adam.py)
_ADAM_DEFAULTS = dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False,
                      foreach=None, maximize=False, capturable=False, differentiable=False,
                      fused=None, decoupled_weight_decay=False)


def softplus_params(softplus_kwargs):
    kw = _DEFAULT_SOFTPLUS if softplus_kwargs is None else softplus_kwargs
    # torch.nn.functional.softplus defaults when a key is absent
    return float(kw.get("beta", 1.0)), float(kw.get("threshold", 20.0))


def nonlin_key(non_negative, softplus_kwargs, n_factors):
    """The per-factor softplus switches and (beta, threshold) a plan is built with: the reference
    reads self.non_negative / self.softplus_kwargs on every call, so a plan whose key differs from
    the model's current one must be rebuilt."""
    nn = tuple(1 if bool(non_negative[f]) else 0 for f in range(n_factors))
    return (nn,) + softplus_params(softplus_kwargs)


def adam_hparams(Adam_kwargs):
    """Resolve Adam kwargs exactly like torch.optim.Adam(params, **Adam_kwargs)."""
    if Adam_kwargs is None:
        # reference quirk (standard_tensor_regression.py:442-453): the default dict is never
        # assigned, so torch.optim.Adam(..., **None) raises this TypeError
        raise TypeError("torch.optim.adam.Adam() argument after ** must be a mapping, not NoneType")
    hp = dict(_ADAM_DEFAULTS)
    for k, v in Adam_kwargs.items():
        if k not in hp:
            raise TypeError(f"Adam.__init__() got an unexpected keyword argument '{k}'")
        hp[k] = v
    lr = float(hp["lr"])
    b1, b2 = (float(b) for b in hp["betas"])
    eps, wd = float(hp["eps"]), float(hp["weight_decay"])
    if not 0.0 <= lr:
        raise ValueError(f"Invalid learning rate: {lr}")
    if not 0.0 <= eps:
        raise ValueError(f"Invalid epsilon value: {eps}")
    if not 0.0 <= b1 < 1.0:
        raise ValueError(f"Invalid beta parameter at index 0: {b1}")
    if not 0.0 <= b2 < 1.0:
        raise ValueError(f"Invalid beta parameter at index 1: {b2}")
    if not 0.0 <= wd:
        raise ValueError(f"Invalid weight_decay value: {wd}")
    if hp["maximize"] or hp["decoupled_weight_decay"] or hp["differentiable"]:
        raise NotImplementedError("maximize / decoupled_weight_decay / differentiable Adam are not "
                                  "implemented by the gfx950 fit loop")
    return dict(lr=lr, beta1=b1, beta2=b2, eps=eps, weight_decay=wd, amsgrad=bool(hp["amsgrad"]))


def device_index(device):
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(
            f"tensor_regression_amd runs the hot path on the GPU (HIP); got device '{device}'. "
            "Use device='cuda' / 'cuda:N'.")
    return d.index if d.index is not None else torch.cuda.current_device()


def compute_device(X, model_device):
    """HIP device the hot path runs on: X's device if X is on the GPU, else the model's device
    if that is a GPU, else the current GPU (parameters may stay on the host; they are packed
    into the device arena per fit and written back in place)."""
    if isinstance(X, torch.Tensor) and X.device.type == "cuda":
        return X.device.index if X.device.index is not None else torch.cuda.current_device()
    d = torch.device(model_device)
    if d.type == "cuda":
        return d.index if d.index is not None else torch.cuda.current_device()
    if not torch.cuda.is_available():
        raise _lib.HipLibraryError("no HIP device available: the gfx950 hot path has no CPU fallback")
    return torch.cuda.current_device()


_live_plans = weakref.WeakSet()
_atexit_registered = False


def _track(plan):
    """Remember a live plan; the first one registers the exit hook.  Registered after torch has
    initialised HIP, so (atexit is LIFO) it runs before torch's and the HIP runtime's own teardown."""
    global _atexit_registered
    _live_plans.add(plan)
    if not _atexit_registered:
        atexit.register(_destroy_all_plans)
        _atexit_registered = True


def _destroy_all_plans():
    """Free every plan's workspace and timing events while the HIP runtime is still fully alive.
    Plans held by module-level caches would otherwise be destroyed during interpreter teardown,
    after a profiler's tool finalisation or the runtime's static destructors (the exit-time SIGSEGV
    seen under rocprofv3)."""
    for plan in list(_live_plans):
        try:
            plan.destroy()
        except Exception:
            pass


def stream_handle(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


_FOREACH_READY = set()


def _ready_foreach_copy(arena):
    """The process's first torch._foreach_copy_ on a (device, dtype) costs ~36 ms of host time
    (measured on the GPU box: the multi-tensor kernel is loaded on first use).  Paid inside the
    unpack at the end of the first fit, it left the GPU idle that long after the fit's last
    launch; paid here, at the start of the first fit, it precedes that fit's GPU work."""
    key = (arena.device, arena.dtype)
    if key in _FOREACH_READY:
        return
    a, b = torch.zeros(1, dtype=arena.dtype, device=arena.device), torch.zeros(1, dtype=arena.dtype, device=arena.device)
    torch._foreach_copy_([a], [b])
    _FOREACH_READY.add(key)


def _pack_arena(srcs, n, dtype, device):
    """Concatenate the flattened factors (and bias) into a fresh arena: one launch when they all
    live on the plan's device in its dtype, else one copy per tensor."""
    arena = torch.empty(n, dtype=dtype, device=device)
    if arena.is_cuda:
        _ready_foreach_copy(arena)
    with torch.no_grad():
        if sum(s.numel() for s in srcs) == n and all(s.device == arena.device and s.dtype == dtype for s in srcs):
            torch.cat(srcs, out=arena)
        else:
            o = 0
            for s in srcs:
                arena[o:o + s.numel()].copy_(s)
                o += s.numel()
            if o != n:
                raise ValueError(f"the parameters hold {o} values, the plan's arena {n}")
    return arena


def _unpack_arena(arena, offsets, dsts):
    """Copy the arena's segments back into the caller's tensors in place (like an optimizer step):
    one multi-tensor launch when they all live on the arena's device in its dtype."""
    bounds = list(offsets[:len(dsts)]) + [arena.numel()]
    with torch.no_grad():
        srcs = [arena[bounds[i]:bounds[i + 1]][:d.numel()].view(d.shape) for i, d in enumerate(dsts)]
        if all(d.device == arena.device and d.dtype == arena.dtype for d in dsts):
            torch._foreach_copy_(dsts, srcs)
        else:
            for d, s in zip(dsts, srcs):
                d.copy_(s.to(device=d.device, dtype=d.dtype))


class Plan:
    """Owns one `tr_plan` (workspace + kernel strategy) for a model shape."""

    def __init__(self, model, feature_dims, n_classes, rank, max_rows, non_negative, softplus_kwargs,
                 device, dtype=torch.float32):
        self.lib = _lib.load()
        self.dev = device_index(device)
        self.device_str = f"cuda:{self.dev}"
        self.model = model
        if dtype not in (torch.float32, torch.float64):
            raise NotImplementedError(f"the gfx950 kernels compute in float32 or float64; got dtype={dtype}")
        if dtype == torch.float64 and model != _lib.TR_MODEL_LINEAR:
            raise NotImplementedError("float64 is offered for CP_linear_regression only (the reference's multinomial "
                                      "class is float32-only, multinomial_tensor_regression.py:255)")
        self.dtype = dtype
        self.f64 = dtype == torch.float64
        self._sfx = "_f64" if self.f64 else ""
        self.feature_dims = [int(d) for d in feature_dims]
        self.n_classes = int(n_classes)
        self.rank = int(rank)
        self.max_rows = int(max_rows)
        nf = len(self.feature_dims) + (1 if model == _lib.TR_MODEL_MULTINOMIAL else 0)
        self.n_factors = nf
        self.nonlin = nonlin_key(non_negative, softplus_kwargs, nf)
        nn, beta, thr = self.nonlin
        dims = (ctypes.c_int64 * len(self.feature_dims))(*self.feature_dims)
        nna = (ctypes.c_int32 * nf)(*nn)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            if self.f64:
                rc = self.lib.tr_plan_create_f64(ctypes.byref(h), self.dev, len(self.feature_dims), dims, self.rank,
                                                 max(1, self.max_rows), nna, beta, thr)
            else:
                rc = self.lib.tr_plan_create(ctypes.byref(h), self.dev, model, len(self.feature_dims), dims,
                                             self.n_classes, self.rank, max(1, self.max_rows), nna, beta, thr)
        check(rc, "tr_plan_create" + self._sfx)
        self.h = h
        _track(self)
        self.num_params = int(self.lib.tr_plan_num_params(h))
        self.num_grads = int(self.lib.tr_plan_num_grads(h))
        self.offsets = [int(self.lib.tr_plan_factor_offset(h, f)) for f in range(nf + 1)]
        self.describe = self.lib.tr_plan_describe(h).decode()

    def destroy(self):
        """Release the C plan (idempotent); its hipFree orders the release after the work that uses it."""
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.h = None
            self.lib.tr_plan_destroy(h)

    def __del__(self, _is_finalizing=sys.is_finalizing):
        # during interpreter shutdown the exit hook has already destroyed every plan; never call
        # into HIP from a finaliser that may run after the runtime is gone (the default argument
        # keeps the function reachable after module globals such as `sys` have been cleared)
        if _is_finalizing():
            return
        try:
            self.destroy()
        except Exception:
            pass

    # ---- parameter arena -------------------------------------------------------------------
    def factor_shapes(self):
        dims = self.feature_dims + ([self.n_classes] if self.model == _lib.TR_MODEL_MULTINOMIAL else [])
        return [(d, self.rank) for d in dims]

    def pack(self, Bcp, bias=None):
        shapes = self.factor_shapes()
        if len(Bcp) != len(shapes):
            raise ValueError(f"expected {len(shapes)} Kruskal factors, got {len(Bcp)}")
        srcs = []
        for f, (A, shp) in enumerate(zip(Bcp, shapes)):
            A = torch.as_tensor(A)
            if tuple(A.shape) != shp:
                raise ValueError(f"factor {f} has shape {tuple(A.shape)}, expected {shp}")
            srcs.append(A.detach().reshape(-1))
        if self.model == _lib.TR_MODEL_LINEAR:
            srcs.append(torch.as_tensor(bias).detach().reshape(-1)[:1])
        return _pack_arena(srcs, self.num_params, self.dtype, self.device_str)

    def unpack_into(self, arena, Bcp, bias=None):
        """Write the arena back into the caller's tensors in place (like an optimizer step)."""
        dsts = list(Bcp) + ([bias] if bias is not None and self.model == _lib.TR_MODEL_LINEAR else [])
        _unpack_arena(arena, self.offsets, dsts)

    def factor_views(self, arena):
        return [arena[self.offsets[f]:self.offsets[f + 1]].view(shp)
                for f, shp in enumerate(self.factor_shapes())]

    # ---- timing ------------------------------------------------------------------------------
    def set_prepare_next(self, enable):
        """tr_plan_set_prepare_next: each adam_step also prepares the next loss_grad's factors."""
        check(self.lib.tr_plan_set_prepare_next(self.h, 1 if enable else 0), "tr_plan_set_prepare_next")

    def set_timing(self, enable, kinds=None, every=1):
        """Enable hipEvent timing for the given kernel kinds (names of _lib.KERNEL_KINDS; None = all),
        bracketing every `every`-th launch of each (tr_plan_set_timing_every)."""
        mask = 0
        if enable:
            mask = -1 if kinds is None else sum(1 << _lib.KERNEL_KINDS.index(k) for k in kinds)
        check(self.lib.tr_plan_set_timing_every(self.h, int(every)), "tr_plan_set_timing_every")
        check(self.lib.tr_plan_set_timing(self.h, mask), "tr_plan_set_timing")

    def read_timing(self):
        """{kernel kind: (total_ms, launches)} since the last read (synchronises the events)."""
        n = len(_lib.KERNEL_KINDS)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        check(self.lib.tr_plan_read_timing(self.h, ms, cnt), "tr_plan_read_timing")
        return {k: (ms[i], cnt[i]) for i, k in enumerate(_lib.KERNEL_KINDS)}

    def check_status(self):
        """Raise if a kernel of this plan reported a device-side failure (tr_plan_status: a wide-row
        cluster exchange that timed out because the GPU was shared).  Only a plan whose pass can
        fail on the device (may_fail_on_device) has anything to check; it synchronises the device."""
        if not self.may_fail_on_device:
            return
        torch.cuda.synchronize(self.dev)
        st = ctypes.c_int32(0)
        check(self.lib.tr_plan_status(self.h, ctypes.byref(st)), "tr_plan_status")
        if st.value:
            raise RuntimeError(f"gfx950 kernel status {st.value:#x}: a cross-workgroup exchange timed out "
                               "(the GPU was shared with another kernel); the affected gradients are NaN")

    @property
    def may_fail_on_device(self):
        """Only the wide-row cluster pass depends on co-resident workgroups."""
        return "cluster-1pass" in self.describe and "recovered=2pass" not in self.describe

    def recover(self, where):
        """After a failed pass: two-pass from now on (tr_plan_recover), or raise (TR_ON_DEVICE_ERROR=raise)."""
        if _ON_DEVICE_ERROR == "raise":
            raise RuntimeError(f"gfx950 single-pass kernel failed on the device ({where}): a cross-workgroup "
                               "exchange timed out (the GPU was shared with another kernel); no step was applied")
        import warnings
        warnings.warn(f"gfx950 wide-row single pass failed on the device ({where}; GPU shared?): continuing on "
                      "the two-pass path from the last good iteration", RuntimeWarning, stacklevel=3)
        check(self.lib.tr_plan_recover(self.h), "tr_plan_recover")
        self.describe = self.lib.tr_plan_describe(self.h).decode()

    def loss_grad_checked(self, X, target, class_weight, norm, arena, weights, grad):
        """loss_grad for callers outside the Adam loop (LBFGS closures, one-off evaluations): on a
        plan whose pass can fail on the device, check the status slot and redo the pass on the
        two-pass path if it failed (one host sync, only on such plans)."""
        self.loss_grad(X, target, class_weight, norm, arena, weights, grad)
        if self.may_fail_on_device and float(grad[self.num_params + 1].item()) != 0.0:
            self.recover("loss_grad")
            self.loss_grad(X, target, class_weight, norm, arena, weights, grad)

    # ---- entry points ------------------------------------------------------------------------
    def _set_stride(self, X):
        """Tell the plan X's row stride (windowed / strided views) when it changes."""
        stride = int(X.stride(0)) if X.ndim >= 1 and X.shape[0] > 1 else 0
        if stride == int(np.prod(X.shape[1:])):
            stride = 0
        if stride != getattr(self, "_xstride", 0):
            check(self.lib.tr_plan_set_x_stride(self.h, stride), "tr_plan_set_x_stride")
            self._xstride = stride
            self._xrange_key = None  # (the re-chosen split body starts in its fast form)
            self.describe = self.lib.tr_plan_describe(self.h).decode()

    def _x_form(self, X):
        """The split kernels' X form follows X's range (tr_plan_set_x_range): max |x|, min x and the
        smallest mean x^2 of a nonzero sample, measured on the device (tr_x_range, one streaming
        read of X) once per X — keyed
        by its data pointer, shape, strides and torch version counter, so a new or modified X is
        measured again — and skipped for plans of other kernels.  X a util.HostStream: its host
        copy's range, measured once (HostStream.range)."""
        if "form=bf16split" not in self.describe and "bf16split" not in self.describe:
            return
        from .util import HostStream
        X = getattr(X, "_tr_stream", X)  # a HostStream chunk: the stream's host X
        if isinstance(X, HostStream):
            key = ("hoststream", id(X))
            if key != getattr(self, "_xrange_key", None):
                mx, msq, mn = X.range()
                check(self.lib.tr_plan_set_x_range(self.h, mx, msq, mn), "tr_plan_set_x_range")
                self._xrange_key = key
                self.describe = self.lib.tr_plan_describe(self.h).decode()
            return
        key = (X.data_ptr(), tuple(X.shape), tuple(X.stride()), X._version)
        if key == getattr(self, "_xrange_key", None):
            return
        N = int(X.shape[0])
        P = int(np.prod(X.shape[1:]))
        nb = int(min(1024, max(1, N)))
        out = torch.empty(3 * nb, dtype=torch.float64, device=self.device_str)
        ld = int(X.stride(0)) if N > 1 else P
        check(self.lib.tr_x_range(ptr(X), N, P, ld, ptr(out), nb, stream_handle(self.dev)), "tr_x_range")
        r = out.cpu().numpy()
        mx = float(np.max(r[:nb])) if not np.isnan(r[:nb]).any() else float("nan")
        msq = float(np.min(r[nb:2 * nb]))  # the smallest mean x^2 of a nonzero sample
        mn = float(np.min(r[2 * nb:]))
        check(self.lib.tr_plan_set_x_range(self.h, mx, msq, mn), "tr_plan_set_x_range")
        self._xrange_key = key
        self.describe = self.lib.tr_plan_describe(self.h).decode()

    def forward(self, X, arena, weights, out=None):
        N = X.shape[0]
        C = self.n_classes if self.model == _lib.TR_MODEL_MULTINOMIAL else 1
        if out is None:
            shape = (N, C) if self.model == _lib.TR_MODEL_MULTINOMIAL else (N,)
            out = torch.empty(shape, dtype=self.dtype, device=X.device)
        self._set_stride(X)
        fwd = self.lib.tr_forward_f64 if self.f64 else self.lib.tr_forward
        rc = fwd(self.h, ptr(X), N, ptr(arena), ptr(weights), ptr(out), stream_handle(self.dev))
        check(rc, "tr_forward" + self._sfx)
        return out

    def loss_grad(self, X, target, class_weight, norm, arena, weights, grad, yhat=None, stop=None):
        self._set_stride(X)
        self._x_form(X)
        if self.f64:
            rc = self.lib.tr_loss_grad_f64(self.h, ptr(X), X.shape[0], ptr(target), float(norm), ptr(arena),
                                           ptr(weights), ptr(grad), ptr(yhat), ptr(stop), stream_handle(self.dev))
        else:
            rc = self.lib.tr_loss_grad(self.h, ptr(X), X.shape[0], ptr(target), ptr(class_weight), float(norm),
                                       ptr(arena), ptr(weights), ptr(grad), ptr(yhat), ptr(stop),
                                       stream_handle(self.dev))
        check(rc, "tr_loss_grad" + self._sfx)

    def finalize_grad(self, arena, grad, lambda_l2, grad_total, loss_out):
        fin = self.lib.tr_finalize_grad_f64 if self.f64 else self.lib.tr_finalize_grad
        rc = fin(self.h, ptr(arena), ptr(grad), float(lambda_l2), ptr(grad_total), ptr(loss_out),
                 stream_handle(self.dev))
        check(rc, "tr_finalize_grad" + self._sfx)

    def adam_step(self, arena, grad, m, v, vmax, lambda_l2, hp, step, hist, hist_base, it, patience, tol,
                  stop):
        step_fn = self.lib.tr_adam_step_f64 if self.f64 else self.lib.tr_adam_step
        rc = step_fn(self.h, ptr(arena), ptr(grad), ptr(m), ptr(v), ptr(vmax), float(lambda_l2),
                     hp["lr"], hp["beta1"], hp["beta2"], hp["eps"], hp["weight_decay"],
                     1 if hp["amsgrad"] else 0, int(step), ptr(hist), int(hist_base), int(it),
                     int(patience), float(tol), ptr(stop), stream_handle(self.dev))
        check(rc, "tr_adam_step" + self._sfx)


class SpectralPlan(Plan):
    """`tr_plan` of the spectral model (spectral_tensor_regression.CP_linear_regression):
    arena = Bcp_n (3 factors (I, Rn, 1)) + Bcp_c (3 factors, the first (W, Rs, Cc)) + bias (n_out)."""

    def __init__(self, n_w, n_d, n_out, rank_normal, rank_spectral, n_complex, max_rows, non_negative,
                 softplus_kwargs, device):
        self.lib = _lib.load()
        self.dev = device_index(device)
        self.device_str = f"cuda:{self.dev}"
        self.model = _lib.TR_MODEL_SPECTRAL
        self.dtype, self.f64, self._sfx = torch.float32, False, ""
        self.dims = (int(n_w), int(n_d), int(n_out))
        self.rank_normal, self.rank_spectral, self.n_complex = int(rank_normal), int(rank_spectral), int(n_complex)
        self.max_rows = int(max_rows)
        self.n_factors = 6
        self.nonlin = nonlin_key(non_negative, softplus_kwargs, 3)
        nn = (ctypes.c_int32 * 3)(*self.nonlin[0])
        beta, thr = self.nonlin[1:]
        h = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            rc = self.lib.tr_plan_create_spectral(ctypes.byref(h), self.dev, self.dims[0], self.dims[1], self.dims[2],
                                                  self.rank_normal, self.rank_spectral, self.n_complex,
                                                  max(1, self.max_rows), nn, beta, thr)
        check(rc, "tr_plan_create_spectral")
        self.h = h
        _track(self)
        self.num_params = int(self.lib.tr_plan_num_params(h))
        self.num_grads = int(self.lib.tr_plan_num_grads(h))
        self.offsets = [int(self.lib.tr_plan_factor_offset(h, f)) for f in range(7)]
        self.describe = self.lib.tr_plan_describe(h).decode()

    def factor_shapes(self):
        W, D, O = self.dims
        Rn, Rs, Cc = self.rank_normal, self.rank_spectral, self.n_complex
        return [(W, Rn, 1), (D, Rn, 1), (O, Rn, 1), (W, Rs, Cc), (D, Rs, 1), (O, Rs, 1)]

    def pack(self, Bcp_n, Bcp_c, bias):
        shapes = self.factor_shapes()
        facs = list(Bcp_n) + list(Bcp_c)
        if len(facs) != 6:
            raise ValueError(f"expected 3 + 3 Kruskal factors, got {len(Bcp_n)} + {len(Bcp_c)}")
        srcs = []
        for f, (A, shp) in enumerate(zip(facs, shapes)):
            A = torch.as_tensor(A)
            if tuple(A.shape) != shp:
                raise ValueError(f"factor {f} has shape {tuple(A.shape)}, expected {shp}")
            srcs.append(A.detach().reshape(-1))
        srcs.append(torch.as_tensor(bias).detach().reshape(-1))
        return _pack_arena(srcs, self.num_params, torch.float32, self.device_str)

    def unpack_into(self, arena, Bcp_n, Bcp_c, bias=None):
        _unpack_arena(arena, self.offsets, list(Bcp_n) + list(Bcp_c) + ([bias] if bias is not None else []))

    def forward(self, X, arena, weights, out=None):
        """The reference's predict model: lin_model + spectral_model (N, n_out)."""
        if out is None:
            out = torch.empty((X.shape[0], self.dims[2]), dtype=torch.float32, device=X.device)
        self._set_stride(X)
        rc = self.lib.tr_forward(self.h, ptr(X), X.shape[0], ptr(arena), ptr(weights), ptr(out),
                                 stream_handle(self.dev))
        check(rc, "tr_forward")
        return out

    def latents(self, X, arena, out=None):
        """stepwise_latents_model (N, rank_normal)."""
        if out is None:
            out = torch.zeros((X.shape[0], self.rank_normal), dtype=torch.float32, device=X.device)
        self._set_stride(X)
        rc = self.lib.tr_spectral_latents(self.h, ptr(X), X.shape[0], ptr(arena), ptr(out), stream_handle(self.dev))
        check(rc, "tr_spectral_latents")
        return out


def _rows_contiguous(X):
    """Each X[n] block is contiguous (any stride, even overlapping, along dim 0)."""
    expect = 1
    for d in range(X.ndim - 1, 0, -1):
        if X.shape[d] != 1 and X.stride(d) != expect:
            return False
        expect *= X.shape[d]
    return X.ndim >= 1 and X.stride(0) >= 1


def as_device_rows(X, dev, dtype=torch.float32):
    """X as a `dtype` tensor on cuda:dev whose samples X[n] are contiguous blocks; the stride along
    dim 0 is kept (strided / windowed views, e.g. util.windowed_view, are NOT materialised).  A
    view the 16-byte kernel paths cannot read (misaligned base with a stride % 4 == 0) is copied."""
    if not isinstance(X, torch.Tensor):
        X = torch.as_tensor(np.asarray(X), dtype=dtype)
    if X.dtype != dtype:
        raise TypeError(f"the gfx950 path of this model computes in {dtype}; got X of dtype {X.dtype}")
    if X.device.type != "cuda" or X.device.index != dev:
        X = X.to(f"cuda:{dev}")
    if not _rows_contiguous(X) or (X.stride(0) % 4 == 0 and X.data_ptr() % 16 != 0):
        X = X.contiguous()
    return X


def as_device_f32(X, dev, dtype=torch.float32):
    """X as a contiguous `dtype` tensor on cuda:dev (copies only when needed)."""
    if not isinstance(X, torch.Tensor):
        X = torch.as_tensor(np.asarray(X), dtype=dtype)
    if X.dtype != dtype:
        raise TypeError(f"the gfx950 path of this model computes in {dtype}; got a tensor of dtype {X.dtype}")
    if X.device.type != "cuda" or X.device.index != dev:
        X = X.to(f"cuda:{dev}")
    return X.contiguous()


def loss_grad_any(plan, X, target, class_weight, norm, arena, weights, grad, stop=None, tmp=None):
    """plan.loss_grad over a device X, or over a util.HostStream chunk by chunk (the chunk arenas
    are summed like sample shards: every data gradient is already normalised by `norm`)."""
    from .util import HostStream
    if not isinstance(X, HostStream):
        plan.loss_grad(X, target, class_weight, norm, arena, weights, grad, stop=stop)
        return
    first = True
    for r0, r1, Xc in X.chunks():
        if first:
            plan.loss_grad(Xc, target[r0:r1], class_weight, norm, arena, weights, grad, stop=stop)
            first = False
        else:
            plan.loss_grad(Xc, target[r0:r1], class_weight, norm, arena, weights, tmp, stop=stop)
            grad.add_(tmp)


def collective_device(process_group):
    """Device for the small host-logic collectives of a sharded fit: gloo takes CPU tensors, RCCL
    ("nccl") the rank's current HIP device."""
    import torch.distributed as dist
    return "cpu" if dist.get_backend(process_group) == "gloo" else f"cuda:{torch.cuda.current_device()}"


def agree(process_group, fn):
    """Run this rank's local preparation `fn()` (argument checks, device copies, plan creation) and
    make its failure collective: one MAX all-reduce of a failure flag, so if `fn` raised on any
    rank every rank raises (the failing rank its own exception) and no rank is left blocked in a
    later collective of the fit."""
    import torch.distributed as dist
    err, out = None, None
    try:
        out = fn()
    except Exception as e:  # re-raised below, after the other ranks have been told
        err = e
    flag = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=collective_device(process_group))
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=process_group)
    if err is not None:
        raise err
    if int(flag.item()):
        raise RuntimeError("the sharded fit failed on another rank of the process group (see that rank's error); "
                           "no rank started fitting")
    return out


def fit_start(process_group, fn, norm_of, size_of):
    """The start of a sharded fit in ONE collective: run this rank's preparation `fn()` (as
    `agree` does), then a single MAX all-reduce of a float64 vector settles
      - whether `fn` raised on any rank (every rank raises then, like `agree`);
      - that every rank's parameter arena has the same size, `size_of(out)` (ValueError on every
        rank otherwise, like `check_uniform`: no rank is left in a later collective);
      - the global normaliser, the sum of every rank's `norm_of(out)` (the sample count, or the
        class-weight total of the CE mean): each rank writes its value into its own slot, -inf
        into the others, so the MAX hands every rank every value, summed in rank order.
    One host read of the result.  Replaces agree + an all-reduce of the normaliser + the arena
    check of sync_replicas (three collectives and three host synchronisations per fit call: at
    world 1 on RCCL most of the process-group path's per-call cost, tools/pg_account.py).
    Returns (fn's result, global normaliser)."""
    import torch.distributed as dist
    world = dist.get_world_size(process_group)
    me = dist.get_rank(process_group)
    err, out = None, None
    try:
        out = fn()
    except Exception as e:  # re-raised below, after the other ranks have been told
        err = e
    v = [float("-inf")] * (3 + world)
    v[0] = 0.0 if err is None else 1.0
    if err is None:
        size = float(size_of(out))
        v[1], v[2], v[3 + me] = size, -size, float(norm_of(out))
    comm = direct_comm(process_group, None)
    if comm is not None:  # RCCL: ncclAllReduce on the compute stream (RcclAllReduce.max_f64)
        r = comm.max_f64(v)
    else:
        t = torch.tensor(v, dtype=torch.float64, device=collective_device(process_group))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=process_group)
        r = t.tolist()
    if err is not None:
        raise err
    if r[0] > 0:
        raise RuntimeError("the sharded fit failed on another rank of the process group (see that rank's error); "
                           "no rank started fitting")
    if r[1] != size or -r[2] != size:
        raise ValueError(f"ranks disagree on the parameter arena size (this rank {int(size)}, max {int(r[1])}, "
                         f"min {int(-r[2])}); every rank's model must have the same factor shapes")
    total = 0.0
    for x in r[3:]:
        total += x
    return out, total


def check_uniform(value, process_group, what, device):
    """Raise ValueError on EVERY rank when the ranks disagree on an integer (one all-reduce), so a
    mismatch cannot leave some ranks blocked in a later collective."""
    import torch.distributed as dist
    n = torch.tensor([int(value), -int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=process_group)
    if int(n[0]) != int(value) or -int(n[1]) != int(value):
        raise ValueError(f"ranks disagree on {what} (this rank {int(value)}, max {int(n[0])}, min {-int(n[1])}); "
                         "every rank's model must have the same factor shapes")


def sync_replicas(arena, process_group, checked=False):
    """Start every rank's replica from the same parameters (multi-GPU fit_Adam).

    The ranks must agree on the arena layout (a multinomial model takes the global class set
    before this point, CP_logistic_regression._sync_class_set) — checked with one MIN/MAX
    all-reduce so a mismatch raises on every rank instead of hanging in the per-iteration
    all-reduce — and then
    take group rank 0's parameters (one broadcast per fit).  From there the replicas stay in
    lock-step: every rank applies the identical step to the bitwise-identical all-reduced sums.
    checked: the arena sizes were already compared (fit_start)."""
    import torch.distributed as dist
    if not checked:
        check_uniform(arena.numel(), process_group, "the parameter arena size", arena.device)
    comm = direct_comm(process_group, arena.device.index if arena.is_cuda else None)
    if comm is not None:  # RCCL: ncclBroadcast on the compute stream
        comm.broadcast(arena, root=0)
        return
    src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
    dist.broadcast(arena, src=src, group=process_group)


def fit_state(plan, dtype, amsgrad):
    """(grad, m, v, vmax | None, stop, tmp) of one Adam fit: views of ONE per-plan device buffer,
    zeroed with a single fill per fit (one launch instead of six allocations and fills).  The
    buffer is reused by the plan's next fit; fits on one plan run one after another, and each
    ends in a host synchronisation on its final status before it returns."""
    G, P = plan.num_grads, plan.num_params
    seg = lambda n: -(-n // 64) * 64  # 256-byte aligned segments
    sizes = (seg(G), seg(P), seg(P), seg(P), seg(G), 64)
    n = sum(sizes)
    buf = getattr(plan, "_fit_state", None)
    if buf is None or buf.numel() != n or buf.dtype != dtype:
        buf = torch.empty(n, dtype=dtype, device=plan.device_str)
        plan._fit_state = buf
    buf.zero_()
    parts = torch.split(buf, sizes)
    grad, m, v, vmax, tmp = parts[0][:G], parts[1][:P], parts[2][:P], parts[3][:P], parts[4][:G]
    stop = parts[5].view(torch.int32)[:1]
    return grad, m, v, (vmax if amsgrad else None), stop, tmp


# ---- the per-iteration gradient all-reduce -------------------------------------------------------
_RCCL_DIRECT = os.environ.get("TR_RCCL_DIRECT", "1") != "0"
# seconds a host sync of a sharded fit waits for the direct all-reduce before aborting the
# communicator (a dead or diverged peer would otherwise block the survivors forever)
_RCCL_TIMEOUT = float(os.environ.get("TR_RCCL_TIMEOUT", "600"))
_rccl_comms = {}


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # ncclUniqueId (rccl.h: NCCL_UNIQUE_ID_BYTES)


def uid_to_bytes(uid):
    """The raw 128 bytes of an ncclUniqueId (reading the c_char array field would cut them at
    the first NUL, and the id is binary)."""
    return ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid))


def uid_from_bytes(raw):
    if len(raw) != ctypes.sizeof(_UniqueId):
        raise ValueError(f"an ncclUniqueId is {ctypes.sizeof(_UniqueId)} bytes, got {len(raw)}")
    return _UniqueId.from_buffer_copy(bytes(raw))


def _rccl_lib():
    """The RCCL library torch's NCCL backend runs on (same file: the loader hands back the already
    loaded instance), with the four entry points used here."""
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    lib = ctypes.CDLL(path if os.path.exists(path) else "librccl.so")
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
    lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    lib.ncclBroadcast.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    lib.ncclGetErrorString.argtypes = [ctypes.c_int]
    lib.ncclCommGetAsyncError.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    lib.ncclCommAbort.argtypes = [ctypes.c_void_p]
    lib.ncclCommCount.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    for fn in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclBroadcast", "ncclCommDestroy",
               "ncclCommGetAsyncError", "ncclCommAbort", "ncclCommCount"):
        getattr(lib, fn).restype = ctypes.c_int
    return lib


class _CollectiveTimeout(Exception):
    pass


class _CollectiveError(Exception):
    pass


def wait_progress(events, async_error, timeout, clock=None, sleep=None):
    """Poll `events` (objects with .query(), completing in order: one per all-reduce, the last one
    behind all queued work) until every one has completed.  Raise _CollectiveError as soon as
    `async_error()` reports an error, and _CollectiveTimeout when `timeout` seconds pass in which
    no further event completed: the clock restarts at every completed event, so the bound is on
    time WITHOUT progress, whatever the number of iterations between host syncs."""
    import time
    clock = time.monotonic if clock is None else clock
    sleep = time.sleep if sleep is None else sleep
    i, n = 0, len(events)
    t0 = clock()
    spins = 0
    while i < n:
        if events[i].query():
            i += 1
            t0 = clock()
            continue
        msg = async_error()
        if msg is not None:
            raise _CollectiveError(msg)
        if clock() - t0 > timeout:
            raise _CollectiveTimeout(f"{i} of the {n} queued steps had completed")
        spins += 1
        sleep(0 if spins < 2000 else 1e-4)


class RcclAllReduce:
    """Sum all-reduce of a device tensor over the ranks of a torch.distributed NCCL (= RCCL) group,
    issued with ncclAllReduce on the caller's current stream.

    torch's ProcessGroupNCCL runs a collective on its own stream and joins it to the compute
    stream with events before and after: a rocprofv3 trace of the world-1 RCCL path shows
    ≈ 11 µs of idle GPU between the gradient kernel and the Adam step per iteration.  Here the
    collective is one more launch in the compute stream's order.  The communicator is built once
    per (ranks, device) from a unique id broadcast over the group, and kept for the process."""

    def __init__(self, process_group, device_index):
        import torch.distributed as dist
        self.lib = _rccl_lib()
        self.dev = int(device_index)
        ranks = dist.get_process_group_ranks(process_group)
        me = dist.get_rank(process_group)
        self.size = len(ranks)
        uid = _UniqueId()
        if me == 0:
            self._check(self.lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        buf = torch.frombuffer(bytearray(uid_to_bytes(uid)), dtype=torch.uint8).to(f"cuda:{self.dev}")
        dist.broadcast(buf, src=ranks[0], group=process_group)
        uid = uid_from_bytes(buf.cpu().numpy().tobytes())
        self._pending, self._free = [], []  # watchdog events: recorded / completed and reusable
        self._t_every, self._t_calls, self._t_pairs = 0, 0, []  # sampled all-reduce timing (bench.py)
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            self._check(self.lib.ncclCommInitRank(ctypes.byref(self.comm), len(ranks), uid, me), "ncclCommInitRank")

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.ncclGetErrorString(rc).decode()} (RCCL error {rc})")

    def __call__(self, t):
        dt = {torch.float32: 7, torch.float64: 8}[t.dtype]  # ncclFloat32 / ncclFloat64
        p = ctypes.c_void_p(t.data_ptr())
        timed = self._t_every > 0 and self._t_calls % self._t_every == 0
        self._t_calls += 1
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream(self.dev))
        self._check(self.lib.ncclAllReduce(p, p, t.numel(), dt, 0, self.comm, stream_handle(self.dev)),
                    "ncclAllReduce")
        if timed:
            e1.record(torch.cuda.current_stream(self.dev))
            self._t_pairs.append((e0, e1, t.numel() * t.element_size()))
        if self.size > 1:  # progress marker for the watchdog: one event behind every all-reduce
            ev = self._free.pop() if self._free else torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            self._pending.append(ev)

    def max_f64(self, values):
        """MAX all-reduce of a short host list of floats over the ranks (ncclAllReduce, ncclMax, on
        the compute stream) and its result back on the host: the host-logic collective of a
        sharded fit's start (fit_start), without torch's collective stream and its event joins
        (≈ 80 µs per call at world 1 through ProcessGroupNCCL, tools/pg_account.py)."""
        dev = torch.device("cuda", self.dev)
        buf = getattr(self, "_f64_buf", None)
        if buf is None or buf.numel() != len(values):
            buf = torch.empty(len(values), dtype=torch.float64, device=dev)
            self._f64_host = torch.empty(len(values), dtype=torch.float64, pin_memory=True)
            self._f64_buf = buf
        self._f64_host.copy_(torch.tensor(values, dtype=torch.float64))
        buf.copy_(self._f64_host, non_blocking=True)
        p = ctypes.c_void_p(buf.data_ptr())
        self._check(self.lib.ncclAllReduce(p, p, buf.numel(), 8, 2, self.comm, stream_handle(self.dev)),
                    "ncclAllReduce(max)")  # ncclFloat64, ncclMax
        self._f64_host.copy_(buf, non_blocking=True)
        torch.cuda.current_stream(self.dev).synchronize()
        return self._f64_host.tolist()

    def broadcast(self, t, root=0):
        """ncclBroadcast of a device tensor from communicator rank `root`, on the compute stream."""
        dt = {torch.float32: 7, torch.float64: 8}[t.dtype]
        p = ctypes.c_void_p(t.data_ptr())
        self._check(self.lib.ncclBroadcast(p, p, t.numel(), dt, int(root), self.comm, stream_handle(self.dev)),
                    "ncclBroadcast")

    def barrier(self):
        """Every rank past this point once all have reached it: a one-element all-reduce on the
        compute stream, then a device synchronisation (bench.py's timed-region bracket)."""
        self.max_f64([0.0])

    def wait(self, timeout=None):
        """Block until the work queued on the current stream (this rank's all-reduces included) has
        finished, polling the communicator: an asynchronous RCCL error, or `timeout` seconds
        (TR_RCCL_TIMEOUT, default 600) in which no further all-reduce of this rank completed,
        aborts the communicator and raises, so a rank whose peer died does not hang in the next
        host sync.  Progress is counted per all-reduce (one event behind each), not per host sync:
        a slow but healthy chunk of sync_every iterations never trips it.  ProcessGroupNCCL's
        watchdog does this for torch's own collectives; this communicator is outside it."""
        timeout = _RCCL_TIMEOUT if timeout is None else timeout
        tail = self._free.pop() if self._free else torch.cuda.Event()
        tail.record(torch.cuda.current_stream(self.dev))
        pending, self._pending = self._pending + [tail], []
        try:
            wait_progress(pending, self._async_error, timeout)
        except _CollectiveTimeout as e:
            self.abort()
            raise RuntimeError(f"RCCL all-reduce of the sharded fit made no progress for {timeout:.0f} s "
                               f"({e}; a peer rank died or left the fit); the communicator was aborted") from None
        except _CollectiveError as e:
            self.abort()
            raise RuntimeError(f"RCCL all-reduce of the sharded fit failed asynchronously: {e}") from None
        self._free.extend(pending)

    def count(self):
        """Ranks of the communicator (ncclCommCount): what RCCL itself sees, not the torch group."""
        n = ctypes.c_int(0)
        self._check(self.lib.ncclCommCount(self.comm, ctypes.byref(n)), "ncclCommCount")
        return int(n.value)

    def set_timing(self, every):
        """Bracket every `every`-th all-reduce with timing events (0: off; bench.py's N > 1 line)."""
        self._t_every, self._t_calls, self._t_pairs = max(0, int(every)), 0, []

    def read_timing(self):
        """[(ms, bytes)] of the sampled all-reduces since set_timing (synchronises their events)."""
        out = []
        for e0, e1, nb in self._t_pairs:
            e1.synchronize()
            out.append((e0.elapsed_time(e1), nb))
        self._t_pairs = []
        return out

    def _async_error(self):
        """None while the communicator is healthy, else RCCL's error string."""
        err = ctypes.c_int(0)
        rc = self.lib.ncclCommGetAsyncError(self.comm, ctypes.byref(err))
        if rc != 0 or err.value not in (0, 7):  # 7 = ncclInProgress
            return self.lib.ncclGetErrorString(err.value or rc).decode()
        return None

    def abort(self):
        if self.comm is not None and self.comm.value:
            self.lib.ncclCommAbort(self.comm)
            self.comm = None
        for k, v in list(_rccl_comms.items()):
            if v is self:
                del _rccl_comms[k]

    def destroy(self):
        if self.comm is not None and self.comm.value:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = None


def _destroy_rccl_comms():
    for c in list(_rccl_comms.values()):
        try:
            c.destroy()
        except Exception:
            pass
    _rccl_comms.clear()


def direct_comm(process_group, device_index):
    """The process's RcclAllReduce communicator for an NCCL (= RCCL) group on `device_index` (the
    current device when None), built on first use (collective: every rank of the group calls it
    at the same point); None for other backends or with TR_RCCL_DIRECT=0."""
    import torch.distributed as dist
    if not (_RCCL_DIRECT and dist.get_backend(process_group) == "nccl"):
        return None
    if device_index is None:
        device_index = torch.cuda.current_device()
    key = (tuple(dist.get_process_group_ranks(process_group)), int(device_index))
    comm = _rccl_comms.get(key)
    if comm is None:
        comm = RcclAllReduce(process_group, device_index)
        if not _rccl_comms:
            atexit.register(_destroy_rccl_comms)  # LIFO: before torch's and HIP's teardown
        _rccl_comms[key] = comm
    return comm


def gradient_allreduce(process_group, device_index):
    """The per-iteration sum all-reduce of the gradient arena for `process_group`: ncclAllReduce on
    the compute stream (RcclAllReduce) for an NCCL group, torch.distributed.all_reduce otherwise
    (gloo; or TR_RCCL_DIRECT=0).  Collective: every rank of the group calls it at the same point."""
    import torch.distributed as dist
    comm = direct_comm(process_group, device_index)
    if comm is not None:
        return comm

    def allreduce(g):
        dist.all_reduce(g, group=process_group)
    return allreduce


def run_adam_fit(plan, X, target, class_weight, norm, arena, weights, lambda_L2, max_iter, tol, patience,
                 hp, loss_running, verbose_cb=None, process_group=None, sync_every=64, arena_checked=False):
    """The fit_Adam loop (standard…py:453-470 / multinomial…py:447-465), device resident.

    Returns (convergence_reached, number_of_iterations_run).  `loss_running` is extended in place
    with the reference's per-iteration losses.  With a `process_group` (torch.distributed; RCCL
    on the GPU) X / target are this rank's sample shard: the replicas start from group rank 0's
    parameters (sync_replicas) and one all-reduce(sum) of the gradient arena — data gradients,
    data loss and the device status slot — runs between the local gradient and the Adam step.
    """
    dev = plan.device_str
    fdt = getattr(plan, "dtype", torch.float32)
    allreduce = None
    if process_group is not None:
        sync_replicas(arena, process_group, checked=arena_checked)
        allreduce = gradient_allreduce(process_group, getattr(plan, "dev", None))
    grad, m, v, vmax, stop, tmp = fit_state(plan, fdt, hp["amsgrad"])
    base = len(loss_running)
    # every entry a reader touches is written first: the loop writes [base, base + n_run) and the
    # plateau test (launched only when tol > 0) also reads the earlier losses, which are copied in
    hist = torch.empty(base + max(int(max_iter), 0) + 1, dtype=torch.float64, device=dev)
    if base and tol > 0:
        hist[:base] = torch.tensor(loss_running, dtype=torch.float64)
    if verbose_cb is not None:
        sync_every = 1
    # the loop changes the arena only through adam_step: let each step prepare the next
    # iteration's factors (one launch fewer per iteration, bitwise identical results)
    prep_next = _PREPARE_NEXT and isinstance(plan, Plan) and not isinstance(plan, SpectralPlan)
    if prep_next:
        plan.set_prepare_next(True)
    try:
        ii, stopped_at = _adam_loop(plan, X, target, class_weight, norm, arena, weights, lambda_L2, max_iter, tol,
                                    patience, hp, verbose_cb, allreduce, sync_every, grad, m, v, vmax, hist, base,
                                    stop, tmp)
    finally:
        if prep_next:
            plan.set_prepare_next(False)
    # stop flag: > 0 plateau convergence after that many iterations; < 0 NaN stop (spectral)
    n_run = abs(stopped_at) if stopped_at else ii
    loss_running.extend(hist[base:base + n_run].tolist())
    plan.last_stop = stopped_at
    return stopped_at > 0, n_run


def _adam_loop(plan, X, target, class_weight, norm, arena, weights, lambda_L2, max_iter, tol, patience, hp,
               verbose_cb, allreduce, sync_every, grad, m, v, vmax, hist, base, stop, tmp):
    ii = 0
    stopped_at = 0
    while ii < max_iter:
        n = min(sync_every, max_iter - ii)
        for k in range(n):
            it = ii + k
            if verbose_cb is not None:
                verbose_cb.before_step(arena)
            loss_grad_any(plan, X, target, class_weight, norm, arena, weights, grad, stop=stop, tmp=tmp)
            if allreduce is not None:
                allreduce(grad)
            plan.adam_step(arena, grad, m, v, vmax, lambda_L2, hp, it + 1, hist, base, it, patience, tol, stop)
        ii += n
        if isinstance(allreduce, RcclAllReduce) and allreduce.size > 1:
            allreduce.wait()  # the host sync below, with a watchdog on the peers
        stopped_at = int(stop.item())  # one host sync per chunk
        if stopped_at <= _lib.TR_STOP_DEVICE_ERROR:
            # a pass failed on the device (on any rank: the status slot is all-reduced with the
            # gradients, so every rank stops at the same iteration): nothing from that iteration on
            # was applied, so resume it on the two-pass path with the same parameters / Adam state
            failed = _lib.TR_STOP_DEVICE_ERROR - stopped_at
            plan.recover(f"iteration {failed}")
            stop.zero_()
            ii, stopped_at = failed, 0
            continue
        plan.check_status()
        if verbose_cb is not None:
            verbose_cb.after_step(ii - 1, float(hist[base + ii - 1].item()))
        if stopped_at:
            break
    return ii, stopped_at
