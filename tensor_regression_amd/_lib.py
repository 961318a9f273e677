"""ctypes binding of the gfx950 C ABI (include/tensor_regression_hip.h).

The shared library `libtr_hip.so` is built in-tree by `__graft_entry__.build()` (or
`make -C tensor_regression_amd/csrc`).  There is deliberately NO fallback: if the library
is missing or fails to load, every product entry point raises, so a test or benchmark can
never silently run on a CPU / eager-PyTorch path.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TR_HIP_LIB", os.path.join(_HERE, "libtr_hip.so"))

TR_ABI_VERSION = 5
TR_MODEL_LINEAR = 0
TR_MODEL_MULTINOMIAL = 1
TR_MODEL_SPECTRAL = 2
TR_MAX_FACTORS = 8
KERNEL_KINDS = ["stream_fused", "stream_rows", "stream_cols", "reduce", "mttkrp", "prep", "update"]

# exported symbol -> (restype, argtypes)
_c = ctypes
_vp = _c.c_void_p
SIGNATURES = {
    "tr_abi_version": (_c.c_int, []),
    "tr_last_error": (_c.c_char_p, []),
    "tr_plan_create": (_c.c_int, [_c.POINTER(_vp), _c.c_int, _c.c_int, _c.c_int, _c.POINTER(_c.c_int64),
                                  _c.c_int, _c.c_int, _c.c_int64, _c.POINTER(_c.c_int32), _c.c_float,
                                  _c.c_float]),
    "tr_plan_destroy": (_c.c_int, [_vp]),
    "tr_plan_num_params": (_c.c_int64, [_vp]),
    "tr_plan_num_grads": (_c.c_int64, [_vp]),
    "tr_plan_factor_offset": (_c.c_int64, [_vp, _c.c_int]),
    "tr_plan_workspace_bytes": (_c.c_int64, [_vp]),
    "tr_plan_describe": (_c.c_char_p, [_vp]),
    "tr_forward": (_c.c_int, [_vp, _vp, _c.c_int64, _vp, _vp, _vp, _vp]),
    "tr_loss_grad": (_c.c_int, [_vp, _vp, _c.c_int64, _vp, _vp, _c.c_double, _vp, _vp, _vp, _vp, _vp, _vp]),
    "tr_finalize_grad": (_c.c_int, [_vp, _vp, _vp, _c.c_float, _vp, _vp, _vp]),
    "tr_plan_set_timing": (_c.c_int, [_vp, _c.c_int]),
    "tr_plan_read_timing": (_c.c_int, [_vp, _c.POINTER(_c.c_double), _c.POINTER(_c.c_int64)]),
    "tr_plan_create_spectral": (_c.c_int, [_c.POINTER(_vp), _c.c_int, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int,
                                           _c.c_int, _c.c_int, _c.c_int64, _c.POINTER(_c.c_int32), _c.c_float,
                                           _c.c_float]),
    "tr_spectral_latents": (_c.c_int, [_vp, _vp, _c.c_int64, _vp, _vp, _vp]),
    "tr_plan_set_x_stride": (_c.c_int, [_vp, _c.c_int64]),
    "tr_plan_status": (_c.c_int, [_vp, _c.POINTER(_c.c_int32)]),
    "tr_adam_step": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _c.c_float, _c.c_double, _c.c_double,
                                _c.c_double, _c.c_double, _c.c_double, _c.c_int, _c.c_int64, _vp,
                                _c.c_int64, _c.c_int64, _c.c_int64, _c.c_double, _vp, _vp]),
    "tr_plan_set_prepare_next": (_c.c_int, [_vp, _c.c_int]),
}

_lock = threading.Lock()
_lib = None


class HipLibraryError(RuntimeError):
    """The gfx950 extension is missing, stale, or a call into it failed."""


def load():
    """Load (once) and return the ctypes library; raises HipLibraryError if unavailable."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HipLibraryError(
                f"gfx950 extension not built: {LIB_PATH} is missing. Run "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C tensor_regression_amd/csrc`.")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise HipLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError = stale library, surfaced loudly
            fn.restype = res
            fn.argtypes = args
        v = lib.tr_abi_version()
        if v != TR_ABI_VERSION:
            raise HipLibraryError(f"{LIB_PATH} has ABI version {v}, expected {TR_ABI_VERSION}; rebuild it")
        _lib = lib
        return lib


def check(rc, what):
    """Raise on a non-zero return code (ValueError for argument errors, HipLibraryError otherwise)."""
    if rc == 0:
        return
    msg = (_lib.tr_last_error() or b"").decode(errors="replace") if _lib is not None else ""
    if rc < 0:
        raise ValueError(f"{what}: {msg} (code {rc})")
    raise HipLibraryError(f"{what}: {msg} (hipError {rc})")


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())
