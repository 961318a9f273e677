"""ctypes binding of the gfx950 C ABI (include/tensor_regression_hip.h).

The shared library `libtr_hip.so` is built in-tree by `__graft_entry__.build()` (or
`make -C tensor_regression_amd/csrc`).  There is deliberately NO fallback: if the library
is missing or fails to load, every product entry point raises, so a test or benchmark can
never silently run on a CPU / eager-PyTorch path.
"""
import ctypes
import hashlib
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TR_HIP_LIB", os.path.join(_HERE, "libtr_hip.so"))

TR_ABI_VERSION = 8
TR_STOP_DEVICE_ERROR = -(1 << 30)
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
    "tr_build_id": (_c.c_char_p, []),
    "tr_plan_recover": (_c.c_int, [_vp]),
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
    "tr_plan_set_timing_every": (_c.c_int, [_vp, _c.c_int]),
    "tr_plan_read_timing": (_c.c_int, [_vp, _c.POINTER(_c.c_double), _c.POINTER(_c.c_int64)]),
    "tr_plan_create_spectral": (_c.c_int, [_c.POINTER(_vp), _c.c_int, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int,
                                           _c.c_int, _c.c_int, _c.c_int64, _c.POINTER(_c.c_int32), _c.c_float,
                                           _c.c_float]),
    "tr_spectral_latents": (_c.c_int, [_vp, _vp, _c.c_int64, _vp, _vp, _vp]),
    "tr_plan_set_x_stride": (_c.c_int, [_vp, _c.c_int64]),
    "tr_x_range": (_c.c_int, [_vp, _c.c_int64, _c.c_int64, _c.c_int64, _vp, _c.c_int, _vp]),
    "tr_mnl_geometry": (_c.c_int, [_c.c_int64, _c.c_int64, _c.c_int, _c.c_int, _vp, _c.c_int]),
    "tr_plan_set_x_range": (_c.c_int, [_vp, _c.c_double, _c.c_double, _c.c_double]),
    "tr_plan_status": (_c.c_int, [_vp, _c.POINTER(_c.c_int32)]),
    "tr_adam_step": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _c.c_float, _c.c_double, _c.c_double,
                                _c.c_double, _c.c_double, _c.c_double, _c.c_int, _c.c_int64, _vp,
                                _c.c_int64, _c.c_int64, _c.c_int64, _c.c_double, _vp, _vp]),
    "tr_plan_set_prepare_next": (_c.c_int, [_vp, _c.c_int]),
    "tr_plan_create_f64": (_c.c_int, [_c.POINTER(_vp), _c.c_int, _c.c_int, _c.POINTER(_c.c_int64), _c.c_int,
                                      _c.c_int64, _c.POINTER(_c.c_int32), _c.c_double, _c.c_double]),
    "tr_forward_f64": (_c.c_int, [_vp, _vp, _c.c_int64, _vp, _vp, _vp, _vp]),
    "tr_loss_grad_f64": (_c.c_int, [_vp, _vp, _c.c_int64, _vp, _c.c_double, _vp, _vp, _vp, _vp, _vp, _vp]),
    "tr_finalize_grad_f64": (_c.c_int, [_vp, _vp, _vp, _c.c_double, _vp, _vp, _vp]),
    "tr_adam_step_f64": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _c.c_double, _c.c_double, _c.c_double,
                                    _c.c_double, _c.c_double, _c.c_double, _c.c_int, _c.c_int64, _vp,
                                    _c.c_int64, _c.c_int64, _c.c_int64, _c.c_double, _vp, _vp]),
}

_lock = threading.Lock()
_lib = None


class HipLibraryError(RuntimeError):
    """The gfx950 extension is missing, stale, or a call into it failed."""


def source_build_id():
    """sha256 of the sources next to the package, exactly as the Makefile's build/tr_build_id.h
    computes it (csrc/*.hip and csrc/*.h in byte order of their names, then the public header);
    None when the sources are not shipped."""
    csrc = os.path.join(_HERE, "csrc")
    header = os.path.join(os.path.dirname(_HERE), "include", "tensor_regression_hip.h")
    if not os.path.isdir(csrc) or not os.path.exists(header):
        return None
    names = sorted(n for n in os.listdir(csrc) if n.endswith((".hip", ".h")))
    h = hashlib.sha256()
    for path in [os.path.join(csrc, n) for n in names] + [header]:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


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
        want = source_build_id()
        got = (lib.tr_build_id() or b"").decode()
        if want is not None and got != want and os.environ.get("TR_HIP_LIB") is None:
            raise HipLibraryError(f"{LIB_PATH} was built from other sources (build id {got[:12]}, sources "
                                  f"{want[:12]}); rebuild it with `make -C tensor_regression_amd/csrc`")
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
