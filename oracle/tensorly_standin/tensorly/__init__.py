"""Minimal stand-in for the three `tensorly` entry points the reference's hot path calls.

TEST INFRASTRUCTURE ONLY (see oracle/README.md): this package exists so that the
read-only reference under /root/reference can be imported in the build container to
generate golden fixtures (tools/gen_golden.py).  It never travels into the product
path, and nothing in `tensor_regression_amd/` imports it.

`tensorly` is an un-vendored third-party dependency of the reference with NO pinned
version (no requirements/lock file; notebooks show only `import tensorly as tl`).  The
semantics below restate tensorly's published pytorch-backend algorithm (SURVEY.md
Appendix C) for exactly the functions the reference calls:

  * tl.set_backend('pytorch')                      standard_tensor_regression.py:364,451
  * tl.cp_tensor.cp_to_tensor((weights, factors))  standard_tensor_regression.py:124,
                                                   multinomial_tensor_regression.py:182
  * tl.tenalg.inner(X, B, n_modes)                 standard_tensor_regression.py:123-130,
                                                   multinomial_tensor_regression.py:181-186

The stand-in is pinned by the notebooks' printed traces (KAT-1 / KAT-2, tests/golden).
"""
from . import cp_tensor, tenalg  # noqa: F401

_BACKEND = "pytorch"


def set_backend(name):
    """No-op backend switch; only the pytorch backend is restated."""
    global _BACKEND
    _BACKEND = name


def get_backend():
    return _BACKEND
