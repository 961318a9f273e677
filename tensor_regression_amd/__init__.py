"""tensor_regression_amd — MI355X (gfx950) CP tensor-regression fitter.

Drop-in for the hot path of kimerein/tensor_regression: `standard_tensor_regression`
(CP_linear_regression), `multinomial_tensor_regression` (CP_logistic_regression) and
`spectral_tensor_regression` (the spectral CP_linear_regression, config 5) keep the
reference's Python API and Kruskal-factor list layout; the forward / loss / gradient / Adam
loop runs as hand-written HIP kernels behind the C ABI in include/tensor_regression_hip.h.
"""
from . import _lib  # noqa: F401
from . import standard_tensor_regression  # noqa: F401
from . import multinomial_tensor_regression  # noqa: F401
from . import spectral_tensor_regression  # noqa: F401
from .standard_tensor_regression import CP_linear_regression  # noqa: F401
from .multinomial_tensor_regression import CP_logistic_regression  # noqa: F401

__version__ = "0.1.0"
