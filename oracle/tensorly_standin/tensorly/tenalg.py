"""tensorly.tenalg.inner restated (TEST INFRASTRUCTURE ONLY).

inner(t1, t2, n_modes): n_modes None -> sum(t1 * t2); otherwise the trailing n_modes of
t1 must equal the leading n_modes of t2 (ValueError otherwise), and the result is
reshape(reshape(t1, (-1, P)) @ reshape(t2, (P, -1)), t1.shape[:-n] + t2.shape[n:]).
"""
import numpy as np
import torch


def inner(tensor1, tensor2, n_modes=None):
    if n_modes is None:
        if tensor1.shape != tensor2.shape:
            raise ValueError(
                "Taking a generalised product between two tensors without specifying common modes"
                f" is equivalent to taking inner product. This requires tensor1.shape == tensor2.shape."
                f" However, got tensor1.shape={tensor1.shape} and tensor2.shape={tensor2.shape}")
        return torch.sum(tensor1 * tensor2)
    shape_t1 = list(tensor1.shape)
    shape_t2 = list(tensor2.shape)
    common_modes = shape_t1[len(shape_t1) - n_modes:]
    if common_modes != shape_t2[:n_modes]:
        raise ValueError(
            f"Incorrect shapes for inner product along {n_modes} common modes."
            f" tensor_1.shape={shape_t1}, tensor_2.shape={shape_t2}")
    common_size = int(np.prod(common_modes))
    output_shape = shape_t1[:-n_modes] + shape_t2[n_modes:]
    a = torch.reshape(tensor1, (-1, common_size))
    b = torch.reshape(tensor2, (common_size, -1))
    return torch.reshape(torch.matmul(a, b), output_shape)
