"""tensorly.cp_tensor.cp_to_tensor restated (TEST INFRASTRUCTURE ONLY).

Algorithm (tensorly pytorch backend):
  khatri_rao(F, skip_matrix=0): drop F[0]; fold the rest left to right with the first
  matrix's row index varying slowest:  res = reshape(res[:, None, :] * e[None, :, :], (-1, R)).
  cp_to_tensor((w, F)) = reshape((F[0] * w) @ khatri_rao(F, skip 0).T, [f.shape[0] for f in F]);
  for a single factor: sum(w * F[0], dim=1).
"""
import torch


def _khatri_rao_skip_first(factors):
    mats = list(factors[1:])
    res = mats[0]
    for e in mats[1:]:
        res = torch.reshape(res[:, None, :] * e[None, :, :], (-1, res.shape[1]))
    return res


def cp_to_tensor(cp_tensor, mask=None):
    weights, factors = cp_tensor
    factors = list(factors)
    shape = [f.shape[0] for f in factors]
    if len(factors) == 1:
        return torch.sum(weights * factors[0], dim=1)
    if weights is None:
        left = factors[0]
    else:
        left = factors[0] * weights
    full = torch.matmul(left, torch.transpose(_khatri_rao_skip_first(factors), 0, 1))
    return torch.reshape(full, shape)
