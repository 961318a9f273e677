#!/usr/bin/env python3
"""Per-phase cycle breakdown of the 4-wave spectral kernel k_spec_quad (profiling build, GPU box).

    make -C tensor_regression_amd/csrc slice-variant V=prof VFLAGS=-DTR_SLICE_PROFILE=1
    TR_HIP_LIB=$PWD/tensor_regression_amd/libtr_hip_slice_prof.so python tools/quad_profile.py

Phases per sample (lane 0 of each wave of workgroups 0..255, __builtin_readcyclecounter deltas):
forward GEMMs (and, as a subset, the LDS-DMA waits in it), column partials, the barrier, the
post-barrier epilogue (Z / V, y_hat, residual, dT), the gradient GEMMs + next sample's DMA issue.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensor_regression_amd import _lib  # noqa: E402
from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression  # noqa: E402

N, W, D, O = int(os.environ.get("N", 32768)), 256, 129, 2
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(N, W, D, device=dev, generator=g).abs_()
y = torch.randn(N, O, device=dev, generator=g)
torch.manual_seed(1)
m = CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=dev)
m.fit_Adam(X, y, lambda_L2=0.01, max_iter=3, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
torch.cuda.synchronize()
plan = m._plan
plan.set_timing(True, kinds=["stream_fused"])
m.fit_Adam(X, y, lambda_L2=0.01, max_iter=5, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
torch.cuda.synchronize()
kt = plan.read_timing()
ms = kt["stream_fused"][0] / max(1, kt["stream_fused"][1])
print(f"lib {os.environ.get('TR_HIP_LIB', 'default')}: kernel {ms:.4f} ms  plan {plan.describe}")
lib = _lib.load()
if hasattr(lib, "tr_slice_profile_read"):
    fn = lib.tr_slice_profile_read
    fn.restype = ctypes.c_int
    buf = (ctypes.c_ulonglong * (256 * 8 * 8))()
    assert fn(buf) == 0
    per_wg = N // 256
    names = {0: "forward GEMMs (+waits)", 6: "  of which DMA waits", 1: "column partials", 2: "barrier wait",
             4: "Z/V, y_hat, resid, dT", 5: "gradient GEMMs + DMA"}
    print(f"{'cycles / sample':26s}" + "".join(f"  wave{w}" for w in range(4)) + "     mean")
    for q, nm in names.items():
        vals = [sum(buf[(b * 8 + w) * 8 + q] for b in range(256)) / 256 / per_wg for w in range(4)]
        print(f"{nm:26s}" + "".join(f"{v:7.0f}" for v in vals) + f"  {sum(vals) / 4:7.0f}")
    tot = [sum(buf[(b * 8 + w) * 8 + q] for b in range(256) for q in (0, 1, 2, 4, 5)) / 256 / per_wg
           for w in range(4)]
    print(f"{'total':26s}" + "".join(f"{v:7.0f}" for v in tot))
