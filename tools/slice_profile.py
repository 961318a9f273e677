#!/usr/bin/env python3
"""Per-phase cycle breakdown of the column-slice spectral kernel (profiling build, GPU box).

    make -C tensor_regression_amd/csrc slice-variant V=prof VFLAGS=-DTR_SLICE_PROFILE=1
    TR_HIP_LIB=$PWD/tensor_regression_amd/libtr_hip_slice_prof.so python tools/slice_profile.py

Phases (wave 0 of each workgroup, __builtin_readcyclecounter deltas per sample): forward GEMM
(+ its LDS-DMA waits), exchange + barrier A, column partials + barrier B, y_hat / residual / dT,
gradient GEMM (+ the next sample's LDS-DMA issue).  With TR_SLICE_SKIP builds (timing only) the
same breakdown shows what each part costs when the others are removed.
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
    names = ["fwd GEMM (+waits)", "  of which DMA waits", "exchange write", "barrier A wait", "column partials",
             "barrier B wait", "yhat/resid/dT", "grad GEMM + DMA issue"]
    print(f"{'cycles / sample':26s}" + "".join(f"  wave{w}" for w in range(8)) + "     mean")
    for q, nm in enumerate(names):
        vals = [sum(buf[(b * 8 + w) * 8 + q] for b in range(256)) / 256 / per_wg for w in range(8)]
        print(f"{nm:26s}" + "".join(f"{v:7.0f}" for v in vals) + f"  {sum(vals) / 8:7.0f}")
    tot = [sum(buf[(b * 8 + w) * 8 + q] for b in range(256) for q in (0, 2, 3, 4, 5, 6, 7)) / 256 / per_wg
           for w in range(8)]
    print(f"{'total':26s}" + "".join(f"{v:7.0f}" for v in tot))
