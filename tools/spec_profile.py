#!/usr/bin/env python3
"""Per-phase cycle breakdown of the spectral kernel (profiling build, GPU box).

    make -C tensor_regression_amd/csrc prof
    TR_HIP_LIB=$PWD/tensor_regression_amd/libtr_hip_prof.so python tools/spec_profile.py

Phases (wave 0 of each workgroup, __builtin_readcyclecounter deltas): forward GEMM (with the
LDS-DMA waits), column sums, y_hat/residual/small-factor grads, dT + A1/C1 grads, gradient GEMM
(with the per-block barrier + next-sample DMA issue); two sub-totals split out the waits.
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
lib = _lib.load()
fn = lib.tr_spec_profile_read
fn.restype = ctypes.c_int
buf = (ctypes.c_ulonglong * (256 * 8))()
assert fn(buf) == 0
rows = [[buf[b * 8 + q] for q in range(8)] for b in range(256)]
per_wg = N // 256
names = ["fwd GEMM (+DMA waits)", "column sums", "yhat/resid/small grads", "dT + A1/C1 grads", "grad GEMM + DMA issue",
         "  of which DMA waits (fwd)", "  of which barrier+DMA issue (grad)"]
tot = 0
for q, nm in enumerate(names):
    avg = sum(r[q] for r in rows) / 256 / per_wg
    if q < 5:
        tot += avg
    print(f"{nm:36s} {avg:10.0f} cycles/sample")
print(f"{'total':32s} {tot:10.0f} cycles/sample  (x {per_wg} samples/WG)")
