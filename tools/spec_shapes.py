#!/usr/bin/env python3
"""Step time of the spectral fit across sample shapes (GPU box).

    python tools/spec_shapes.py > gpurun_out/spec_shapes.txt

For each (W, D) the sample count N fills ~2 GiB of |randn| X; rank_normal = rank_spectral = 8,
n_complex_dim 1, n_out 2.  fit_Adam runs 50 warm-up iterations, then 30 timed ones; prints the
plan's kernel path and the step time against the HBM time of one read of X (8 TB/s).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression  # noqa: E402

dev = "cuda:0"
SHAPES = [(256, 129), (256, 100), (256, 97), (256, 96), (256, 65), (128, 129), (128, 65), (512, 129), (256, 257)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for W, D in SHAPES:
    N = (1 << 29) // (W * D)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, W, D, device=dev, generator=g).abs_()
    y = torch.randn(N, 2, device=dev, generator=g)
    torch.manual_seed(1)
    try:
        m = CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=dev)
        kw = dict(lambda_L2=0.01, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
        m.fit_Adam(X, y, max_iter=50, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.fit_Adam(X, y, max_iter=30, **kw)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / 30
        desc = m._plan.describe
        path = desc.split(" path=")[1].split()[0] if " path=" in desc else desc[:40]
        xb = N * W * D * 4
        print(f"(N, W, D) = ({N}, {W}, {D}): {path:36s} {ms:8.4f} ms/step = {xb / (ms * 1e-3) / 1e12:.2f} TB/s "
              f"= {xb / (ms * 1e-3) / 8e12 * 100:.1f} % of HBM (X read once)", flush=True)
    except Exception as e:  # an envelope error is a result too
        print(f"(N, W, D) = ({N}, {W}, {D}): {type(e).__name__}: {e}", flush=True)
    del X, y
    torch.cuda.empty_cache()
