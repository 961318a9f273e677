#!/usr/bin/env python3
"""Kernel path and stream-kernel rate of the linear (standard) fit across sample shapes (GPU box).

    python tools/lin_shapes.py [I,J[,K] ...] > gpurun_out/lin_shapes.txt

For each sample shape, N fills ~2 GiB of X; fit_Adam runs 100 warm-up iterations, then 30 with
the X-streaming kernels timed by hipEvents; prints the plan's path and the rate against one read
of X (8 TB/s).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensor_regression_amd import CP_linear_regression  # noqa: E402

dev = "cuda:0"
SHAPES = [(256, 128), (100, 100), (160, 160), (250, 130), (99, 97), (64, 64, 30), (300, 300)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for shape in SHAPES:
    P = 1
    for d in shape:
        P *= d
    N = (1 << 29) // P
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn((N,) + shape, device=dev, generator=g)
    y = torch.randn(N, device=dev, generator=g)
    torch.manual_seed(1)
    m = CP_linear_regression(X.shape, rank=8, device=dev)
    kw = dict(lambda_L2=0.01, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    m.fit_Adam(X, y, max_iter=100, **kw)
    plan = m._plan
    plan.read_timing()
    plan.set_timing(True, kinds=["stream_fused", "stream_rows", "stream_cols"])
    m.fit_Adam(X, y, max_iter=30, **kw)
    plan.set_timing(False)
    kt = plan.read_timing()
    ms = {k: v[0] / v[1] for k, v in kt.items() if v[1]}
    tot = sum(ms.values())
    xb = N * P * 4
    path = plan.describe.split(" path=")[1].split()[0]
    print(f"(N, sample) = ({N}, {shape}): {path:22s} stream kernels {tot:.4f} ms = {xb / (tot * 1e-3) / 1e12:.2f} TB/s "
          f"= {xb / (tot * 1e-3) / 8e12 * 100:.1f} % of HBM  {ms}", flush=True)
    del m, X, y
    torch.cuda.empty_cache()
