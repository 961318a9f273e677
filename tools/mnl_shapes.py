#!/usr/bin/env python3
"""Kernel time and HBM fraction of the multinomial single pass across sample shapes (GPU box).

    python tools/mnl_shapes.py > gpurun_out/mnl_shapes.txt

For each (I, J) the sample count N fills ~2 GiB of X; fit_Adam runs 200 warm-up iterations, then
30 with the stream kernel timed by hipEvents.  Prints the plan's path (k_mnl_duo in its rank-block
or bf16-split form and its wave count, or k_mnl_fused, or the two-pass kernels) and the stream kernel's rate against
its algorithmic bytes (4 I J + 8 per sample) and the 8 TB/s HBM peak.
"""
import os
import sys

import numpy as np
import torch

# TR_PKG_ROOT: another copy of the package (an earlier round's, with TR_HIP_LIB its library) for A/B
sys.path.insert(0, os.environ.get("TR_PKG_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensor_regression_amd import CP_logistic_regression  # noqa: E402

dev = "cuda:0"
SHAPES = [((128, 64), 8), ((64, 128), 8), ((128, 64), 3), ((64, 64), 8), ((96, 64), 8), ((160, 64), 8),
          ((192, 64), 8), ((224, 64), 8), ((256, 64), 8), ((64, 64), 3), ((96, 128), 8), ((128, 128), 8),
          ((256, 128), 8), ((512, 64), 8), ((384, 64), 8), ((768, 64), 8), ((192, 128), 8), ((512, 128), 8)]
if len(sys.argv) > 1:  # a subset: "I,J" or "I,J,R" arguments (rank 8 by default)
    SHAPES = [((int(a.split(",")[0]), int(a.split(",")[1])), int(a.split(",")[2]) if a.count(",") > 1 else 8)
              for a in sys.argv[1:]]
C = 10
for (I, J), R in SHAPES:
    N = (1 << 29) // (I * J)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, I, J, device=dev, generator=g)
    y = torch.randint(0, C, (N,), device=dev, generator=g)
    y[:C] = torch.arange(C, device=dev)
    torch.manual_seed(1)
    m = CP_logistic_regression(X, y, rank=R, device=dev)
    kw = dict(lambda_L2=0.01, tol=0, patience=10, weights=np.ones(C), Adam_kwargs={"lr": 0.01})
    m.fit_Adam(max_iter=200, **kw)
    plan = m._plan
    plan.read_timing()
    plan.set_timing(True, kinds=["stream_fused", "stream_rows", "stream_cols"])
    m.fit_Adam(max_iter=30, **kw)
    plan.set_timing(False)
    kt = plan.read_timing()
    ms = {k: v[0] / v[1] for k, v in kt.items() if v[1]}
    tot = sum(ms.values())
    alg = N * (4 * I * J + 8)
    path = plan.describe.split(" path=")[1].split()[0]
    form = (f"duo {plan.describe.split('form=')[1].split()[0]} waves={plan.describe.split('waves=')[1].split()[0]}"
            f" nbuf={plan.describe.split('nbuf=')[1].split()[0]}"
            + (f" blocks={plan.describe.split('rowblocks=')[1].split()[0]}" if "rowblocks=" in plan.describe else "")
            if " duo " in plan.describe else path)
    print(f"(N, I, J) = ({N}, {I}, {J}) R={R}: {form:32s} stream kernels {tot:.4f} ms = "
          f"{alg / (tot * 1e-3) / 1e12:.2f} TB/s = {alg / (tot * 1e-3) / 8e12 * 100:.1f} % of HBM  {ms}", flush=True)
    del m, X, y
    torch.cuda.empty_cache()
