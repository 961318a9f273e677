#!/usr/bin/env python3
"""Host-side timeline of a config's first fit_Adam call (two iterations) with the HIP runtime's
own API log: run as  AMD_LOG_LEVEL=3 python tools/first_fit_log.py c5 2> log  and read the
timestamps around the kernel launches between the MARK lines (a first-call stall shows as a
gap in the HIP calls)."""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c5"
    cfg = bench.CONFIGS[name]
    dev = "cuda:0"
    X, y = bench.make_data(cfg, 0, dev)
    torch.cuda.synchronize()
    torch.manual_seed(1)
    if cfg["kind"] == "spectral":
        from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression as SpectralCP
        model = SpectralCP(X.shape, y.shape, rank_normal=cfg["rank"], rank_spectral=cfg["rank_spectral"],
                           n_complex_dim=cfg["n_complex_dim"], device=dev)
        fit = lambda n: model.fit_Adam(X, y, lambda_L2=0.01, max_iter=n, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    elif cfg["kind"] == "linear":
        from tensor_regression_amd import CP_linear_regression
        model = CP_linear_regression(X.shape, rank=cfg["rank"], device=dev)
        fit = lambda n: model.fit_Adam(X, y, lambda_L2=0.01, max_iter=n, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    else:
        from tensor_regression_amd import CP_logistic_regression
        model = CP_logistic_regression(X, y, rank=cfg["rank"], device=dev)
        cw = np.ones(cfg["classes"], np.float32)
        fit = lambda n: model.fit_Adam(lambda_L2=0.01, max_iter=n, tol=0, patience=10, weights=cw,
                                       Adam_kwargs={"lr": 0.01})
    for k in range(2):
        t0 = time.perf_counter()
        print(f"MARK fit {k} start", file=sys.stderr, flush=True)
        fit(2)
        torch.cuda.synchronize()
        print(f"MARK fit {k} end {1e3 * (time.perf_counter() - t0):.2f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
