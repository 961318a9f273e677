#!/usr/bin/env python3
"""Fixed per-call cost of fit_Adam (everything outside the per-iteration launches).

    python tools/fit_overhead.py [--config c3] [--profile]

Times fit_Adam(max_iter=n) for several n on bench.py's synthetic workload; the intercept of
time(n) = a + n * b is the per-call cost (argument checks, parameter packing, state buffers,
the final loss history / parameter copy-back) that a short fit pays once.  --profile prints the
host-side cProfile of fit_Adam(max_iter=1).
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = "cuda:0"
    X, y = bench.make_data(cfg, cfg["rows"], 0, dev)
    torch.manual_seed(1)
    R = cfg["rank"]
    if cfg["kind"] == "spectral":
        from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression as SpectralCP
        model = SpectralCP(X.shape, y.shape, rank_normal=R, rank_spectral=cfg["rank_spectral"],
                           n_complex_dim=cfg["n_complex_dim"], device=dev)
        fit = lambda n: model.fit_Adam(X, y, lambda_L2=0.01, max_iter=n, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    elif cfg["kind"] == "linear":
        from tensor_regression_amd import CP_linear_regression
        model = CP_linear_regression(X.shape, rank=R, device=dev)
        fit = lambda n: model.fit_Adam(X, y, lambda_L2=0.01, max_iter=n, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    else:
        from tensor_regression_amd import CP_logistic_regression
        model = CP_logistic_regression(X, y, rank=R, device=dev)
        cw = np.ones(cfg["classes"], np.float32)
        fit = lambda n: model.fit_Adam(lambda_L2=0.01, max_iter=n, tol=0, patience=10, weights=cw,
                                       Adam_kwargs={"lr": 0.01})
    fit(5)
    res = {}
    for n in (1, 2, 10, 50, 200):
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fit(n)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[n] = min(ts)
        print(f"{args.config} fit_Adam(max_iter={n:4d}): {1e3 * res[n]:9.3f} ms  ({1e3 * res[n] / n:.4f} ms/iter)",
              flush=True)
    b = (res[200] - res[50]) / 150
    a = res[50] - 50 * b
    print(f"{args.config}: per-iteration {1e3 * b:.4f} ms, per-call {1e3 * a:.3f} ms", flush=True)
    if args.profile:
        reps = 50
        pr = cProfile.Profile()
        torch.cuda.synchronize()
        pr.enable()
        for _ in range(reps):
            fit(1)
        torch.cuda.synchronize()
        pr.disable()
        st = pstats.Stats(pr).stats
        rows = sorted(((ct / reps, tt / reps, nc / reps, f"{os.path.basename(k[0])}:{k[1]}({k[2]})")
                       for k, (cc, nc, tt, ct, _) in st.items()), reverse=True)
        print(f"host profile of fit_Adam(max_iter=1), mean over {reps} calls (us): cum / own / calls per fit")
        for ct, tt, nc, name in rows[:40]:
            print(f"  {1e6 * ct:9.1f} {1e6 * tt:9.1f} {nc:6.1f}  {name}")

if __name__ == "__main__":
    main()
