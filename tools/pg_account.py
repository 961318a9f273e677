#!/usr/bin/env python3
"""Where the sharded fit's extra time goes at world size 1 (GPU box): bench.py's config-2 step
through fit_Adam with and without an RCCL ("nccl") process group, alternating, and the host wall
time of every collective / host sync of the process-group path, per fit call.

    python tools/pg_account.py [--config c2] [--steps 20] [--reps 6] > gpurun_out/pg_account.json

Each timed fit is bracketed like bench.py's timed region (synchronize + barrier on both sides;
the barrier is a no-op without a group).  The phase timers are host wall clock around the calls
(the collectives' own host syncs included), summed per fit call.
"""
import argparse
import collections
import functools
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TR_PKG_ROOT: another copy of the package (an earlier round's, with TR_HIP_LIB its library) for A/B
sys.path.insert(0, os.environ.get("TR_PKG_ROOT", ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    pg = dist.group.WORLD
    from tensor_regression_amd import CP_linear_regression, CP_logistic_regression, _engine
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    if args.config == "c2":
        X = torch.randn(65536, 256, 128, device=dev, generator=g)
        y = torch.randn(65536, device=dev, generator=g)
        model = CP_linear_regression(X.shape, rank=8, device=dev)

        def fit(k, group):
            model.fit_Adam(X, y, lambda_L2=0.01, max_iter=k, tol=0, patience=10, Adam_kwargs={"lr": 0.01},
                           process_group=group)
    else:
        X = torch.randn(65536, 128, 64, device=dev, generator=g)
        y = torch.randint(0, 10, (65536,), device=dev, generator=g)
        model = CP_logistic_regression(X, y, rank=8, device=dev)

        def fit(k, group):
            model.fit_Adam(lambda_L2=0.01, max_iter=k, tol=0, patience=10, weights=np.ones(10, np.float32),
                           Adam_kwargs={"lr": 0.01}, process_group=group)

    acc = collections.defaultdict(float)
    cnt = collections.defaultdict(int)

    def timed(obj, name, label):
        f = getattr(obj, name)

        @functools.wraps(f)
        def w(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[label] += time.perf_counter() - t
                cnt[label] += 1
        setattr(obj, name, w)

    for name in ("all_reduce", "broadcast", "barrier", "all_gather"):
        timed(dist, name, f"dist.{name}")
    for name in ("agree", "sync_replicas", "check_uniform", "fit_start"):
        if hasattr(_engine, name):
            timed(_engine, name, f"_engine.{name}")
    timed(_engine, "gradient_allreduce", "_engine.gradient_allreduce")
    if hasattr(_engine, "RcclAllReduce"):
        for name in ("max_f64", "broadcast", "barrier"):
            if hasattr(_engine.RcclAllReduce, name):
                timed(_engine.RcclAllReduce, name, f"RcclAllReduce.{name}")
    timed(_engine, "_adam_loop", "_engine._adam_loop")

    comm = _engine.direct_comm(pg, 0) if hasattr(_engine, "direct_comm") else None

    def bracket(group):  # as bench.py's timed region
        torch.cuda.synchronize()
        if group is not None:
            if comm is not None:
                comm.barrier()
            else:
                dist.barrier()

    fit(5, None)
    fit(5, pg)
    out = {"config": args.config, "steps": args.steps, "local_ms_per_step": [], "pg_ms_per_step": [], "phases": []}
    for r in range(args.reps):
        for group in (None, pg):
            bracket(group)
            acc.clear()
            cnt.clear()
            t0 = time.perf_counter()
            fit(args.steps, group)
            bracket(group)
            el = time.perf_counter() - t0
            key = "pg_ms_per_step" if group is not None else "local_ms_per_step"
            out[key].append(1e3 * el / args.steps)
            if group is not None:
                out["phases"].append({k: [round(1e6 * v, 1), cnt[k]] for k, v in sorted(acc.items())})
    out["local_median"] = float(np.median(out["local_ms_per_step"]))
    out["pg_median"] = float(np.median(out["pg_ms_per_step"]))
    out["pg_minus_local_us_per_step"] = 1e3 * (out["pg_median"] - out["local_median"])
    out["phase_note"] = "phases: [host us per fit call, calls]; the bracketing barrier after the fit is dist.barrier"
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
