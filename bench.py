#!/usr/bin/env python3
"""Benchmark: CP tensor-regression fit_Adam iterations on MI355X (gfx950 HIP path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--scaling weak|strong]
                    [--no-cpu-baseline]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N ...   (N > 1)

--scaling weak (default): every rank holds the config's per-GPU sample count (c4: 16384);
--scaling strong: the config's total (c4: the 131072 samples of BASELINE configs[3], 68.7 GB of X
on one GPU at N = 1) split over the ranks.  Samples come from one synthetic global dataset
(seeded by 4096-row blocks), so a rank's shard is the same rows whichever mode or N made it.
For N > 1 the line carries a "ranks" block: RCCL's own rank count (ncclCommCount), the sampled
all-reduce time per step, every rank's dominant-kernel average, time and rate.

`--gpus N` outside a launcher (no WORLD_SIZE in the environment) starts the N ranks itself: one
child process per GPU with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT
set as torchrun sets them, so the N > 1 path is the one torchrun runs; the parent never touches
the GPU, passes rank 0's JSON line through and exits non-zero (no JSON line) if any rank fails
or fewer than N devices are visible.  Under a launcher, WORLD_SIZE must equal --gpus.

A "step" is one fit_Adam iteration of the reference (standard_tensor_regression.py:458-470):
forward + MSE (+L2) + gradient + Adam over every sample the rank holds.  Default workload =
BASELINE.json configs[1]: X (65536, 256, 128) fp32 per GPU, rank 8 (weak scaling: every rank
holds its own 65536-sample shard; one RCCL all-reduce of the gradient arena per step).
Inputs are synthetic (seeded torch.randn on the device; planted rank-8 model + noise) and are
resident in HBM before the timed region.  `value` = samples processed by all ranks / max-over-
ranks wall time of the K timed steps.  The default warm-up (200 untimed iterations, < 0.5 s) brings
the GPU to its steady clock first: the latency-bound multinomial kernel runs 9 % faster after 50
iterations than after 5 (tools/warmup_sweep.sh); the HBM-bound c2 kernel does not change.

roofline: the dominant kernel (the single-pass X stream, k_linear_fused) timed with hipEvents on
its own stream during the timed region; algorithmic bytes per launch = N*P*4 (X read once) +
N*4 (y).  cpu_baseline: the oracle (a torch-CPU restatement of the reference's op sequence,
oracle/cp_oracle.py) timed on this host on the same X for a bounded number of iterations.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "training samples/sec + achieved HBM GB/s, 3-D CP regression rank=8, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    "c2": dict(kind="linear", rows=65536, total_rows=65536, dims=(256, 128), rank=8, expect="fused-1pass",
               workload="configs[1]: 3-D standard CP regression, X (65536, 256, 128) fp32 per GPU, rank 8, "
                        "MSE + L2 (lambda 0.01), Adam lr 0.01"),
    "c3": dict(kind="multinomial", rows=65536, total_rows=65536, dims=(128, 64), rank=8, classes=10,
               expect="mnl-fused-1pass",
               workload="configs[2]: multinomial CP regression, X (65536, 128, 64) fp32 per GPU, 10 classes, "
                        "rank 8, softmax + weighted CE + L2, Adam lr 0.01"),
    "c4": dict(kind="linear", rows=16384, total_rows=131072, cpu_rows=16384, dims=(64, 64, 32), rank=16,
               expect="cluster-1pass",
               workload="configs[3]: 4-D CP regression, X (131072, 64, 64, 32) sharded 16384 samples per GPU "
                        "(--scaling strong: the 131072 samples split over the ranks), rank 16, Adam lr 0.01"),
    "c5": dict(kind="spectral", rows=32768, total_rows=32768, dims=(256, 129), rank=8, rank_spectral=8,
               n_complex_dim=1, n_out=2,
               expect="slice-1pass-mfma",
               workload="configs[4]: spectral_tensor_regression.py fit_Adam, X (32768, 256, 129) fp32 (real: the "
                        "reference rejects complex X; |rfft|-like non-negative synthetic data), rank_normal = "
                        "rank_spectral = 8, n_complex_dim 1, y (32768, 2), Adam lr 0.01"),
}
CONFIGS["c6"] = dict(kind="linear", rows=65536, dims=(256, 128), rank=8, windowed=True, expect="fused-1pass",
                     workload="windowed variant of configs[1] (util.py:67-114 WindowedDataset): 65536 windows of "
                              "256 x 128 over an untiled (65791, 128) fp32 series, read in place through the row "
                              "stride (no materialised windows), rank 8, Adam lr 0.01")
CONFIGS["c7"] = dict(kind="linear", rows=65536, dims=(256, 128), rank=8, hoststream=True, chunk_rows=8192,
                     expect="fused-1pass", default_warmup=3,
                     workload="out-of-core variant of configs[1] (util.py HostStream): X (65536, 256, 128) fp32 in "
                              "pinned host memory, streamed through two 1 GiB HBM buffers in 8 chunks of 8192 "
                              "samples every iteration (copies on their own stream, double-buffered against the "
                              "kernels), rank 8, Adam lr 0.01")
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 = the fp32 vector rate


class _Phases:
    """TR_BENCH_PHASES=1: host time of each set-up phase around the timed fit, on stderr"""
    def __init__(self):
        self.on = os.environ.get("TR_BENCH_PHASES") == "1"
        self.t = time.perf_counter()

    def __call__(self, what):
        if self.on:
            now = time.perf_counter()
            log(f"bench phase {what}: {1e3 * (now - self.t):.3f} ms")
            self.t = now


def log(*a):
    print(*a, file=sys.stderr, flush=True)


DATA_BLOCK = 4096  # rows per seeded generator block of the synthetic global dataset


def shard_rows(total, world, rank_id):
    """(row0, rows) of this rank's contiguous shard of `total` samples (the first total % world
    ranks take one more)."""
    base, extra = divmod(int(total), int(world))
    rows = base + (1 if rank_id < extra else 0)
    return rank_id * base + min(rank_id, extra), rows


def _block_gen(dev, b):
    return torch.Generator(device=dev).manual_seed(1234 + b)


def make_data(cfg, rows, row0, dev):
    """Seeded synthetic shard: global rows [row0, row0 + rows) of one synthetic dataset (X ~ N(0,1)
    by DATA_BLOCK-row blocks, each from its own seed, so a sample is the same whatever the rank
    count or the scaling mode), a planted CP model (identical on every rank) and y / labels."""
    N, dims, R = rows, cfg["dims"], cfg["rank"]
    if cfg.get("windowed"):
        from tensor_regression_amd.util import windowed_view
        L = dims[0]
        g = _block_gen(dev, 0)
        Xu = torch.randn((N + L - 1,) + tuple(dims[1:]), device=dev, generator=g, dtype=torch.float32)
        X, _ = windowed_view(Xu, torch.zeros(N + L - 1, device=dev), (0, L))
    else:
        X = torch.empty((N,) + tuple(dims), device=dev, dtype=torch.float32)
        for b in range(row0 // DATA_BLOCK, -(-(row0 + N) // DATA_BLOCK)):
            blk = torch.randn((DATA_BLOCK,) + tuple(dims), device=dev, generator=_block_gen(dev, b),
                              dtype=torch.float32)
            lo, hi = max(row0, b * DATA_BLOCK), min(row0 + N, (b + 1) * DATA_BLOCK)
            X[lo - row0:hi - row0] = blk[lo - b * DATA_BLOCK:hi - b * DATA_BLOCK]
            del blk
    gn = torch.Generator(device=dev).manual_seed(4321 + row0)  # noise / label draws of this shard
    gc = torch.Generator().manual_seed(99)  # planted factors identical on every rank
    if cfg["kind"] == "spectral":
        from tensor_regression_amd.spectral_tensor_regression import lin_model as spec_lin
        X.abs_()  # magnitude-spectrum-like (non-negative) features
        O = cfg["n_out"]
        A = [(torch.randn(d, R, 1, generator=gc) / 8).to(dev) for d in dims] + [torch.randn(O, R, 1, generator=gc).to(dev)]
        y = spec_lin(X, A, torch.ones(R, device=dev), [False] * 3, torch.zeros(O, device=dev))
        y = y + 0.1 * torch.randn(N, O, device=dev, generator=gn)
        return X, y
    if cfg["kind"] == "linear":
        from tensor_regression_amd.standard_tensor_regression import lin_model
        A = [(torch.randn(d, R, generator=gc) / 4).to(dev) for d in dims]
        y = lin_model(X, A, torch.ones(R, device=dev), [False] * len(A), torch.zeros(1, device=dev))
        y = y + 0.1 * torch.randn(N, device=dev, generator=gn)
        return X, y
    from tensor_regression_amd.multinomial_tensor_regression import model as mnl_model
    C = cfg["classes"]
    A = [(torch.randn(d, R, generator=gc) / 3).to(dev) for d in dims] + [torch.randn(C, R, generator=gc).to(dev)]
    S = mnl_model(X, A, torch.ones(R, device=dev), [False] * len(A))
    y = torch.multinomial(S, 1, generator=gn).reshape(-1)
    if N >= C:
        y[:C] = torch.arange(C, device=dev)  # every class present in every shard
    return X, y


def host_cpu_info():
    """Cores this process may run on (affinity), the machine's logical CPUs and the physical
    cores among the allowed CPUs (distinct (package, core) pairs in /proc/cpuinfo)."""
    allowed = sorted(os.sched_getaffinity(0))
    phys = None
    try:
        cores, cur = set(), {}
        with open("/proc/cpuinfo") as f:
            for line in f:
                if ":" in line:
                    k, v = (s.strip() for s in line.split(":", 1))
                    cur[k] = v
                elif cur:
                    if int(cur.get("processor", -1)) in allowed:
                        cores.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
        if cur and int(cur.get("processor", -1)) in allowed:
            cores.add((cur.get("physical id"), cur.get("core id")))
        phys = len(cores) or None
    except (OSError, ValueError):
        pass
    return {"affinity_cpus": len(allowed), "os_cpu_count": os.cpu_count(), "physical_cores_allowed": phys,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(cfg, X, y, model_init, budget_s=15.0, threads=None):
    """Oracle (reference op sequence on torch CPU) on the same X: 2 warm-up + >= 5 timed
    iterations at the full per-GPU size.  Threads: the host's CPU quota for this
    job (OMP_NUM_THREADS, which the GPU pool sets to this box's share of the host) or, without
    one, every CPU in the affinity mask.  On the pool's boxes the mask shows all 256 CPUs of a
    host shared with other jobs: 256 threads measured 4x (c2) to 10x (c3) slower than 16."""
    from oracle import cp_oracle
    info = host_cpu_info()
    quota = os.environ.get("OMP_NUM_THREADS")
    nthreads = threads or (int(quota) if quota and quota.isdigit() else info["affinity_cpus"])
    torch.set_num_threads(nthreads)
    cap = cfg.get("cpu_rows")
    if cap and X.shape[0] > cap:  # bounded sample of the workload: the first cap samples
        X, y = X[:cap], y[:cap]
    Xc = X.cpu()
    yc = y.cpu()
    R = cfg["rank"]
    lam, adam = 0.01, {"lr": 0.01}

    def run(iters):
        if cfg["kind"] == "spectral":
            return cp_oracle.fit_adam_spectral(Xc, yc, model_init[0], model_init[1], np.zeros(cfg["n_out"], np.float32),
                                               np.ones(R + cfg["rank_spectral"], np.float32), R, [False] * 3, lam,
                                               iters, 0.0, 10, adam)
        if cfg["kind"] == "linear":
            return cp_oracle.fit_adam_linear(Xc, yc, model_init[0], model_init[1], np.ones(R, np.float32),
                                             [False] * len(cfg["dims"]), lam, iters, 0.0, 10, adam)
        return cp_oracle.fit_adam_mnl(Xc, yc, model_init[0], np.ones(R, np.float32),
                                      [False] * (len(cfg["dims"]) + 1), np.ones(cfg["classes"], np.float32), lam,
                                      iters, 0.0, 10, adam)

    t0 = time.perf_counter()
    run(2)  # warm-up: 2 iterations (allocator, thread pool)
    t1 = time.perf_counter()
    per = max((t1 - t0) / 2, 1e-3)
    iters = int(max(5, min(200, budget_s / per)))
    log(f"cpu baseline: {nthreads} threads, {per:.2f} s/iteration, timing {iters} iterations one by one")
    times = []
    load0 = os.getloadavg()
    for k in range(iters):  # each timed alone: one fit_Adam iteration (the op sequence of every later one)
        t0 = time.perf_counter()
        run(1)
        times.append(time.perf_counter() - t0)
        if k % 5 == 4 or k == iters - 1:
            log(f"cpu baseline: {k + 1}/{iters} iterations, {sum(times):.1f} s")
    load1 = os.getloadavg()
    t = np.array(times)
    med, lo, hi = float(np.median(t)), float(t.min()), float(t.max())
    spread = hi / lo
    N = X.shape[0]
    note = (f"; per-iteration spread {spread:.1f}x > 2x: the host is shared (load average {load0[0]:.0f} -> "
            f"{load1[0]:.0f} on {info['os_cpu_count']} CPUs), the median is the reported value"
            if spread > 2.0 else "")
    return {"value": N / med, "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/cp_oracle.py fit_Adam (torch {torch.__version__} CPU, the reference's op order) on "
                      f"the same {N} x {list(cfg['dims'])} X ("
                      f"{'full per-GPU size' if not cap or N < cap else f'the first {N} samples of the GPU shard'}"
                      f"): {iters} iterations each timed "
                      f"alone after 2 warm-up ({t.sum():.1f} s), value = N / median iteration time, "
                      f"torch.set_num_threads({nthreads}) "
                      f"({'OMP_NUM_THREADS quota of this job' if threads is None and quota else 'threads'})" + note,
            "iteration_s": {"median": med, "min": lo, "max": hi, "spread_max_over_min": spread, "n": iters},
            "samples_per_s_range": [N / hi, N / lo], "loadavg_1min": [load0[0], load1[0]],
            "host": info, "ms_per_step": 1e3 * med}


def host_stream_report(model, hs, Xres, y, fit, ms_step, dev):
    """Out-of-core fit (util.HostStream): H2D rate of the streamed fit against this host's pinned
    copy rate, and how much of the copy time the kernels hide.
      copy_only_ms     every chunk of X copied through the two buffers, no kernels
      compute_only_ms  the same fit step with X resident in HBM
      overlap          (copy_only + compute_only - step) / min(copy_only, compute_only): 1 = the
                       shorter of the two is completely hidden behind the longer."""
    nbytes = hs.X.numel() * 4
    torch.cuda.synchronize()
    # pinned H2D peak: one 1 GiB copy from the same pinned X, best of 3
    n = min(hs.X.numel(), 1 << 28)
    dst = torch.empty(n, dtype=torch.float32, device=dev)
    src = hs.X.reshape(-1)[:n]
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src, non_blocking=True)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    del dst
    peak = n * 4 / (best * 1e-3) / 1e9
    # copy only: the stream's own chunk loop with no kernels
    reps = 3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for _c in hs.chunks():
            pass
    torch.cuda.synchronize()
    copy_ms = 1e3 * (time.perf_counter() - t0) / reps
    # compute only: the same model, X resident (a fresh plan for the resident rows)
    state = [a.detach().clone() for a in model.Bcp], model.bias.detach().clone(), list(model.loss_running)
    k = 20
    model.fit_Adam(Xres, y, lambda_L2=0.01, max_iter=3, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.fit_Adam(Xres, y, lambda_L2=0.01, max_iter=k, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    torch.cuda.synchronize()
    compute_ms = 1e3 * (time.perf_counter() - t0) / k
    with torch.no_grad():
        for a, b in zip(model.Bcp, state[0]):
            a.copy_(b)
        model.bias.copy_(state[1])
    model.loss_running[:] = state[2]
    h2d = nbytes / (ms_step * 1e-3) / 1e9
    overlap = (copy_ms + compute_ms - ms_step) / min(copy_ms, compute_ms)
    return {"h2d_GBps": h2d, "pinned_copy_peak_GBps": peak, "h2d_frac_of_peak": h2d / peak,
            "copy_only_ms": copy_ms, "compute_only_ms": compute_ms, "step_ms": ms_step,
            "overlap_hidden_frac": overlap, "chunk_rows": hs.chunk_rows, "bytes_per_step": nbytes}


def launch_ranks(n, argv, json_out, timeout=None, cmd=None, grace=10.0):
    """Start the N ranks of `bench.py --gpus N` as child processes (torchrun's environment; the
    parent makes no HIP call: torch.cuda.device_count() does not initialise HIP on this image).
    Returns the exit code; rank 0's stdout (the JSON line) is written only if every rank succeeded.
    `timeout` (seconds, --launch-timeout) bounds the whole run: past it the ranks still running
    are terminated, killed after `grace` seconds, and the run fails (a rank stuck in rendezvous
    or communicator set-up, before the fit's RCCL watchdog applies, cannot hang the parent).
    `cmd` replaces the child command (tests)."""
    import socket
    import subprocess
    visible = torch.cuda.device_count()
    if visible < n:
        log(f"bench: --gpus {n} needs {n} visible GPUs, found {visible}; no measurement")
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen((cmd or [sys.executable, os.path.abspath(__file__)]) + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    rc = 0
    pending = set(range(n))
    t_end = None if timeout is None else time.monotonic() + timeout
    killed_at = None
    while pending:
        for r in sorted(pending):
            code = procs[r].poll()
            if code is None:
                continue
            pending.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                log(f"bench: rank {r} exited with {code}; stopping the other ranks")
                for q in pending:
                    procs[q].terminate()
                killed_at = time.monotonic()
        now = time.monotonic()
        if pending and t_end is not None and now > t_end and killed_at is None:
            log(f"bench: the {n}-rank run exceeded --launch-timeout {timeout:.0f} s; terminating ranks "
                f"{sorted(pending)}")
            rc = rc or 124
            for q in pending:
                procs[q].terminate()
            killed_at = now
        if pending and killed_at is not None and now > killed_at + grace:
            for q in pending:
                procs[q].kill()
        time.sleep(0.05)
    out = procs[0].stdout.read().decode()
    if rc == 0:
        json_out.write(out)
        json_out.flush()
    return rc


def rank_summary(world, rows, el_s, dom_ms, steps, comm_ranks, allreduce_samples, arena_bytes, scaling):
    """The N > 1 block of the JSON line from every rank's numbers (index = rank): what the driver's
    scaling run must show, from the run itself — the communicator's own rank count (ncclCommCount),
    the sampled all-reduce time per step, the spread of the dominant kernel over the ranks, and
    each rank's own rate.  allreduce_samples: [(ms, bytes)] sampled on rank 0."""
    ar_us = [1e3 * ms for ms, _ in allreduce_samples]
    return {
        "world_size": world,
        "scaling": scaling,
        "rccl_ranks": comm_ranks,
        "rows_per_rank": [int(r) for r in rows],
        "allreduce_us_per_step": float(np.median(ar_us)) if ar_us else None,
        "allreduce_us_range": [float(min(ar_us)), float(max(ar_us))] if ar_us else None,
        "allreduce_samples": len(ar_us),
        "allreduce_bytes": int(allreduce_samples[0][1]) if allreduce_samples else arena_bytes,
        "dominant_kernel_ms_min": float(min(dom_ms)),
        "dominant_kernel_ms_max": float(max(dom_ms)),
        "dominant_kernel_ms_per_rank": [float(v) for v in dom_ms],
        "per_rank_ms_per_step": [1e3 * float(e) / steps for e in el_s],
        "per_rank_samples_per_s": [float(r) * steps / float(e) for r, e in zip(rows, el_s)],
    }


def main():
    # exactly ONE line on stdout: route everything else (RCCL's banner, library prints) to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the run: under a launcher WORLD_SIZE must match; without one, N > 1 "
                         "starts the N ranks as child processes (default: WORLD_SIZE or 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed fit_Adam iterations first: the compute-bound kernels (c3, c5) reach their "
                         "steady clock only after ~50 iterations (c3 kernel 0.402 ms after 5, 0.367 ms after 200)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--allow-other-path", action="store_true",
                    help="measure even when the plan did not take the config's expected kernel path")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=None, help="CPU baseline threads (default: affinity size)")
    ap.add_argument("--time-all-kernels", action="store_true",
                    help="hipEvent-time every kernel kind (adds per-launch event overhead)")
    ap.add_argument("--timing-every", type=int, default=1,
                    help="bracket only every n-th launch of the timed kernels with HIP events (default: every launch)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no hipEvents in the timed region (ms_per_step without event packets; no roofline)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak (default): every rank holds the config's per-GPU sample count; strong: the config's "
                         "total sample count (c4: 131072) split over the ranks")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launched N > 1 runs: seconds before the remaining ranks are terminated (exit non-zero)")
    ap.add_argument("--allreduce-sample-every", type=int, default=5,
                    help="N > 1: time every n-th gradient all-reduce of the timed fit with HIP events")
    ap.add_argument("--traffic", default=os.path.join(HERE, "profiles", "traffic.json"),
                    help="PMC traffic summary (tools/pmc_traffic.py output) for the roofline 'traffic' field")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world) if env_world else 1
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], json_out, timeout=args.launch_timeout))
    if env_world is not None and int(env_world) != args.gpus:
        log(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks; no measurement")
        sys.exit(2)
    cfg = CONFIGS[args.config]
    if args.warmup is None:  # 200 (< 0.5 s) resident; the PCIe-bound streamed config: 3 (0.5 s)
        args.warmup = cfg.get("default_warmup", 200)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank_id = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1 or os.environ.get("TR_BENCH_FORCE_PG") == "1":  # force: exercise RCCL at world 1
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        pg = dist.group.WORLD
    dev = f"cuda:{local}"
    torch.cuda.set_device(local)

    from tensor_regression_amd import CP_linear_regression, CP_logistic_regression

    if args.scaling == "strong":
        if cfg.get("windowed") or cfg.get("hoststream"):
            ap.error(f"--scaling strong is not defined for {args.config}")
        row0, rows = shard_rows(cfg["total_rows"], world, rank_id)
    else:
        rows = cfg["rows"]
        row0 = rank_id * rows
    X, y = make_data(cfg, rows, row0, dev)
    torch.cuda.synchronize()
    Xres = X  # the device-resident X (hoststream: for the copy / compute-only reference timings)
    if cfg.get("hoststream"):
        from tensor_regression_amd.util import HostStream
        X = HostStream(X.cpu(), chunk_rows=cfg["chunk_rows"], device=dev)
    R = cfg["rank"]
    torch.manual_seed(1)
    if cfg["kind"] == "spectral":
        from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression as SpectralCP
        model = SpectralCP(X.shape, y.shape, rank_normal=R, rank_spectral=cfg["rank_spectral"],
                           n_complex_dim=cfg["n_complex_dim"], device=dev)
        init = ([a.detach().cpu().numpy().copy() for a in model.Bcp_n],
                [a.detach().cpu().numpy().copy() for a in model.Bcp_c])

        def fit(iters):
            return model.fit_Adam(X, y, lambda_L2=0.01, max_iter=iters, tol=0, patience=10,
                                  Adam_kwargs={"lr": 0.01}, process_group=pg)
    elif cfg["kind"] == "linear":
        model = CP_linear_regression(X.shape, rank=R, device=dev)
        init = ([a.detach().cpu().numpy().copy() for a in model.Bcp], model.bias.detach().cpu().numpy().copy())

        def fit(iters):
            return model.fit_Adam(X, y, lambda_L2=0.01, max_iter=iters, tol=0, patience=10,
                                  Adam_kwargs={"lr": 0.01}, process_group=pg)
    else:
        model = CP_logistic_regression(X, y, rank=R, device=dev)
        init = ([a.detach().cpu().numpy().copy() for a in model.Bcp], None)
        cw = np.ones(cfg["classes"], np.float32)

        def fit(iters):
            return model.fit_Adam(lambda_L2=0.01, max_iter=iters, tol=0, patience=10, weights=cw,
                                  Adam_kwargs={"lr": 0.01}, process_group=pg)

    _ph = _Phases()
    if _ph.on:  # where the warm-up (first) fit call spends its host time
        import cProfile
        import pstats
        prof = cProfile.Profile()
        prof.enable()
        fit(args.warmup)
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(35)
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(15)
    else:
        fit(args.warmup)
    _ph("warm-up fit")
    plan = model._plan
    # the kernel strategy this config is benchmarked on: a silent fallback (e.g. a spilling
    # single-pass variant dropping the plan to two passes) must not pass as this config's number
    want = cfg.get("expect")
    if want and (f"path={want}" not in plan.describe or "recovered=" in plan.describe) and not args.allow_other_path:
        raise SystemExit(f"bench {args.config}: plan took an unexpected path ({plan.describe}); expected "
                         f"path={want} (--allow-other-path to measure it anyway)")
    _ph("plan path check")
    plan.read_timing()
    _ph("read_timing")
    # time only the X-streaming kernels by default (timing-only events, no system-scope fence:
    # with the default fence each record idled the GPU ~6 us on its side of the launch in a
    # rocprofv3 kernel trace; --timing-every n brackets only every n-th launch)
    if not args.no_kernel_timing:
        plan.set_timing(True, kinds=None if args.time_all_kernels else ["stream_fused", "stream_rows", "stream_cols"],
                        every=max(1, args.timing_every))

    comm = None
    if pg is not None:  # (world 1 too with TR_BENCH_FORCE_PG=1: the RCCL path on one GPU)
        from tensor_regression_amd import _engine
        comm = _engine.gradient_allreduce(pg, local)
        if isinstance(comm, _engine.RcclAllReduce):
            comm.set_timing(args.allreduce_sample_every)
        else:
            comm = None

    def barrier():
        # every rank past this point once all have reached it: on RCCL a one-element ncclAllReduce
        # on the compute stream + device sync (RcclAllReduce.barrier; dist.barrier() through
        # ProcessGroupNCCL cost ~55 us per call at world 1, tools/pg_account.py)
        if comm is not None:
            comm.barrier()
        elif pg is not None:
            torch.distributed.barrier()

    _ph("set_timing")
    barrier()
    torch.cuda.synchronize()
    _ph("barrier + sync")
    t0 = time.perf_counter()
    fit(args.steps)
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    plan.set_timing(False)
    kt = plan.read_timing()
    ar_samples = []
    if comm is not None:
        ar_samples = comm.read_timing()
        comm.set_timing(0)
    el_local = el
    N = X.shape[0]
    P = int(np.prod(cfg["dims"]))

    if args.no_kernel_timing:
        tot = float(N)
        if pg is not None:
            t = torch.tensor([el, float(N)], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t[:1], op=torch.distributed.ReduceOp.MAX)
            torch.distributed.all_reduce(t[1:], op=torch.distributed.ReduceOp.SUM)
            el, tot = float(t[0]), float(t[1])
        if rank_id == 0:
            json_out.write(json.dumps({"metric": METRIC, "value": tot * args.steps / el, "unit": "samples/s",
                                       "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                                       "ms_per_step": 1e3 * el / args.steps, "scaling": args.scaling,
                                       "config": {"workload": cfg["workload"], "plan": plan.describe},
                                       "roofline": None, "note": "--no-kernel-timing"}) + "\n")
            json_out.flush()
        if pg is not None:
            torch.distributed.destroy_process_group()
        return
    stream_kinds = ["stream_fused"] if kt["stream_fused"][1] else ["stream_rows", "stream_cols"]
    kernel_avg = {k: (v[0] / v[1] if v[1] else None) for k, v in kt.items()}
    flops_launch = None
    if cfg["kind"] == "spectral":
        dom = "stream_fused"
        bytes_launch = N * P * 4 + N * 4 * cfg["n_out"]
        # algorithmic minimum: the lin term as a dense (W x D x n_out) contraction
        # forward + backward, the spectral term's two GEMMs over Rs*Cc columns (Cc = n_complex_dim + 1):
        # 4*N*P*(n_out + Rs*Cc)
        flops_launch = 4 * N * P * (cfg["n_out"] + cfg["rank_spectral"] * (cfg["n_complex_dim"] + 1))
        dom_name = "k_spec_slice" if "slice-1pass" in plan.describe else "k_spec_fused"
    elif kt["stream_fused"][1] and "mnl-fused-1pass" in plan.describe:
        dom = "stream_fused"
        bytes_launch = N * P * 4 + N * 8  # X row + int64 label per sample
        dom_name = "k_mnl_duo" if " duo " in plan.describe else "k_mnl_fused"
    elif kt["stream_fused"][1]:
        dom = "stream_fused"
        bytes_launch = N * P * 4 + N * 4
        if cfg.get("hoststream"):  # one launch per chunk
            bytes_launch = bytes_launch // (kt["stream_fused"][1] // args.steps)
        if cfg.get("windowed"):
            # overlapping windows: the unique series (N + L - 1) x F is what must cross HBM; the
            # N * P window bytes are logical reads, mostly served by L2 / MALL
            L, F = cfg["dims"][0], int(np.prod(cfg["dims"][1:]))
            bytes_launch = (N + L - 1) * F * 4 + N * 4
        dom_name = "k_linear_cluster" if "cluster-1pass" in plan.describe else "k_linear_fused"
    else:
        dom = "stream_rows" if kt["stream_rows"][0] >= kt["stream_cols"][0] else "stream_cols"
        bytes_launch = N * P * 4 + N * 4 * (cfg.get("classes", 1))
        dom_name = "k_rows" if dom == "stream_rows" else "k_cols"
        if dom == "stream_rows" and "+mfma-fwd" in plan.describe:
            dom_name = "k_rows_mfma"
    dom_ms = kernel_avg[dom]
    ranks_block = None
    rows_all = [N]
    if pg is not None:
        # every rank's wall time, dominant-kernel average and rows (value uses the max wall time)
        t = torch.tensor([el_local, dom_ms, float(N)], dtype=torch.float64, device=dev)
        parts = [torch.zeros_like(t) for _ in range(world)]
        torch.distributed.all_gather(parts, t)
        el_all = [float(p[0]) for p in parts]
        dom_all = [float(p[1]) for p in parts]
        rows_all = [int(p[2]) for p in parts]
        el = max(el_all)
        if world > 1 or comm is not None:
            ranks_block = rank_summary(world, rows_all, el_all, dom_all, args.steps,
                                       comm.count() if comm is not None else None, ar_samples,
                                       plan.num_grads * 4, args.scaling)
            if comm is None:
                ranks_block["note"] = "torch.distributed all_reduce path (TR_RCCL_DIRECT=0): no RCCL count / timing"
    ms_step = 1e3 * el / args.steps
    value = sum(rows_all) * args.steps / el
    hoststream = host_stream_report(model, X, Xres, y, fit, ms_step, dev) if cfg.get("hoststream") else None
    achieved = bytes_launch / (dom_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    if os.path.exists(args.traffic):
        try:
            with open(args.traffic) as f:
                tj = json.load(f)
            # the counter passes were taken at the config's per-GPU size; another row count (strong
            # scaling) has no entry: traffic stays null rather than another size's bytes
            key = args.config if N == cfg["rows"] else f"{args.config}@{N}"
            ent = tj.get(key, {}).get(dom_name)
            if ent:
                traffic = ent.get("hbm_bytes_per_launch")
                traffic_src = (f"read from {os.path.relpath(args.traffic, HERE)} (rocprofv3 FETCH_SIZE/WRITE_SIZE "
                               f"passes of this kernel, {tj.get('round', 'earlier run')}), not measured in this run")
        except Exception:
            traffic = None
    iter_bytes = sum(N * P * 4 for _ in stream_kinds)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded torch.randn X on device, planted CP model + noise)",
        "config": {"workload": cfg["workload"], "samples_per_gpu": N, "feature_dims": list(cfg["dims"]),
                   "rank": R, "global_batch": sum(rows_all),
                   "parallelism": f"dp{world} sample-sharded, one RCCL all-reduce of the gradient arena per step",
                   "plan": plan.describe},
        "achieved_hbm_GBps_per_gpu": iter_bytes / (ms_step * 1e-3) / 1e9,
        "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel_avg_ms": dom_ms, "algorithmic_bytes_per_launch": bytes_launch},
        "kernel_avg_ms": kernel_avg,
    }
    # the launches the kernel average is over (every --timing-every-th launch of the timed region)
    out["roofline"].update({"timed_launches": int(kt[dom][1]), "timing_every": max(1, args.timing_every)})
    if hoststream is not None:
        out["hoststream"] = hoststream
        out["data"] += "; X resident in pinned host memory, copied to HBM every step (inside the timed region)"
    if flops_launch is not None:
        # spectral: the roofline time is the larger of the HBM time of the algorithmic bytes and
        # the fp32 matrix time of the algorithmic flops; at config 5 (18 flop/B < the 19.7 flop/B
        # ridge) that is HBM, so achieved / peak are GB/s and the flop rate is reported beside it
        tflops = flops_launch / (dom_ms * 1e-3) / 1e12
        t_hbm = bytes_launch / (HBM_PEAK_GBPS * 1e9)
        t_mfma = flops_launch / (FP32_MFMA_PEAK_TFLOPS * 1e12)
        if t_hbm >= t_mfma:
            out["roofline"].update({"tflops": tflops, "tflops_frac": tflops / FP32_MFMA_PEAK_TFLOPS,
                                    "algorithmic_flops_per_launch": flops_launch,
                                    "roofline_ms": 1e3 * t_hbm})
        else:
            out["roofline"] = {"bound": "mfma", "kernel": dom_name, "achieved": tflops, "peak": FP32_MFMA_PEAK_TFLOPS,
                               "unit": "TFLOP/s", "frac": tflops / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic,
                               "traffic_source": traffic_src,
                               "kernel_avg_ms": dom_ms, "algorithmic_flops_per_launch": flops_launch,
                               "algorithmic_bytes_per_launch": bytes_launch, "hbm_GBps": achieved,
                               "hbm_frac": achieved / HBM_PEAK_GBPS, "roofline_ms": 1e3 * t_mfma}
        out["dtype"] = "fp32"
        if "bf16split" in plan.describe:
            # fp32 operands and accumulation; the GEMMs run on the bf16 matrix cores through split
            # operands (DESIGN.md "bf16 split GEMMs"): factors / dT in three round-to-nearest pieces
            # (exact), the sample data in two (|x - x1 - x2| < 2^-16 |x|) or three
            xp = "three" if "xpieces=3" in plan.describe else "two"
            out["roofline"]["gemm_form"] = (f"bf16 split GEMMs: factor-side operands in three RNE bf16 pieces, X in "
                                            f"{xp}, fp32 accumulate")
            # the arithmetic is not plain fp32 GEMMs: say so in the field consumers read
            out["dtype"] = f"fp32 (GEMMs on bf16 pieces: X in {xp}, factors in three; fp32 accumulate)"
    if ranks_block is not None:
        out["ranks"] = ranks_block
    if rank_id == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        out["cpu_baseline"] = cpu_baseline(cfg, Xres, y, init, args.cpu_budget, args.cpu_threads)
    else:
        out["cpu_baseline"] = None
    if rank_id == 0:
        json_out.write(json.dumps(out) + "\n")
        json_out.flush()
    if pg is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
