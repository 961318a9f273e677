#!/usr/bin/env python3
"""Per-phase cycle breakdown of the two-workgroups-per-CU multinomial kernel (profiling build).

    make -C tensor_regression_amd/csrc duo-variant V=prof VFLAGS=-DTR_DUO_PROFILE=1
    TR_HIP_LIB=$PWD/tensor_regression_amd/libtr_hip_duo_prof.so python tools/duo_profile.py

Phases per wave (__builtin_readcyclecounter deltas of the last launch, averaged over workgroups,
per sample): LDS-DMA wait, barrier, GEMM steps with the interleaved epilogue, tail (U chain /
accumulator hand-over).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensor_regression_amd import _lib  # noqa: E402
from tensor_regression_amd import CP_logistic_regression  # noqa: E402

# I, J, R from the environment too (the split body's shapes; NW = 8 waves at most, row blocks)
I, J, R = int(os.environ.get("I", 128)), int(os.environ.get("J", 64)), int(os.environ.get("R", 8))
N, C = int(os.environ.get("N", 65536 * 8192 // (I * J))), 10
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(N, I, J, device=dev, generator=g)
y = torch.randint(0, C, (N,), device=dev, generator=g)
y[:C] = torch.arange(C, device=dev)
torch.manual_seed(1)
m = CP_logistic_regression(X, y, rank=R, device=dev)
m.fit_Adam(lambda_L2=0.01, max_iter=3, tol=0, patience=10, weights=np.ones(C), Adam_kwargs={"lr": 0.01})
torch.cuda.synchronize()
print(m._plan.describe)
lib = _lib.load()
fn = lib.tr_duo_profile_read
fn.restype = ctypes.c_int
buf = (ctypes.c_ulonglong * (512 * 8 * 4))()
assert fn(buf) == 0
a = np.array(buf[:], dtype=np.float64).reshape(512, 8, 4)
d = m._plan.describe
nw = int(d.split("waves=")[1].split()[0])
wpc = int(d.split("wg/cu=")[1].split()[0])
nb = int(d.split("rowblocks=")[1].split()[0]) if "rowblocks=" in d else 1
per_wg = (N + 256 * wpc - 1) // (256 * wpc) * nb  # sample blocks per workgroup (one per sample without row blocks)
a = a[: min(512, 256 * wpc)]
names = ["DMA wait", "barrier", "GEMM+epi", "tail"]
print(f"cycles/{'block' if nb > 1 else 'sample'}   " + " ".join(f"{n:>10s}" for n in names) + "      total")
for w in range(nw):
    v = a[:, w, :].mean(axis=0) / per_wg
    print(f"wave {w}          " + " ".join(f"{x:10.0f}" for x in v) + f" {v.sum():10.0f}")
