#!/usr/bin/env python3
"""Distribution of the split body's gradient error on "mixed"-scale X (every sample at 10^U(-2, 2))
against fp64 and the reference's fp32 op sequence (GPU box; test_multinomial_split_body_x_scale's
setup with explicit seeds).  python tools/mnl_mixed_scan.py I J R C nseeds"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cp_oracle  # noqa: E402  (test infrastructure: the checker)
from tensor_regression_amd import CP_logistic_regression  # noqa: E402


def nrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


I, J, R, C, ns = (int(v) for v in sys.argv[1:6])
N = int(sys.argv[6]) if len(sys.argv) > 6 else 90
for seed in range(ns):
    g = torch.Generator().manual_seed(1000 + seed)
    X = torch.randn(N, I, J, generator=g)
    X *= (10.0 ** (4 * torch.rand(N, generator=g) - 2)).reshape(-1, 1, 1)
    y = torch.randint(0, C, (N,), generator=g)
    y[:C] = torch.arange(C)
    sc = 0.3 * min(1.0, (2048.0 / (I * J)) ** 0.5)
    B = [torch.randn(I, R, generator=g) * sc, torch.randn(J, R, generator=g) * sc, torch.randn(C, R, generator=g) * sc]
    cw = (torch.rand(C, generator=g) + 0.5).numpy()
    nn = [False] * 3
    r32 = cp_oracle.mnl_loss_grad(X, y, B, np.ones(R), nn, cw, 0.0)
    r64 = cp_oracle.closed_form_mnl(X.double().numpy(), y.numpy(), [b.double().numpy() for b in B], np.ones(R), nn,
                                    cw, 0.0)
    mm = CP_logistic_regression(X.numpy(), y.numpy(), rank=R, non_negative=nn, device="cuda:0",
                                Bcp_init=[b.cuda() for b in B])
    dev, Xd, yd = mm._device_data()
    plan = mm._get_plan(Xd, N)
    cwd, W = mm._class_weights(cw, dev, yd)
    arena = plan.pack(mm.Bcp)
    grad = torch.zeros(plan.num_grads, device="cuda:0")
    gtot = torch.zeros(plan.num_params, device="cuda:0")
    loss = torch.zeros(1, device="cuda:0")
    plan.loss_grad(Xd, yd, cwd, W, arena, mm.weights, grad)
    plan.finalize_grad(arena, grad, 0.0, gtot, loss)
    ours = [t.cpu().numpy() for t in plan.factor_views(gtot)]
    row = []
    for f in range(3):
        row.append((nrel(ours[f], r64["grads"][f]), nrel(r32["grads"][f], r64["grads"][f])))
    form = "exact" if "xform=exact" in plan.describe else "fast"
    print(f"seed {seed} {form} " + "  ".join(f"g{f}: ours {a:.2e} ref32 {b:.2e}" for f, (a, b) in enumerate(row)),
          flush=True)
