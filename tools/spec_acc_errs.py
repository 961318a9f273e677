#!/usr/bin/env python3
"""Config-5 full-size gradient errors against the fp64 closed form for the library TR_HIP_LIB
names (GPU box): the split forms of k_spec_slice (X in two / three bf16 pieces) on |X| and on
signed X, one JSON line per (X sign, form).  Uses tests/test_gpu_fullsize.py's helpers.

    TR_HIP_LIB=... python tools/spec_acc_errs.py [forms=split,x3]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_fullsize as F  # noqa: E402

forms = (sys.argv[1] if len(sys.argv) > 1 else "split,x3").split(",")
DEV = "cuda:0"
for signed in (False, True):
    from tensor_regression_amd import spectral_tensor_regression as SP
    N, W, D, O = 32768, 256, 129, 2
    gen = torch.Generator(device=DEV).manual_seed(1234 + int(signed))
    X = torch.randn((N, W, D), device=DEV, generator=gen)
    if not signed:
        X.abs_()
    y = torch.randn((N, O), device=DEV, generator=gen)
    torch.manual_seed(1)
    m0 = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    ref64 = F._spectral_fp64(X, y, m0.Bcp_n, m0.Bcp_c, m0.bias, 0.01)
    for form in forms:
        d, e = F._spectral_errs(X, y, form, ref64)
        worst = max(e[f"grad{f}"] for f in range(6))
        print(json.dumps({"lib": os.path.basename(os.environ.get("TR_HIP_LIB", "libtr_hip.so")), "signed": signed,
                          "form": form, "worst_grad": worst, "errs": e, "describe": d}), flush=True)
    # the default form's pass time on this X (loss_grad: the slice kernel + its reduction), 30 calls
    torch.manual_seed(1)
    m1 = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    plan = m1._get_plan(X, N)
    arena = plan.pack(m1.Bcp_n, m1.Bcp_c, m1.bias)
    w = torch.ones(16, device=DEV)
    grad = torch.zeros(plan.num_grads, device=DEV)
    for _ in range(20):
        plan.loss_grad(X, y, None, float(N * O), arena, w, grad)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        plan.loss_grad(X, y, None, float(N * O), arena, w, grad)
    e1.record()
    e1.synchronize()
    print(json.dumps({"signed": signed, "loss_grad_ms": e0.elapsed_time(e1) / 30, "describe": plan.describe}),
          flush=True)
    del X, y
    torch.cuda.empty_cache()
