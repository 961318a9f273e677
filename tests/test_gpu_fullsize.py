"""Parity at BASELINE.json's full sizes (configs 2-5), one GPU.

The CPU oracle cannot run these sizes in seconds, so the gfx950 path is checked against
properties that hold at any size:
  * configs 2-4: one loss + gradient evaluation against a float64 closed form of the same
    math computed with torch on the same GPU, chunked over
    samples (X is 8.6 GB at config 2).  fp32 kernel vs fp64 truth: the data loss agrees to
    LOSS_TOL and every factor gradient to GRAD_TOL normwise — tolerances set from the measured
    error with a margin (the fp32 reference itself sits ~1e-6..1e-5 from fp64 at these sizes,
    SURVEY.md §8(c));
  * config 5 (spectral): the same fp64 comparison on the product kernel (k_spec_slice's bf16
    split GEMMs) and on its f32-MFMA form, both held to twice the error of the reference's own
    op sequence run in fp32 on the host CPU; and properties: the full-size gradient equals the sum of the two half-shard gradients
    (linearity over samples), calls of equal traversal parity are bitwise identical, and the
    first loss fit_Adam logs is the loss of one loss_grad + finalize_grad at the same factors.
Inputs are generated on the device from fixed seeds (same recipe as bench.py).
"""
import os

import numpy as np
import pytest
import torch

from golden_util import normwise_rel

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
LOSS_TOL = 1e-6   # measured (r01, MI355X): <= 4e-8 on c2 / c3 / c4
GRAD_TOL = 2e-6   # measured: <= 3.2e-7 normwise on every factor gradient
CHUNK = 4096


def _l2(As, lam):
    """L2_penalty term and its gradient (standard_tensor_regression.py:180-196), fp64."""
    tot = sum(torch.linalg.norm(A) for A in As)
    return lam * tot, [lam * A / torch.linalg.norm(A) for A in As]


def _linear_fp64(X, y, As, bias, lam):
    N = X.shape[0]
    P = int(np.prod(X.shape[1:]))
    A64 = [A.detach().double() for A in As]
    if len(A64) == 2:
        B = torch.einsum('ir,jr->ij', A64[0], A64[1])
    else:
        B = torch.einsum('ir,jr,kr->ijk', A64[0], A64[1], A64[2])
    b = B.reshape(P)
    G = torch.zeros(P, dtype=torch.float64, device=DEV)
    sse = torch.zeros((), dtype=torch.float64, device=DEV)
    rsum = torch.zeros((), dtype=torch.float64, device=DEV)
    for a in range(0, N, CHUNK):
        Xc = X[a:a + CHUNK].reshape(-1, P).double()
        e = Xc @ b + float(bias) - y[a:a + CHUNK].double()
        sse += (e * e).sum()
        r = 2.0 * e / N
        G += Xc.T @ r
        rsum += r.sum()
        del Xc
    G = G.reshape(B.shape)
    if len(A64) == 2:
        grads = [G @ A64[1], G.T @ A64[0]]
    else:
        grads = [torch.einsum('ijk,jr,kr->ir', G, A64[1], A64[2]),
                 torch.einsum('ijk,ir,kr->jr', G, A64[0], A64[2]),
                 torch.einsum('ijk,ir,jr->kr', G, A64[0], A64[1])]
    pen, pg = _l2(A64, lam)
    data = sse / N
    return float(data), float(data + pen), [g + q for g, q in zip(grads, pg)], float(rsum)


def _linear_case(shape, rank, seed):
    from tensor_regression_amd import CP_linear_regression
    gen = torch.Generator(device=DEV).manual_seed(seed)
    X = torch.randn(shape, device=DEV, generator=gen)
    gc = torch.Generator().manual_seed(99)
    Astar = [(torch.randn(d, rank, generator=gc) / 4).to(DEV) for d in shape[1:]]
    P = int(np.prod(shape[1:]))
    if len(shape) == 3:
        Bs = torch.einsum('ir,jr->ij', *Astar)
    else:
        Bs = torch.einsum('ir,jr,kr->ijk', *Astar)
    y = X.reshape(shape[0], P) @ Bs.reshape(P) + 0.1 * torch.randn(shape[0], device=DEV, generator=gen)
    torch.manual_seed(1)
    model = CP_linear_regression(X.shape, rank=rank, device=DEV)
    plan = model._get_plan(X, shape[0])
    arena = plan.pack(model.Bcp, model.bias)
    grad = torch.zeros(plan.num_grads, device=DEV)
    gtot = torch.zeros(plan.num_params, device=DEV)
    loss = torch.zeros(1, device=DEV)
    lam = 0.01
    plan.loss_grad(X, y, None, float(shape[0]), arena, model.weights, grad)
    plan.finalize_grad(arena, grad, lam, gtot, loss)
    data, total, grads, dbias = _linear_fp64(X, y, model.Bcp, model.bias.item(), lam)
    errs = {"data_loss": abs(grad[plan.num_params].item() - data) / abs(data), "loss": abs(loss.item() - total) / abs(total),
            "bias": abs(gtot[plan.offsets[-1]].item() - dbias) / max(abs(dbias), 1e-30)}
    for f, (v, ref) in enumerate(zip(plan.factor_views(gtot), grads)):
        errs[f"grad{f}"] = normwise_rel(v.cpu().numpy(), ref.cpu().numpy())
    return plan.describe, errs


@pytest.mark.parametrize("cfg", ["c2", "c4", "c4full"])
def test_linear_full_size_vs_fp64(cfg):
    """c2; c4 as one GPU's shard of the 8-GPU config (16384 samples); c4full: BASELINE configs[3]
    whole on one GPU (X (131072, 64, 64, 32), 68.7 GB: the N = 1 point of bench.py --scaling
    strong), k_linear_cluster over 8x the rows per cluster of the shard case."""
    shape, rank = {"c2": ((65536, 256, 128), 8), "c4": ((16384, 64, 64, 32), 16),
                   "c4full": ((131072, 64, 64, 32), 16)}[cfg]
    desc, errs = _linear_case(shape, rank, 1234)
    print(cfg, desc, errs)
    assert ("fused-1pass" if cfg == "c2" else "cluster-1pass") in desc
    assert "recovered=" not in desc, desc
    assert errs["data_loss"] <= LOSS_TOL and errs["loss"] <= LOSS_TOL, errs
    for k in ("grad0", "grad1", "grad2"):
        if k in errs:
            assert errs[k] <= GRAD_TOL, errs
    assert errs["bias"] <= 1e-5, errs  # a sum of signed residuals (measured <= 1e-6)


@pytest.mark.parametrize("form", ["bf16split", "rankblock", "fused", "wide64", "wide256", "wide128x128", "wide512",
                                  "wide256x128", "rank16", "wide128x32", "wide256x32"])
def test_multinomial_full_size_vs_fp64(form, monkeypatch):
    """Config 3: X (65536, 128, 64), 10 classes, rank 8 (the factored single pass: two 4-wave
    workgroups per CU in the f32 rank-block form (default) and the bf16-split form
    (TR_DUO_SPLIT=1); with TR_MNL_DUO=0 one 8-wave workgroup per CU).  wide64 / wide256 /
    wide128x128: the split body on (64, 64) samples (2 waves, 4 workgroups per CU), on (256, 64)
    samples (8 waves, one workgroup per CU, a shape k_mnl_fused does not fit) and on (128, 128)
    samples (8 waves of 16 rows) at the same sample bytes per GPU; wide512 / wide256x128: samples of
    128 KiB, (512, 64) and (256, 128), streamed through the split body in two row blocks of (256, 64) /
    (128, 128) (round 6; the two-pass kernels before); wide128x32 / wide256x32: the split body's 32-wide
    form (4 and 8 waves, one-wave epilogue; round 6).  Bars: GRAD_TOL normwise, and no further from fp64 than the reference's own op sequence
    in fp32 on the host CPU (the oracle, same factors) is, x2 + 1e-7.  Measured (r05, worst
    gradient): rank-block 3.1e-7, split 7.2e-7, wide64 3.0e-7, wide256 1.47e-6, wide128x128
    1.53e-6; the reference in fp32 4.0e-6 (c3), 3.2e-6 (wide64), 9.8e-6 (wide256), 1.03e-5
    (wide128x128)."""
    from tensor_regression_amd import CP_logistic_regression
    duo = form != "fused"
    monkeypatch.delenv("TR_DUO_SPLIT", raising=False)
    monkeypatch.delenv("TR_MNL_DUO", raising=False)
    if not duo:
        monkeypatch.setenv("TR_MNL_DUO", "0")
    if form == "bf16split":
        monkeypatch.setenv("TR_DUO_SPLIT", "1")
    N, I, J, C, R = 65536, 128, 64, 10, 8
    if form == "rank16":  # config 3's samples at rank 16: the split body's 16-rank form (round 6)
        R = 16
    if form.startswith("wide"):
        I, J = (int(form[4:]), 64) if "x" not in form else (int(v) for v in form[4:].split("x"))
        N = 65536 * 128 * 64 // (I * J)
    gen = torch.Generator(device=DEV).manual_seed(1234)
    X = torch.randn((N, I, J), device=DEV, generator=gen)
    gc = torch.Generator().manual_seed(99)
    Astar = [(torch.randn(I, R, generator=gc) / 3).to(DEV), (torch.randn(J, R, generator=gc) / 3).to(DEV),
             torch.randn(C, R, generator=gc).to(DEV)]
    Bs = torch.einsum('ir,jr,cr->ijc', *Astar).reshape(I * J, C)
    S = torch.softmax(X.reshape(N, I * J) @ Bs, dim=1)
    y = torch.multinomial(S, 1, generator=gen).reshape(-1)
    y[:C] = torch.arange(C, device=DEV)
    torch.manual_seed(1)
    mm = CP_logistic_regression(X, y, rank=R, device=DEV)
    dev, Xd, yd = mm._device_data()
    plan = mm._get_plan(Xd, N)
    assert "mnl-fused-1pass" in plan.describe
    assert (" duo " in plan.describe) == duo, plan.describe
    if form.startswith("wide"):
        nw = min(8, I // 16 if J == 128 else I // 32)
        nb = I // (16 * nw if J == 128 else 32 * nw)
        assert "form=bf16split" in plan.describe and f"waves={nw} " in plan.describe, plan.describe
        assert (f"rowblocks={nb}" in plan.describe) == (nb > 1), plan.describe
        assert (" jt=32" in plan.describe) == (J == 32), plan.describe
    elif form == "rank16":
        assert "form=bf16split" in plan.describe and " rk=16" in plan.describe, plan.describe
    elif duo:
        assert f"form={form}" in plan.describe, plan.describe
    cw = np.ones(C, np.float32)
    cwd, W = mm._class_weights(cw, dev, yd)
    arena = plan.pack(mm.Bcp)
    lam = 0.01
    grad = torch.zeros(plan.num_grads, device=DEV)
    gtot = torch.zeros(plan.num_params, device=DEV)
    loss = torch.zeros(1, device=DEV)
    plan.loss_grad(Xd, yd, cwd, W, arena, mm.weights, grad)
    plan.finalize_grad(arena, grad, lam, gtot, loss)
    # fp64 closed form (double softmax)
    A64 = [A.detach().double() for A in mm.Bcp]
    B = torch.einsum('ir,jr,cr->ijc', *A64).reshape(I * J, C)
    G = torch.zeros(I * J, C, dtype=torch.float64, device=DEV)
    nll = torch.zeros((), dtype=torch.float64, device=DEV)
    wsum = float(N)
    for a in range(0, N, CHUNK):
        Xc = X[a:a + CHUNK].reshape(-1, I * J).double()
        yc = y[a:a + CHUNK]
        Sx = torch.softmax(Xc @ B, dim=1)
        logQ = torch.log_softmax(Sx, dim=1)
        nll += -logQ.gather(1, yc[:, None]).sum()
        dS = (logQ.exp() - torch.nn.functional.one_hot(yc, C).double()) / wsum
        dZ = Sx * (dS - (dS * Sx).sum(1, keepdim=True))
        G += Xc.T @ dZ
        del Xc
    G3 = G.reshape(I, J, C)
    grads = [torch.einsum('ijc,jr,cr->ir', G3, A64[1], A64[2]), torch.einsum('ijc,ir,cr->jr', G3, A64[0], A64[2]),
             torch.einsum('ijc,ir,jr->cr', G3, A64[0], A64[1])]
    pen, pg = _l2(A64, lam)
    data = float(nll) / wsum
    total = data + float(pen)
    errs = {"data_loss": abs(grad[plan.num_params].item() - data) / abs(data), "loss": abs(loss.item() - total) / abs(total)}
    for f, (v, ref, q) in enumerate(zip(plan.factor_views(gtot), grads, pg)):
        errs[f"grad{f}"] = normwise_rel(v.cpu().numpy(), (ref + q).cpu().numpy())
    # the reference's own op sequence in fp32 on the host CPU (oracle.cp_oracle.mnl_loss_grad:
    # multinomial_tensor_regression.py model 148-187 + CrossEntropyLoss + autograd) at the same factors
    import os
    from oracle import cp_oracle
    quota = os.environ.get("OMP_NUM_THREADS")
    torch.set_num_threads(int(quota) if quota and quota.isdigit() else min(16, os.cpu_count() or 1))
    r = cp_oracle.mnl_loss_grad(X.cpu(), y.cpu(), [A.detach().cpu() for A in mm.Bcp], mm.weights.detach().cpu(),
                                mm.non_negative, cw, lam)
    e_ref = {"data_loss": abs(r["data_loss"] - data) / abs(data), "loss": abs(r["loss"] - total) / abs(total)}
    for f, (v, ref, q) in enumerate(zip(r["grads"], grads, pg)):
        e_ref[f"grad{f}"] = normwise_rel(v, (ref + q).cpu().numpy())
    print("c3", form, plan.describe, errs)
    print("c3", form, "ref32", e_ref)
    assert errs["data_loss"] <= LOSS_TOL and errs["loss"] <= LOSS_TOL, errs
    # the 128 KiB sample forms (P = 32768) are a worse-conditioned problem at this data scale (logits
    # grow with P): the reference's own fp32 sits 2.5e-5 from fp64 there (c3: 4.0e-6), the row-block
    # body 2.6e-6 (first run, r06k) -- absolute bar 4e-6 for those two forms, GRAD_TOL elsewhere
    gtol = 4e-6 if form in ("wide512", "wide256x128") else GRAD_TOL
    for f in range(3):
        assert errs[f"grad{f}"] <= gtol, errs
        # no further from fp64 than the reference's own fp32 computation is (x2, + 1e-7)
        assert errs[f"grad{f}"] <= 2 * e_ref[f"grad{f}"] + 1e-7, (errs, e_ref)


def test_spectral_full_size_properties():
    """Config 5: X (32768, 256, 129), rank_normal = rank_spectral = 8, n_complex_dim 1, y (N, 2)."""
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression
    N, W, D, O = 32768, 256, 129, 2
    gen = torch.Generator(device=DEV).manual_seed(1234)
    X = torch.randn((N, W, D), device=DEV, generator=gen).abs_()
    y = torch.randn((N, O), device=DEV, generator=gen)
    torch.manual_seed(1)
    model = CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    plan = model._get_plan(X, N)
    arena = plan.pack(model.Bcp_n, model.Bcp_c, model.bias)
    w = torch.ones(16, device=DEV)
    outs = []
    for _ in range(3):
        grad = torch.zeros(plan.num_grads, device=DEV)
        plan.loss_grad(X, y, None, float(N * O), arena, w, grad)
        outs.append(grad.clone())
    assert torch.equal(outs[0], outs[2])
    assert normwise_rel(outs[1].cpu().numpy(), outs[0].cpu().numpy()) <= 1e-6
    h = N // 2
    g1 = torch.zeros(plan.num_grads, device=DEV)
    g2 = torch.zeros(plan.num_grads, device=DEV)
    plan.loss_grad(X[:h], y[:h], None, float(N * O), arena, w, g1)
    plan.loss_grad(X[h:], y[h:], None, float(N * O), arena, w, g2)
    err = normwise_rel((g1 + g2).cpu().numpy(), outs[0].cpu().numpy())
    print("c5 shard-sum", plan.describe, err)
    assert err <= 1e-6
    gtot = torch.zeros(plan.num_params, device=DEV)
    loss = torch.zeros(1, device=DEV)
    plan.finalize_grad(arena, outs[0], 0.01, gtot, loss)
    model.fit_Adam(X, y, lambda_L2=0.01, max_iter=3, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
    lr = model.loss_running
    assert len(lr) == 3 and all(np.isfinite(lr)), lr
    assert abs(lr[0] - loss.item()) <= 1e-6 * abs(loss.item()), (lr[0], loss.item())


def _spectral_fp64(X, y, Bn, Bc, bias, lam):
    """fp64 closed form of the spectral fit loss and gradients (cp_oracle.closed_form_spectral,
    restated in torch on the device and chunked over samples; spectral_tensor_regression.py
    lin_model :118-165 + stepwise_spectral_model :339-390, loss :716-717; no softplus, unit
    weights, bias added by both terms)."""
    N, W, D = X.shape
    O = y.shape[1]
    A = [a.detach().double()[:, :, 0] for a in Bn]
    C = [c.detach().double() for c in Bc]
    Rn, Rs, Cc = A[0].shape[1], C[0].shape[1], C[0].shape[2]
    b = bias.detach().double()
    Phi0 = torch.cat([A[0], C[0].reshape(W, Rs * Cc)], dim=1)
    C1, C2 = C[1][:, :, 0], C[2][:, :, 0]
    sse = torch.zeros((), dtype=torch.float64, device=DEV)
    gA = [torch.zeros_like(a) for a in A]
    gC = [torch.zeros_like(c) for c in C]
    dPhi0 = torch.zeros_like(Phi0)
    gb = torch.zeros_like(b)
    ch = CHUNK // 2
    for a in range(0, N, ch):
        Xc = X[a:a + ch].double()
        n = Xc.shape[0]
        T = torch.einsum('nwd,wk->ndk', Xc, Phi0)
        Z = torch.einsum('ndr,dr->nr', T[:, :, :Rn], A[1])
        Tc = T[:, :, Rn:].reshape(n, D, Rs, Cc)
        M = torch.sqrt((Tc * Tc).sum(3))
        V = torch.einsum('ndr,dr->nr', M, C1)
        yhat = Z @ A[2].T + b + V @ C2.T + b
        res = yhat - y[a:a + ch].double()
        sse += (res * res).sum()
        r = 2.0 * res / (N * O)
        gb += 2.0 * r.sum(0)
        gA[2] += r.T @ Z
        dZ = r @ A[2]
        gA[1] += torch.einsum('nr,ndr->dr', dZ, T[:, :, :Rn])
        gC[2] += (r.T @ V)[:, :, None]
        dV = r @ C2
        gC[1] += torch.einsum('nr,ndr->dr', dV, M)[:, :, None]
        dM = dV[:, None, :] * C1[None]
        q = torch.where(M > 0, dM / torch.where(M > 0, M, torch.ones_like(M)), torch.zeros_like(M))
        dT = torch.cat([dZ[:, None, :] * A[1][None], (q[..., None] * Tc).reshape(n, D, Rs * Cc)], dim=2)
        dPhi0 += torch.einsum('nwd,ndk->wk', Xc, dT)
        del Xc, T, Tc, dT
    gA[0] = dPhi0[:, :Rn]
    gC[0] = dPhi0[:, Rn:].reshape(W, Rs, Cc)
    grads = [g[:, :, None] for g in gA] + gC
    pen = 0.0
    for i, p in enumerate([a.detach().double() for a in list(Bn) + list(Bc)]):
        nrm = torch.linalg.norm(p)
        pen += float(nrm)
        grads[i] = grads[i] + lam * p / nrm
    data = float(sse) / (N * O)
    return data, data + lam * pen, grads, gb




def _spectral_errs(X, y, form, ref64):
    """Full-size loss + gradient of one slice-kernel form against the fp64 closed form ref64
    (_spectral_fp64's result).  form: 'split' (the default: X in two bf16 pieces), 'x3' (X in
    three, TR_SLICE_XPIECES=3) or 'f32' (the f32-MFMA form, TR_SLICE_SPLIT=0)."""
    import os
    from tensor_regression_amd import spectral_tensor_regression as SP
    N, W, D = X.shape
    O = y.shape[1]
    keys = ("TR_SLICE_SPLIT", "TR_SLICE_XPIECES")
    old = {k: os.environ.pop(k, None) for k in keys}
    if form == "f32":
        os.environ["TR_SLICE_SPLIT"] = "0"
    elif form == "x3":
        os.environ["TR_SLICE_XPIECES"] = "3"
    SP._plan_cache.clear()
    try:
        torch.manual_seed(1)
        model = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1,
                                        device=DEV)
        plan = model._get_plan(X, N)
        arena = plan.pack(model.Bcp_n, model.Bcp_c, model.bias)
        w = torch.ones(16, device=DEV)
        lam = 0.01
        grad = torch.zeros(plan.num_grads, device=DEV)
        gtot = torch.zeros(plan.num_params, device=DEV)
        loss = torch.zeros(1, device=DEV)
        plan.loss_grad(X, y, None, float(N * O), arena, w, grad)
        plan.finalize_grad(arena, grad, lam, gtot, loss)
        data, total, grads, gb = ref64
        errs = {"data_loss": abs(grad[plan.num_params].item() - data) / abs(data),
                "loss": abs(loss.item() - total) / abs(total),
                "bias": normwise_rel(gtot[plan.offsets[6]:].cpu().numpy(), gb.cpu().numpy())}
        for f, (v, ref) in enumerate(zip(plan.factor_views(gtot), grads)):
            errs[f"grad{f}"] = normwise_rel(v.cpu().numpy(), ref.cpu().numpy())
        return plan.describe, errs
    finally:
        for k in keys:
            os.environ.pop(k, None)
            if old[k] is not None:
                os.environ[k] = old[k]
        SP._plan_cache.clear()


def _spectral_ref32_errs(X, y, ref64, lam=0.01):
    """The reference's own op sequence (oracle.cp_oracle.spectral_loss_grad: lin_model through
    cp_to_tensor + inner, stepwise_spectral_model through torch.einsum + norm, MSELoss, autograd;
    spectral_tensor_regression.py:118-165, 339-390, 714-720) in fp32 on the host CPU, at the same
    factors, against the same fp64 closed form: the error an fp32 implementation of the
    reference makes at this size."""
    import os
    from oracle import cp_oracle
    from tensor_regression_amd import spectral_tensor_regression as SP
    N, W, D = X.shape
    torch.manual_seed(1)
    model = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    Bn = [a.detach().cpu() for a in model.Bcp_n]
    Bc = [a.detach().cpu() for a in model.Bcp_c]
    b = model.bias.detach().cpu()
    quota = os.environ.get("OMP_NUM_THREADS")
    torch.set_num_threads(int(quota) if quota and quota.isdigit() else min(16, os.cpu_count() or 1))
    r = cp_oracle.spectral_loss_grad(X.cpu(), y.cpu(), Bn, Bc, b, torch.ones(16), 8, [False] * 3, lam)
    data, total, grads, gb = ref64
    errs = {"data_loss": abs(r["data_loss"] - data) / abs(data), "loss": abs(r["loss"] - total) / abs(total),
            "bias": normwise_rel(r["bias_grad"], gb.cpu().numpy())}
    for f, (v, ref) in enumerate(zip(r["grads_n"] + r["grads_c"], grads)):
        errs[f"grad{f}"] = normwise_rel(v, ref.cpu().numpy())
    return errs


SPEC_GRAD_ABS = 1e-6  # measured (r06, worst gradient): default 9.4e-8 (|X|) / 8.6e-7 (signed: the signed form);
                      # the round-3 truncating split 2.8e-6


@pytest.mark.parametrize("signed", [False, True])
def test_spectral_full_size_vs_fp64(signed):
    """Config 5 at full size (X (32768, 256, 129), rank_normal = rank_spectral = 8, n_complex_dim 1,
    y (N, 2)) against the fp64 closed form, on the product kernel (k_spec_slice, bf16 split
    GEMMs: X in two pieces by default, in three with TR_SLICE_XPIECES=3), on its f32-MFMA form
    (TR_SLICE_SPLIT=0) and on the reference's own op sequence in fp32 on the host CPU (the
    oracle).  Bars on every form: loss within LOSS_TOL; every gradient no further from fp64 than
    the reference's own fp32 computation is (x2, + 1e-7) AND within SPEC_GRAD_ABS normwise — an
    absolute bar the round-3 truncating split (2.8e-6 on dC0, the negative control below) fails —
    on the non-negative X of bench.py and on signed X = N(0, 1) alike.  On signed X (the forward
    T = X Phi0 cancels, and the C0 gradient goes through 1 / ||T||) the plan runs the slice
    kernel's signed form (tr_plan_set_x_range: the forward's X in three pieces and per-sample
    gradient accumulators; 'xform=signed' in describe): round 5's default form was 2.8e-6 there."""
    from tensor_regression_amd import spectral_tensor_regression as SP
    N, W, D, O = 32768, 256, 129, 2
    gen = torch.Generator(device=DEV).manual_seed(1234 + int(signed))
    X = torch.randn((N, W, D), device=DEV, generator=gen)
    if not signed:
        X.abs_()
    y = torch.randn((N, O), device=DEV, generator=gen)
    torch.manual_seed(1)
    m0 = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    ref64 = _spectral_fp64(X, y, m0.Bcp_n, m0.Bcp_c, m0.bias, 0.01)
    runs = {form: _spectral_errs(X, y, form, ref64) for form in ("split", "x3", "f32")}
    e_ref = _spectral_ref32_errs(X, y, ref64)
    for form, (d, e) in runs.items():
        print(f"c5 signed={signed} {form:5s}", d, e)
    print(f"c5 signed={signed} ref32", e_ref)
    assert "slice-1pass-mfma-bf16split" in runs["split"][0] and "slsp=1 xpieces=2" in runs["split"][0], runs["split"][0]
    assert ("xform=signed" in runs["split"][0]) == signed, runs["split"][0]
    assert "slice-1pass-mfma-bf16split" in runs["x3"][0] and "xpieces=3" in runs["x3"][0], runs["x3"][0]
    d_32 = runs["f32"][0]
    assert "slice-1pass-mfma " in d_32 + " " and "bf16split" not in d_32, d_32
    for form, (_, e) in runs.items():
        assert e["data_loss"] <= LOSS_TOL and e["loss"] <= LOSS_TOL, (form, e)
        assert e["bias"] <= 1e-5, (form, e)
        for f in range(6):
            k = f"grad{f}"
            assert e[k] <= 2 * e_ref[k] + 1e-7, (form, k, e, e_ref)
            assert e[k] <= SPEC_GRAD_ABS, (form, k, e)


def _c5_full_size_errs_main():
    """Child-process entry (python tests/test_gpu_fullsize.py c5errs): the full-size config-5
    errors of the split form of whatever library TR_HIP_LIB names, as one JSON line."""
    import json
    from tensor_regression_amd import spectral_tensor_regression as SP
    N, W, D, O = 32768, 256, 129, 2
    gen = torch.Generator(device=DEV).manual_seed(1234)
    X = torch.randn((N, W, D), device=DEV, generator=gen).abs_()
    y = torch.randn((N, O), device=DEV, generator=gen)
    torch.manual_seed(1)
    m0 = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    ref64 = _spectral_fp64(X, y, m0.Bcp_n, m0.Bcp_c, m0.bias, 0.01)
    keep = os.environ.get("TR_SLICE_XPIECES")
    d, e = _spectral_errs(X, y, "x3" if keep == "3" else "split", ref64)
    print(json.dumps({"describe": d, "errs": e}), flush=True)


def test_spectral_full_size_bar_rejects_truncating_split():
    """Negative control for test_spectral_full_size_vs_fp64's absolute bar: the round-3 split
    (every bf16 piece truncated, X in three pieces) built from the same sources
    (csrc/Makefile negctl: libtr_hip_trunc.so, -DTR_SLICE_SPLITMODE=0) and run in a child process
    on the same full-size problem must FAIL SPEC_GRAD_ABS (round 4 measured 2.8e-6 on dC0), while
    its error against the reference's own fp32 stays inside the relative bar that let it pass in
    round 4.  Its pieces are exact, so its product errors alone are tiny
    (tests/test_split_numerics.py::test_split_errors_alone_stay_far_below_the_bar): what fails
    is the bias the bf16 MFMA's accumulation adds to same-signed small pieces
    (tools/mfma_bf16_round.hip)."""
    import json
    import subprocess
    import sys
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tensor_regression_amd",
                       "libtr_hip_trunc.so")
    assert os.path.exists(lib), "build the negative control first: make -C tensor_regression_amd/csrc negctl"
    env = dict(os.environ, TR_HIP_LIB=lib, TR_SLICE_XPIECES="3")
    env.pop("TR_SLICE_SPLIT", None)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "c5errs"], env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print("c5 negative control (round-3 truncating split)", res)
    assert "bf16split" in res["describe"] and "xpieces=3" in res["describe"], res["describe"]
    worst = max(res["errs"][f"grad{f}"] for f in range(6))
    assert worst > SPEC_GRAD_ABS, res["errs"]


if __name__ == "__main__":
    import sys as _sys
    if len(_sys.argv) > 1 and _sys.argv[1] == "c5errs":
        _sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        _c5_full_size_errs_main()
