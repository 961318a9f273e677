"""GPU parity of the spectral model (tensor_regression_amd.spectral_tensor_regression, kernels in
csrc/tr_spectral.hip and, for shapes beyond its LDS envelope, csrc/tr_spectral_gen.hip — forced
with TR_SPEC_GENERIC=1 to run the fixtures through it too) against the reference's golden fixtures (tests/golden/spec_*.npz) and the
oracle's fp64 closed form (oracle.cp_oracle.closed_form_spectral).

Tolerances (fp32; north_star: 1e-5 relative on the learned factors and the loss trajectory):
  * one step: fit-model y_hat and predict() output elementwise rel <= 1e-5 (atol 1e-5 * max),
    loss rel <= 1e-5, every gradient normwise rel <= 1e-5 (bias 1e-4: a sum of N residuals)
  * 10 Adam iterations: loss_running rel <= 1e-5, factors normwise rel <= 1e-5
  * full horizons: loss_running rel <= 1e-5, same length / convergence flag; factors within
    1e-5 of the reference or no further from the fp64 restatement than the reference is (x2)
"""
import contextlib
import os

import numpy as np
import pytest
import torch

from golden_util import load_spectral, names, normwise_rel


@contextlib.contextmanager
def spec_path(kind):
    """'fused': the plan's own choice (the single-pass kernel inside its envelope); 'generic':
    force the three-kernel path (TR_SPEC_GENERIC=1, read at plan creation); 'slicef32': the
    column-slice kernel's f32-MFMA form instead of its default bf16 split (TR_SLICE_SPLIT=0);
    'slicex3': the split form with the sample data in three pieces (TR_SLICE_XPIECES=3) instead of
    the default two."""
    from tensor_regression_amd import spectral_tensor_regression as SP
    old = os.environ.pop("TR_SPEC_GENERIC", None)
    old_sl = os.environ.pop("TR_SPEC_SLICE", None)
    old_sp = os.environ.pop("TR_SLICE_SPLIT", None)
    old_xp = os.environ.pop("TR_SLICE_XPIECES", None)
    if kind == "slicex3":
        os.environ["TR_SLICE_XPIECES"] = "3"
    if kind == "generic":
        os.environ["TR_SPEC_GENERIC"] = "1"
    if kind == "lockstep":  # the whole-sample lock-step kernel where the column-slice one would run
        os.environ["TR_SPEC_SLICE"] = "0"
    if kind == "slicef32":
        os.environ["TR_SLICE_SPLIT"] = "0"
    SP._plan_cache.clear()
    try:
        yield
    finally:
        os.environ.pop("TR_SPEC_GENERIC", None)
        os.environ.pop("TR_SPEC_SLICE", None)
        os.environ.pop("TR_SLICE_SPLIT", None)
        os.environ.pop("TR_SLICE_XPIECES", None)
        if old_sp is not None:
            os.environ["TR_SLICE_SPLIT"] = old_sp
        if old_xp is not None:
            os.environ["TR_SLICE_XPIECES"] = old_xp
        if old is not None:
            os.environ["TR_SPEC_GENERIC"] = old
        if old_sl is not None:
            os.environ["TR_SPEC_SLICE"] = old_sl
        SP._plan_cache.clear()

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
RTOL = 1e-5
SPEC = [n for n in names("spec_") if n not in ("spec_lbfgs",)]


def _model_from(d, device=DEV):
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression
    m = d["meta"]
    Bn = [torch.tensor(a, device=device).requires_grad_(True) for a in d["Bcp_n0_list"]]
    Bc = [torch.tensor(a, device=device).requires_grad_(True) for a in d["Bcp_c0_list"]]
    X = d["X"]
    return CP_linear_regression(X.shape, (X.shape[0], m["n_out"]), rank_normal=m["rank_normal"],
                                rank_spectral=m["rank_spectral"], non_negative=m["non_negative"],
                                Bcp_init=(Bn, Bc), n_complex_dim=m["n_complex_dim"], device=device,
                                softplus_kwargs=m["softplus_kwargs"])


def _close(got, want, tol=RTOL):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    np.testing.assert_allclose(got, want, rtol=tol, atol=tol * max(1e-30, np.nanmax(np.abs(want))))


def _factors_close(got, want, tol=RTOL):
    for a, b in zip(got, want):
        a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
        if b.size:
            assert normwise_rel(a, b) <= tol, (normwise_rel(a, b), a.shape)


def _as_accurate_as_reference(ours, ref32, ref64, tol=RTOL, slack=2.0):
    for a, b, c in zip(ours, ref32, ref64):
        a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
        if not b.size:
            continue
        e_ref = normwise_rel(a, b)
        if e_ref <= tol:
            continue
        assert normwise_rel(a, c) <= slack * normwise_rel(b, c) + tol, (e_ref, a.shape)


@pytest.mark.parametrize("kind", ["fused", "generic"])
@pytest.mark.parametrize("name", SPEC)
def test_spectral_golden(name, kind):
    with spec_path(kind):
        _spectral_golden(name, kind)


@pytest.mark.parametrize("kind", ["lockstep", "slicef32", "slicex3"])
@pytest.mark.parametrize("name", [n for n in SPEC if n.startswith("spec_slice")])
def test_spectral_slice_golden_lockstep(name, kind):
    """the config-5-shaped fixtures through the whole-sample lock-step kernel, the column-slice
    kernel's f32-MFMA form and its three-piece-X split form as well"""
    with spec_path(kind):
        _spectral_golden(name, kind)


def _spectral_golden(name, kind):
    d = load_spectral(name)
    m = d["meta"]
    X = d["X"].to(DEV)
    y = torch.tensor(d["y"], device=DEV)
    model = _model_from(d)
    desc = model._get_plan(X, X.shape[0]).describe
    assert ("generic" in desc) == (kind == "generic"), desc
    if name.startswith("spec_slice"):
        # fixtures at config 5's sample shape (W = 256, D = 129 / 100) pin the kernel config 5
        # trains with (k_spec_slice) to the reference's own fit_Adam trajectory
        assert ("slice-1pass" in desc) == (kind in ("fused", "slicef32", "slicex3")), desc
        # the default form runs its GEMMs through the bf16 split, the sample data in two pieces
        assert ("bf16split" in desc) == (kind in ("fused", "slicex3")), desc
        if kind in ("fused", "slicex3"):  # lin columns packed (Rn <= 8) or unpacked (spec_slice_rn12_f32x)
            sp = (1 if m['rank_normal'] <= 8 else 2) + (2 if kind == "slicex3" else 0)
            assert f"slsp={sp} xpieces={3 if kind == 'slicex3' else 2}" in desc, desc
    # predict() = lin_model + spectral_model (spectral…py:959-960)
    _close(model.predict(X).numpy(), d["predict0"])
    # one forward + loss + gradient (fit model, spectral…py:716-720)
    plan = model._get_plan(X, X.shape[0])
    arena = plan.pack(model.Bcp_n, model.Bcp_c, model.bias)
    w = model.weights.to(DEV)
    grad = torch.zeros(plan.num_grads, device=DEV)
    gtot = torch.zeros(plan.num_params, device=DEV)
    loss = torch.zeros(1, device=DEV)
    yhat = torch.empty_like(y)
    plan.loss_grad(X, y, None, float(y.numel()), arena, w, grad, yhat=yhat)
    plan.finalize_grad(arena, grad, m["lambda_L2"], gtot, loss)
    if m["nan_y"]:
        assert np.isnan(loss.item()) and np.isnan(d["loss0"])
    else:
        _close(yhat.cpu().numpy(), d["y_hat0"])
        assert abs(loss.item() - d["loss0"]) <= RTOL * abs(d["loss0"])
        views = plan.factor_views(gtot)
        if m["rank_normal"]:
            _factors_close(views[:3], d["grads_n0_list"])
        if m["rank_spectral"]:
            _factors_close(views[3:], d["grads_c0_list"])
        assert normwise_rel(gtot[plan.offsets[6]:].cpu().numpy(), d["bias_grad0"]) <= 1e-4
    # 10-iteration snapshot
    m10 = _model_from(d)
    m10.fit_Adam(X, y, lambda_L2=m["lambda_L2"], max_iter=min(10, m["max_iter"]), tol=m["tol"],
                 patience=m["patience"], Adam_kwargs=m["adam_kwargs"])
    if m["nan_y"]:
        assert len(m10.loss_running) == len(d["loss_running_10"]) == 1 and np.isnan(m10.loss_running[0])
    else:
        np.testing.assert_allclose(m10.loss_running, d["loss_running_10"], rtol=RTOL)
        _factors_close(m10.Bcp_n, d["Bcp_n_10_list"])
        _factors_close(m10.Bcp_c, d["Bcp_c_10_list"])
    # full Adam trajectory
    conv = model.fit_Adam(X, y, lambda_L2=m["lambda_L2"], max_iter=m["max_iter"], tol=m["tol"],
                          patience=m["patience"], Adam_kwargs=m["adam_kwargs"])
    assert int(conv) == int(d["converged"])
    assert len(model.loss_running) == len(d["loss_running"])
    if m["nan_y"]:
        assert np.isnan(model.loss_running).all()
        return
    np.testing.assert_allclose(model.loss_running, d["loss_running"], rtol=RTOL)
    from oracle import cp_oracle
    r64 = cp_oracle.fit_adam_spectral(d["X"], d["y"], d["Bcp_n0_list"], d["Bcp_c0_list"], np.zeros(m["n_out"]),
                                      np.ones(m["rank_normal"] + m["rank_spectral"]), m["rank_normal"],
                                      m["non_negative"], m["lambda_L2"], m["max_iter"], m["tol"], m["patience"],
                                      m["adam_kwargs"], m["softplus_kwargs"], dtype=torch.float64)
    _as_accurate_as_reference(model.Bcp_n, d["Bcp_n_final_list"], r64["Bcp_n"])
    _as_accurate_as_reference(model.Bcp_c, d["Bcp_c_final_list"], r64["Bcp_c"])
    # predict() at the final point: the kernel against the fp64 predict model of OUR final factors
    # (1e-5), and the reference's predict_final within the distance the factors themselves allow
    # (the trajectories agree to 1e-5 on the losses; the final factors as accurately as above)
    fin = cp_oracle.spectral_predict(X.cpu().double(), [a.detach().cpu().double() for a in model.Bcp_n],
                                     [a.detach().cpu().double() for a in model.Bcp_c],
                                     torch.ones(m["rank_normal"] + m["rank_spectral"], dtype=torch.float64),
                                     m["rank_normal"], m["non_negative"], model.bias.detach().cpu().double(),
                                     m["softplus_kwargs"]).numpy()
    p_fin = model.predict(X).numpy()
    assert normwise_rel(p_fin, fin) <= RTOL, normwise_rel(p_fin, fin)
    ref_fin = cp_oracle.spectral_predict(X.cpu().double(), [torch.tensor(a).double() for a in d["Bcp_n_final_list"]],
                                         [torch.tensor(a).double() for a in d["Bcp_c_final_list"]],
                                         torch.ones(m["rank_normal"] + m["rank_spectral"], dtype=torch.float64),
                                         m["rank_normal"], m["non_negative"], torch.tensor(d["bias_final"]).double(),
                                         m["softplus_kwargs"]).numpy()
    assert normwise_rel(ref_fin, d["predict_final"]) <= RTOL  # the oracle's predict model is the reference's
    e_ref = normwise_rel(p_fin, d["predict_final"])
    # hard bar whatever arm passes: the pre-round-3 fixed 1e-4 against the reference's output
    assert e_ref <= 1e-4, e_ref
    if e_ref > RTOL:  # as accurate as the reference's own fp32 run, against the fp64 trajectory
        print(f"predict_final: {e_ref:.2e} from the reference's output > {RTOL:g}; fp64-distance arm")
        r64p = cp_oracle.spectral_predict(X.cpu().double(), [torch.tensor(a).double() for a in r64["Bcp_n"]],
                                          [torch.tensor(a).double() for a in r64["Bcp_c"]],
                                          torch.ones(m["rank_normal"] + m["rank_spectral"], dtype=torch.float64),
                                          m["rank_normal"], m["non_negative"], torch.as_tensor(r64["bias"]).double(),
                                          m["softplus_kwargs"]).numpy()
        assert normwise_rel(p_fin, r64p) <= 2 * normwise_rel(d["predict_final"], r64p) + RTOL, e_ref


def test_spectral_lbfgs_golden():
    d = load_spectral("spec_lbfgs")
    m = d["meta"]
    X = d["X"].to(DEV)
    y = torch.tensor(d["y"], device=DEV)
    model = _model_from(d)
    conv = model.fit(X, y, lambda_L2=m["lambda_L2"], max_iter=m["max_iter"], tol=m["tol"], patience=m["patience"],
                     running_loss_logging_interval=m["logging_interval"], LBFGS_kwargs=m["lbfgs_kwargs"])
    assert int(conv) == int(d["converged"])
    assert len(model.loss_running) == len(d["loss_running"])
    # strong-Wolfe line searches amplify fp32 reduction-order differences step by step (the
    # reference's own fp32 run is 3.4e-3 relative away from the fp64 trajectory by step 2), so
    # the bar is: no further from fp64 than 4x the reference's fp32 deviation so far, + 1e-5
    from oracle import cp_oracle
    r64 = cp_oracle.fit_lbfgs_spectral(d["X"], d["y"], d["Bcp_n0_list"], d["Bcp_c0_list"], np.zeros(m["n_out"]),
                                       np.ones(m["rank_normal"] + m["rank_spectral"]), m["rank_normal"],
                                       m["non_negative"], m["lambda_L2"], m["max_iter"], m["tol"], m["patience"],
                                       m["logging_interval"], m["lbfgs_kwargs"], m["softplus_kwargs"],
                                       dtype=torch.float64)
    ours, ref32, ref64 = (np.asarray(v, np.float64) for v in (model.loss_running, d["loss_running"],
                                                              r64["loss_running"]))
    assert abs(ours[0] - ref32[0]) <= RTOL * abs(ref32[0])
    bound = 4 * np.maximum.accumulate(np.abs(ref32 - ref64)) + RTOL * np.abs(ref64)
    assert np.all(np.abs(ours - ref64) <= bound), (ours, ref32, ref64)


SHAPES = [
    # (N, W, D, n_out, Rn, Rs, n_complex_dim, non_negative)
    (300, 256, 129, 2, 8, 8, 1, [False, False, False]),   # config-5 sample shape
    (257, 64, 33, 3, 4, 6, 1, [True, False, True]),
    (130, 100, 50, 2, 5, 3, 2, [False, True, False]),     # W, D not multiples of 16 / 4, even D
    (64, 48, 200, 5, 16, 8, 1, [False, False, False]),    # K = 32, D = 200
    (77, 17, 7, 2, 0, 4, 1, [False, False, False]),       # rank_normal = 0
    (77, 17, 7, 2, 3, 0, 1, [False, False, False]),       # rank_spectral = 0
]
# shapes of the column-slice training kernel (csrc/tr_spectral_slice.hip: W <= 256, D <= 130,
# Rn <= 16, Rs * Cc <= 16, Cc in {1, 2, 4}): every variant of its tail rows (D - 128 = 0, 1, 2),
# masked columns (D < 128) and norm groups
SLICE_SHAPES = [
    (200, 256, 128, 3, 8, 4, 3, [False, True, False]),    # Cc = 4, Rs * Cc = 16, no tail rows
    (150, 256, 130, 2, 8, 8, 0, [True, False, True]),     # Cc = 1, two tail rows
    (120, 256, 100, 5, 3, 5, 1, [False, False, False]),   # D < 128 (columns past D masked)
    (64, 256, 129, 8, 8, 8, 1, [False, False, False]),    # n_out = 8
    (64, 256, 129, 40, 8, 8, 1, [False, False, False]),   # n_out = 40: beyond the slice kernel's LDS
    # 9 <= Rn <= 16: the split form with unpacked lin columns (SP = 2), every tail-row variant
    (96, 256, 129, 2, 12, 4, 1, [False, False, False]),   # Rn = 12, one tail row
    (80, 256, 100, 3, 16, 4, 1, [False, True, False]),    # Rn = 16, D < 128 (with D >= 129 beyond LDS)
    (64, 256, 130, 2, 9, 2, 3, [True, False, False]),     # Rn = 9, Cc = 4, two tail rows
    # D < 128 of any residue: a partial last column quad (its columns past D are the next row's
    # first values, or zeros past the sample, times zero factor rows) and whole padded pairs
    (90, 256, 101, 2, 8, 8, 1, [False, False, False]),    # D % 4 = 1
    (70, 256, 127, 2, 8, 8, 1, [True, False, False]),     # D % 4 = 3
    (100, 256, 96, 3, 8, 4, 1, [False, True, False]),     # the fourth pair's columns all past D
    (80, 256, 65, 2, 6, 8, 1, [False, False, False]),     # D = 65 (a length-128 rfft)
    (60, 256, 34, 2, 4, 4, 1, [False, False, True]),      # one pair and two columns of a second
    (50, 256, 3, 2, 2, 3, 1, [False, False, False]),      # three columns: one partial quad in all
    # W < 256: rows past W read zeros and meet zero Phi0 rows
    (90, 200, 129, 2, 8, 8, 1, [False, False, False]),    # the second half partly past W
    (80, 128, 65, 3, 8, 4, 1, [False, True, False]),      # the second half wholly past W
    (70, 100, 130, 2, 6, 6, 1, [True, False, False]),     # two tail rows, the first half partly past W
]
# beyond the fused kernel's envelope: the generic path whatever TR_SPEC_GENERIC says
WIDE_SHAPES = [
    (40, 300, 257, 3, 4, 5, 1, [False, True, False]),     # W > 256 and D > 256
    (50, 64, 40, 2, 8, 16, 1, [False, False, False]),     # K = 8 + 16*2 = 40 > 32
    (30, 20, 9, 300, 3, 2, 1, [True, False, False]),      # n_out = 300 > 256
    (20, 520, 33, 2, 2, 3, 3, [False, False, True]),      # W = 520, Cc = 4
]


def _slice_shape(W, D, Rn, Rs, ncd, O):
    """the column-slice kernel's envelope (spec_slice_geom in csrc/tr_spectral_slice.hip)"""
    ok = (W <= 256 and D <= 130 and 1 <= Rn <= 16 and Rs >= 1
          and Rs * (ncd + 1) <= 16 and ncd + 1 in (1, 2, 4) and O <= 64)
    small = ((max(D, 128) + 3) // 4 * 4) * (Rn + Rs) + O * 33 + 16 + O * (Rn + Rs + 1) + 64
    return ok and (38144 + ((small + 3) & ~3) + 4) * 4 <= 160 * 1024


@pytest.mark.parametrize("kind", ["lockstep", "slicef32", "slicex3"])
@pytest.mark.parametrize("N,W,D,O,Rn,Rs,ncd,nn", [SHAPES[0]] + SLICE_SHAPES)
def test_spectral_slice_shapes_lockstep_kernel(N, W, D, O, Rn, Rs, ncd, nn, kind):
    """the same shapes through the whole-sample lock-step kernel (TR_SPEC_SLICE=0), the
    column-slice kernel's f32-MFMA form (TR_SLICE_SPLIT=0) and its three-piece-X split form"""
    with spec_path(kind):
        _spectral_shape(N, W, D, O, Rn, Rs, ncd, nn, kind)


@pytest.mark.parametrize("kind", ["fused", "generic"])
@pytest.mark.parametrize("N,W,D,O,Rn,Rs,ncd,nn", SHAPES + SLICE_SHAPES + WIDE_SHAPES)
def test_spectral_shapes_vs_closed_form(N, W, D, O, Rn, Rs, ncd, nn, kind):
    if kind == "fused" and (N, W, D, O, Rn, Rs, ncd, nn) in WIDE_SHAPES:
        pytest.skip("beyond the fused envelope: covered by the generic case")
    with spec_path(kind):
        _spectral_shape(N, W, D, O, Rn, Rs, ncd, nn, kind)


def _spectral_shape(N, W, D, O, Rn, Rs, ncd, nn, kind):
    from oracle import cp_oracle
    g = torch.Generator().manual_seed(N + W + D)
    X = torch.randn(N, W, D, generator=g)
    y = torch.randn(N, O, generator=g)
    Bn = [torch.randn(W, Rn, 1, generator=g) * 0.2, torch.randn(D, Rn, 1, generator=g) * 0.2,
          torch.randn(O, Rn, 1, generator=g)]
    Bc = [torch.randn(W, Rs, ncd + 1, generator=g) * 0.2, torch.randn(D, Rs, 1, generator=g) * 0.2,
          torch.randn(O, Rs, 1, generator=g)]
    bias = torch.randn(O, generator=g) * 0.1
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression
    model = CP_linear_regression(X.shape, y.shape, rank_normal=Rn, rank_spectral=Rs, non_negative=nn,
                                 Bcp_init=([a.to(DEV) for a in Bn], [a.to(DEV) for a in Bc]), n_complex_dim=ncd,
                                 device=DEV)
    model.bias = bias.to(DEV)
    Xd, yd = X.to(DEV), y.to(DEV)
    plan = model._get_plan(Xd, N)
    wide = W > 256 or D > 256 or O > 256 or Rn + Rs * (ncd + 1) > 32
    if kind == "generic" or (kind == "fused" and wide):
        assert "generic" in plan.describe, plan.describe
    slice_ok = _slice_shape(W, D, Rn, Rs, ncd, O)
    assert ("slice" in plan.describe) == (kind in ("fused", "slicef32", "slicex3") and slice_ok), plan.describe
    assert ("bf16split" in plan.describe) == (kind in ("fused", "slicex3") and slice_ok), plan.describe
    if kind in ("fused", "slicex3") and slice_ok:  # lin columns packed two split parts per tile (Rn <= 8) or not
        sp = (1 if Rn <= 8 else 2) + (2 if kind == "slicex3" else 0)
        assert f"slsp={sp} xpieces={3 if kind == 'slicex3' else 2}" in plan.describe, plan.describe
    arena = plan.pack(model.Bcp_n, model.Bcp_c, model.bias)
    w = torch.ones(Rn + Rs, device=DEV)
    grad = torch.zeros(plan.num_grads, device=DEV)
    gtot = torch.zeros(plan.num_params, device=DEV)
    loss = torch.zeros(1, device=DEV)
    yhat = torch.empty_like(yd)
    plan.loss_grad(Xd, yd, None, float(N * O), arena, w, grad, yhat=yhat)
    plan.finalize_grad(arena, grad, 0.01, gtot, loss)
    c = cp_oracle.closed_form_spectral(X.numpy(), y.numpy(), [a.numpy() for a in Bn], [a.numpy() for a in Bc],
                                       bias.numpy(), np.ones(Rn + Rs), Rn, nn, 0.01)
    assert normwise_rel(yhat.cpu().numpy(), c["y_hat"]) <= RTOL
    assert abs(loss.item() - c["loss"]) <= RTOL * abs(c["loss"])
    views = plan.factor_views(gtot)
    for v, ref in zip(views, c["grads_n"] + c["grads_c"]):
        if ref.size:
            assert normwise_rel(v.cpu().numpy(), ref) <= 2 * RTOL, (v.shape, normwise_rel(v.cpu().numpy(), ref))
    assert normwise_rel(gtot[plan.offsets[6]:].cpu().numpy(), c["bias_grad"]) <= 1e-4
    # predict model (norm after the contraction) against the torch restatement in fp64
    p = model.predict(Xd).numpy()
    ref = cp_oracle.spectral_predict(X.double(), [a.double() for a in Bn], [a.double() for a in Bc],
                                     torch.ones(Rn + Rs, dtype=torch.float64), Rn, nn, bias.double()).numpy()
    assert normwise_rel(p, ref) <= RTOL
    # latents (stepwise_latents_model)
    if Rn:
        lat = model.predict_latents(Xd)
        ref_lat = np.einsum('twd,wr,dr->tr', X.double().numpy(), Bn[0][:, :, 0].double().numpy() if not nn[0] else
                            torch.nn.functional.softplus(Bn[0][:, :, 0].double(), beta=50, threshold=1).numpy(),
                            Bn[1][:, :, 0].double().numpy() if not nn[1] else
                            torch.nn.functional.softplus(Bn[1][:, :, 0].double(), beta=50, threshold=1).numpy())
        assert normwise_rel(lat, ref_lat) <= RTOL


@pytest.mark.parametrize("kind", ["fused", "lockstep", "generic"])
def test_spectral_bitwise_reproducible_and_sharded_sum(kind):
    with spec_path(kind):
        _spectral_bitwise(kind)


def _spectral_bitwise(kind):
    N, W, D, O = 1000, 256, 129, 2
    g = torch.Generator().manual_seed(5)
    X = torch.randn(N, W, D, generator=g).to(DEV)
    y = torch.randn(N, O, generator=g).to(DEV)
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression
    torch.manual_seed(0)
    model = CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV)
    plan = model._get_plan(X, N)
    arena = plan.pack(model.Bcp_n, model.Bcp_c, model.bias)
    w = torch.ones(16, device=DEV)
    outs = []
    for _ in range(3):
        grad = torch.zeros(plan.num_grads, device=DEV)
        plan.loss_grad(X, y, None, float(N * O), arena, w, grad)
        outs.append(grad.clone())
    # consecutive calls walk each workgroup's samples in opposite orders (Infinity Cache reuse),
    # so calls of equal parity are bitwise identical and neighbours agree to rounding
    assert torch.equal(outs[0], outs[2])
    assert normwise_rel(outs[1].cpu().numpy(), outs[0].cpu().numpy()) <= 1e-6
    g1 = torch.zeros(plan.num_grads, device=DEV)
    g2 = torch.zeros(plan.num_grads, device=DEV)
    plan.loss_grad(X[:400], y[:400], None, float(N * O), arena, w, g1)
    plan.loss_grad(X[400:], y[400:], None, float(N * O), arena, w, g2)
    assert normwise_rel((g1 + g2).cpu().numpy(), outs[0].cpu().numpy()) <= 1e-6
    # an empty shard contributes exactly zero
    g0 = torch.ones(plan.num_grads, device=DEV)
    plan.loss_grad(X[:0], y[:0], None, float(N * O), arena, w, g0)
    assert not g0.any()


def test_spectral_envelope_errors():
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression
    # K = 10 + 100 * 3 > 256 columns: outside both paths
    X = torch.zeros(4, 30, 10, device=DEV)
    y = torch.zeros(4, 2, device=DEV)
    m = CP_linear_regression(X.shape, y.shape, rank_normal=10, rank_spectral=100, n_complex_dim=2, device=DEV)
    with pytest.raises(ValueError, match="rank_normal"):
        m.fit_Adam(X, y, max_iter=1, Adam_kwargs={'lr': 0.01})
    # one sample's epilogue beyond a CU's LDS (D * (K + 1) floats)
    X = torch.zeros(2, 8, 5000, device=DEV)
    m = CP_linear_regression(X.shape, y[:2].shape, rank_normal=4, rank_spectral=4, device=DEV)
    with pytest.raises(ValueError, match="LDS"):
        m.fit_Adam(X, y[:2], max_iter=1, Adam_kwargs={'lr': 0.01})
    m = CP_linear_regression((4, 8, 5), (4, 1), rank_normal=2, rank_spectral=2, device=DEV)
    with pytest.raises(NotImplementedError):
        m.fit_Adam(torch.zeros(4, 8, 5, device=DEV), torch.zeros(4, 1, device=DEV), max_iter=1,
                   Adam_kwargs={'lr': 0.01})
