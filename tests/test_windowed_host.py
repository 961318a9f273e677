"""Windowed / out-of-core data path (reference util.py:67-98 WindowedDataset).

CPU: windowed_view / WindowedDataset reproduce the reference's windows, pinned by the win_*
fixtures (tools/gen_golden.py stacks the reference WindowedDataset's samples and fits them with
the reference's own fit_Adam): the oracle fitted on our windows reproduces those fixtures bit for
bit.  GPU (gpu-marked): fit_Adam over the strided windowed view, over the materialised windows and
over a HostStream of them, each against the same fixtures at the 1e-5 parity bar; plus
windowed-vs-materialised bitwise checks on wider shapes."""
import numpy as np
import pytest
import torch

from golden_util import load, names, normwise_rel
from tensor_regression_amd import util

WIN = names("win_")


def _windows(d):
    """The fixture's series -> (windows view, targets) through our windowed_view."""
    m = d["meta"]
    S = d["X"]  # the untiled series (X_q / 8)
    y = torch.tensor(d["y_series"])
    return util.windowed_view(S, y, m["win_range"])


@pytest.mark.parametrize("win_range", [(-3, 4), (0, 5), (-6, 1), (2, 6)])
def test_windowed_dataset_indexing(win_range):
    """WindowedDataset numbering: ds[idx] == X[idx + w0 : idx + w1], y[idx] for idx in usable_idx
    (reference util.py:72, 93-96), zero-copy over the series."""
    g = torch.Generator().manual_seed(0)
    X = torch.randn(40, 5, 3, generator=g)
    y = torch.randn(40, generator=g)
    ds = util.WindowedDataset(X, y, list(win_range))
    w0, w1 = win_range
    assert torch.equal(ds.usable_idx, torch.arange(-w0, 40 - w1 + 1))
    assert ds.windows.shape == (len(ds.usable_idx), w1 - w0, 5, 3)
    assert ds.windows.stride(0) == 15 and ds.windows.data_ptr() == X.data_ptr()  # no copy
    for idx in ds.usable_idx.tolist():
        xi, yi = ds[idx]
        assert torch.equal(xi, X[idx + w0: idx + w1]) and torch.equal(yi, y[idx])
    with pytest.raises(IndexError):
        ds[int(ds.usable_idx[-1]) + 1]
    with pytest.raises(ValueError):
        util.WindowedDataset(X, y[:-1], list(win_range))
    with pytest.raises(ValueError):  # a target vector of the wrong length is refused on the host
        util.windowed_view(X, y[:-2], win_range)


@pytest.mark.parametrize("win_range", [(-3, 4), (2, 6)])
def test_windowed_dataloader_surface(win_range):
    """The reference's loader surface (util.py:67-114): WindowedDataset is a torch Dataset whose
    len() is the series length and which takes (and, like the reference, does not apply) transform
    / target_transform; make_WindowedDataloader returns (dataloader, dataset, sampler) with a
    SubsetRandomSampler over usable_idx, drop_last, and sample_shape = [batch_size] + window shape;
    every batch stacks the reference's windows X[idx + w0 : idx + w1] and targets y[idx]."""
    g = torch.Generator().manual_seed(1)
    X = torch.randn(50, 4, 3, generator=g)
    y = torch.randn(50, generator=g)
    w0, w1 = win_range
    ds = util.WindowedDataset(X, y, list(win_range), transform=lambda v: v * 0, target_transform=abs)
    assert isinstance(ds, torch.utils.data.Dataset)
    assert len(ds) == 50 and ds.n_windows == 50 - (w1 - w0) + 1
    xi, yi = ds[int(ds.usable_idx[3])]
    assert torch.equal(xi, X[int(ds.usable_idx[3]) + w0:int(ds.usable_idx[3]) + w1])  # not transformed
    dl, ds2, sampler = util.make_WindowedDataloader(X, y, win_range=list(win_range), batch_size=8, drop_last=True)
    assert isinstance(sampler, torch.utils.data.SubsetRandomSampler)
    assert sorted(int(i) for i in sampler.indices) == ds2.usable_idx.tolist()
    assert dl.sample_shape == [8, w1 - w0, 4, 3]
    seen = []
    usable = set(ds2.usable_idx.tolist())
    for xb, yb in dl:
        assert xb.shape == (8, w1 - w0, 4, 3) and yb.shape == (8,)
        for k in range(8):
            idx = int(torch.nonzero(y == yb[k])[0])  # (the targets are distinct draws)
            if idx not in usable:  # a negative idx (w0 > 0): y[idx] wraps to the end, as in the reference
                idx -= 50
            assert idx in usable and torch.equal(xb[k], X[idx + w0: idx + w1])
            seen.append(idx)
    assert len(seen) == len(set(seen)) == (ds2.n_windows // 8) * 8  # each window once; drop_last


@pytest.fixture()
def _one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)  # fixtures were produced single-threaded (fixed summation order)
    yield
    torch.set_num_threads(n)


@pytest.mark.parametrize("name", WIN)
def test_oracle_on_windowed_view_matches_reference(name, _one_thread):
    """The reference's WindowedDataset samples, fitted by the reference fit_Adam (fixture), are
    reproduced bit for bit by the oracle run on OUR windows: pins windowed_view to util.py:67-98."""
    from oracle import cp_oracle
    d = load(name)
    m = d["meta"]
    Xw, yw = _windows(d)
    assert Xw.shape[0] == m["n_windows"] and list(Xw.shape[1:]) == m["window_shape"]
    ones = np.ones(m["rank"], np.float32)
    X = Xw.contiguous()
    if m["n_classes"]:
        f = cp_oracle.fit_adam_mnl(X, yw, d["Bcp0_list"], ones, m["non_negative"], np.ones(m["n_classes"]),
                                   m["lambda_L2"], m["max_iter"], m["tol"], m["patience"], m["adam_kwargs"],
                                   m["softplus_kwargs"])
    else:
        f = cp_oracle.fit_adam_linear(X, yw, d["Bcp0_list"], d["bias0"], ones, m["non_negative"], m["lambda_L2"],
                                      m["max_iter"], m["tol"], m["patience"], m["adam_kwargs"], m["softplus_kwargs"])
    np.testing.assert_array_equal(np.array(f["loss_running"]), d["loss_running"])
    for a, b in zip(f["Bcp"], d["Bcp_final_list"]):
        np.testing.assert_array_equal(a, b)


def test_rows_contiguous_detection():
    from tensor_regression_amd._engine import _rows_contiguous
    X = torch.randn(50, 7)
    Xw, _ = util.windowed_view(X, torch.zeros(50), (0, 4))
    assert _rows_contiguous(Xw)
    assert _rows_contiguous(torch.randn(6, 4, 3)[::2])
    assert not _rows_contiguous(torch.randn(6, 4, 3).transpose(1, 2))


DEV = "cuda:0"


@pytest.mark.gpu
@pytest.mark.parametrize("twopass,F", [(False, 32), (True, 32), (False, 4096)])
def test_windowed_linear_fit_equals_materialised(twopass, F, monkeypatch):
    """F = 32: windows of 16 rows -> P = 512 (single pass); F = 4096: P = 65536 > LDS (cluster
    single pass reading the overlapping windows through the row stride)."""
    from tensor_regression_amd import standard_tensor_regression as S
    if twopass:
        monkeypatch.setenv("TR_FORCE_TWOPASS", "1")
    S._plan_cache.clear()
    g = torch.Generator().manual_seed(1)
    T = 3000 if F == 32 else 400
    X = torch.randn(T, F, generator=g).to(DEV)  # untiled (T, F)
    y = torch.randn(T, generator=g).to(DEV)
    Xw, yw = util.windowed_view(X, y, (-8, 8))
    Xm = Xw.contiguous()
    res = []
    for XX in (Xw, Xm):
        torch.manual_seed(2)
        m = S.CP_linear_regression(XX.shape, rank=4, device=DEV)
        m.fit_Adam(XX, yw, lambda_L2=0.01, max_iter=20, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
        res.append((m.loss_running, [a.detach().cpu() for a in m.Bcp], m._plan.describe))
    if F == 4096:
        assert "cluster-1pass" in res[0][2], res[0][2]
    assert res[0][0] == res[1][0], "windowed view must give the materialised result bit for bit"
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)
    S._plan_cache.clear()


@pytest.mark.gpu
def test_windowed_spectral_and_multinomial_equal_materialised():
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression as SpecCP
    from tensor_regression_amd import CP_logistic_regression
    g = torch.Generator().manual_seed(3)
    X = torch.randn(600, 33, generator=g).abs().to(DEV)  # windows (16, 33): odd stride -> 4-B DMA path
    y2 = torch.randn(600, 2, generator=g).to(DEV)
    Xw, yw = util.windowed_view(X, y2, (0, 16))
    out = []
    for XX in (Xw, Xw.contiguous()):
        torch.manual_seed(4)
        m = SpecCP(XX.shape, yw.shape, rank_normal=2, rank_spectral=2, n_complex_dim=1, device=DEV)
        m.fit_Adam(XX, yw, lambda_L2=0.01, max_iter=10, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
        out.append((m.loss_running, m.predict(XX)))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1])

    lab = torch.randint(0, 3, (600,), generator=g)
    lab[:3] = torch.arange(3)
    Xw1, lw = util.windowed_view(X, lab, (0, 8))
    outm = []
    for XX in (Xw1, Xw1.contiguous()):
        torch.manual_seed(5)
        mm = CP_logistic_regression(XX, lw.numpy(), rank=2, device=DEV)
        mm.fit_Adam(lambda_L2=0.01, max_iter=10, tol=0, patience=10, weights=np.ones(3), Adam_kwargs={"lr": 0.01})
        outm.append(mm.loss_running)
    assert outm[0] == outm[1]


@pytest.mark.gpu
def test_host_stream_fit_matches_resident():
    from tensor_regression_amd import CP_linear_regression
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression as SpecCP
    g = torch.Generator().manual_seed(6)
    X = torch.randn(5000, 16, 16, generator=g)
    y = torch.randn(5000, generator=g)
    res = []
    for XX in (X.to(DEV), util.HostStream(X, chunk_rows=1234, device=DEV)):
        torch.manual_seed(7)
        m = CP_linear_regression((5000, 16, 16), rank=3, device=DEV)
        m.fit_Adam(XX, y.to(DEV), lambda_L2=0.01, max_iter=15, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
        res.append((np.array(m.loss_running), [a.detach().cpu().numpy() for a in m.Bcp]))
    np.testing.assert_allclose(res[1][0], res[0][0], rtol=1e-5)
    for a, b in zip(res[1][1], res[0][1]):
        assert np.linalg.norm(a - b) <= 1e-5 * np.linalg.norm(b)

    Xs = torch.randn(700, 24, 17, generator=g)
    ys = torch.randn(700, 2, generator=g)
    res = []
    for XX in (Xs.to(DEV), util.HostStream(Xs, chunk_rows=300, device=DEV)):
        torch.manual_seed(8)
        m = SpecCP((700, 24, 17), (700, 2), rank_normal=2, rank_spectral=2, n_complex_dim=1, device=DEV)
        m.fit_Adam(XX, ys.to(DEV), lambda_L2=0.01, max_iter=10, tol=0, patience=10, Adam_kwargs={"lr": 0.01})
        res.append(np.array(m.loss_running))
    np.testing.assert_allclose(res[1], res[0], rtol=1e-5)


def _assert_close_factors(got, want, tol=1e-5):
    for a, b in zip(got, want):
        a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
        assert normwise_rel(a, b) <= tol, (normwise_rel(a, b), a.shape)


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["view", "materialised", "hoststream"])
@pytest.mark.parametrize("name", [n for n in WIN if not n.startswith("win_mnl")])
def test_windowed_linear_golden(name, source):
    """fit_Adam over the windowed data vs the reference's fit of its WindowedDataset samples:
    one loss + gradient at the init point, the 10-iteration factors and the full loss trajectory
    at 1e-5 (SURVEY §8(c) parity definition)."""
    from tensor_regression_amd import CP_linear_regression
    d = load(name)
    m = d["meta"]
    Xw, yw = _windows(d)
    yd = yw.to(DEV)
    if source == "view":
        XX = util.windowed_view(d["X"].to(DEV), torch.tensor(d["y_series"], device=DEV), m["win_range"])[0]
        assert XX.stride(0) != int(np.prod(XX.shape[1:]))  # really the overlapping view
    elif source == "materialised":
        XX = Xw.contiguous().to(DEV)
    else:
        XX = util.HostStream(Xw.contiguous(), chunk_rows=max(1, Xw.shape[0] // 3), device=DEV)

    def make():
        Bcp = [torch.tensor(a, device=DEV).requires_grad_(True) for a in d["Bcp0_list"]]
        return CP_linear_regression((Xw.shape[0],) + tuple(Xw.shape[1:]), rank=m["rank"], Bcp_init=Bcp,
                                    bias_init=float(d["bias0"][0]), device=DEV)

    if source != "hoststream":
        model = make()
        plan = model._get_plan(XX, XX.shape[0])
        arena = plan.pack(model.Bcp, model.bias)
        grad = torch.zeros(plan.num_grads, device=DEV)
        gtot = torch.zeros(plan.num_params, device=DEV)
        loss = torch.zeros(1, device=DEV)
        plan.loss_grad(XX, yd, None, float(XX.shape[0]), arena, model.weights, grad)
        plan.finalize_grad(arena, grad, m["lambda_L2"], gtot, loss)
        assert abs(loss.item() - d["loss0"]) <= 1e-5 * abs(d["loss0"])
        _assert_close_factors(plan.factor_views(gtot), d["grads0_list"])
    m10 = make()
    m10.fit_Adam(XX, yd, lambda_L2=m["lambda_L2"], max_iter=10, tol=0, patience=10, Adam_kwargs=m["adam_kwargs"])
    np.testing.assert_allclose(m10.loss_running, d["loss_running_10"], rtol=1e-5)
    _assert_close_factors(m10.Bcp, d["Bcp_10_list"])
    model = make()
    model.fit_Adam(XX, yd, lambda_L2=m["lambda_L2"], max_iter=m["max_iter"], tol=0, patience=10,
                   Adam_kwargs=m["adam_kwargs"])
    assert len(model.loss_running) == len(d["loss_running"])
    np.testing.assert_allclose(model.loss_running, d["loss_running"], rtol=1e-5)
    # final factors: within 1e-5 of the reference, or no further from the fp64 restatement of
    # the same trajectory than the reference's own fp32 run is (x2) -- the long-horizon bar of
    # test_gpu_parity.py (Adam amplifies fp32 reduction-order noise)
    from oracle import cp_oracle
    r64 = cp_oracle.fit_adam_linear(Xw.contiguous(), yw, d["Bcp0_list"], d["bias0"], np.ones(m["rank"]),
                                    m["non_negative"], m["lambda_L2"], m["max_iter"], 0.0, 10, m["adam_kwargs"],
                                    m["softplus_kwargs"], dtype=torch.float64)
    for a, b, c in zip(model.Bcp, d["Bcp_final_list"], r64["Bcp"]):
        a = a.detach().cpu().numpy()
        if normwise_rel(a, b) > 1e-5:
            assert normwise_rel(a, c) <= 2 * normwise_rel(b, c) + 1e-5, (normwise_rel(a, b), normwise_rel(a, c))


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["view", "materialised", "hoststream"])
def test_windowed_multinomial_golden(source):
    from tensor_regression_amd import CP_logistic_regression
    d = load("win_mnl")
    m = d["meta"]
    Xw, yw = _windows(d)
    if source == "view":
        XX = util.windowed_view(d["X"].to(DEV), torch.tensor(d["y_series"], device=DEV), m["win_range"])[0]
    elif source == "materialised":
        XX = Xw.contiguous().to(DEV)
    else:  # host-resident windows streamed through two device buffers, 3 chunks per iteration
        XX = util.HostStream(Xw.contiguous(), chunk_rows=max(1, Xw.shape[0] // 3), device=DEV)

    def make():
        return CP_logistic_regression(XX, yw.numpy(), rank=m["rank"], device=DEV,
                                      Bcp_init=[torch.tensor(a, device=DEV) for a in d["Bcp0_list"]])

    from tensor_regression_amd.multinomial_tensor_regression import model as mnl_model
    mm = make()
    if source == "hoststream":
        S = mm.predict()[0]
    else:
        S = mnl_model(XX, mm.Bcp, mm.weights, mm.non_negative, mm.softplus_kwargs).cpu().numpy()
    np.testing.assert_allclose(S, d["probs0"], rtol=1e-5, atol=1e-6)
    m10 = make()
    m10.fit_Adam(lambda_L2=m["lambda_L2"], max_iter=10, tol=0, patience=10, weights=np.ones(m["n_classes"]),
                 Adam_kwargs=m["adam_kwargs"])
    np.testing.assert_allclose(m10.loss_running, d["loss_running_10"], rtol=1e-5)
    _assert_close_factors(m10.Bcp, d["Bcp_10_list"])
    mm.fit_Adam(lambda_L2=m["lambda_L2"], max_iter=m["max_iter"], tol=0, patience=10,
                weights=np.ones(m["n_classes"]), Adam_kwargs=m["adam_kwargs"])
    np.testing.assert_allclose(mm.loss_running, d["loss_running"], rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["spec_basic", "spec_nonneg_amsgrad_wd", "spec_slice_shape"])
def test_spectral_hoststream_golden(name):
    """The spectral fit_Adam (spectral…py:652-743) over a HostStream of the fixture's X (3 chunks
    per iteration, each chunk's arena summed like a shard) against the reference's fixture: the
    10-iteration loss trajectory and factors and the full trajectory at 1e-5, predict() at 1e-5."""
    from golden_util import load_spectral
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression as SpecCP
    d = load_spectral(name)
    m = d["meta"]
    X = d["X"]
    y = torch.tensor(d["y"], device=DEV)
    hs = util.HostStream(X.contiguous(), chunk_rows=max(1, X.shape[0] // 3), device=DEV)

    def make():
        Bn = [torch.tensor(a, device=DEV).requires_grad_(True) for a in d["Bcp_n0_list"]]
        Bc = [torch.tensor(a, device=DEV).requires_grad_(True) for a in d["Bcp_c0_list"]]
        return SpecCP(X.shape, (X.shape[0], m["n_out"]), rank_normal=m["rank_normal"],
                      rank_spectral=m["rank_spectral"], non_negative=m["non_negative"], Bcp_init=(Bn, Bc),
                      n_complex_dim=m["n_complex_dim"], device=DEV, softplus_kwargs=m["softplus_kwargs"])

    m10 = make()
    m10.fit_Adam(hs, y, lambda_L2=m["lambda_L2"], max_iter=min(10, m["max_iter"]), tol=m["tol"],
                 patience=m["patience"], Adam_kwargs=m["adam_kwargs"])
    np.testing.assert_allclose(m10.loss_running, d["loss_running_10"], rtol=1e-5)
    _assert_close_factors(m10.Bcp_n, [a for a in d["Bcp_n_10_list"]])
    _assert_close_factors(m10.Bcp_c, [a for a in d["Bcp_c_10_list"]])
    model = make()
    conv = model.fit_Adam(hs, y, lambda_L2=m["lambda_L2"], max_iter=m["max_iter"], tol=m["tol"],
                          patience=m["patience"], Adam_kwargs=m["adam_kwargs"])
    assert int(conv) == int(d["converged"]) and len(model.loss_running) == len(d["loss_running"])
    np.testing.assert_allclose(model.loss_running, d["loss_running"], rtol=1e-5)
