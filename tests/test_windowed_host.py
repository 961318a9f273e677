"""util.py parity (WindowedDataset / make_WindowedDataloader / squeeze_integers, reference
util.py:15-114) and the zero-copy windowed view on the CPU; the windowed and host-streamed fits on
the GPU (gpu-marked)."""
import numpy as np
import pytest
import torch

from tensor_regression_amd import util


def test_squeeze_integers():
    # the reference's own output for its docstring example (util.py:37-61; the docstring's
    # "[3,2,3,1,0]" is not what its code returns)
    np.testing.assert_array_equal(util.squeeze_integers(np.array([7, 2, 7, 4, 1])), [5, 1, 5, 3, 0])
    # (values are shifted while the loop runs, so gaps above a shifted value can stay)
    np.testing.assert_array_equal(util.squeeze_integers(np.array([0, 2, 2, 5])), [0, 1, 1, 3])
    np.testing.assert_array_equal(util.squeeze_integers(np.array([3, 3, 1])), [2, 2, 0])


@pytest.mark.parametrize("win_range", [(-3, 4), (0, 5), (-6, 1)])
def test_windowed_view_matches_dataset(win_range):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(40, 5, 3, generator=g)
    y = torch.randn(40, generator=g)
    ds = util.WindowedDataset(X, y, list(win_range))
    Xw, yw = util.windowed_view(X, y, win_range)
    assert Xw.shape == (len(ds.usable_idx), win_range[1] - win_range[0], 5, 3)
    assert Xw.stride(0) == 15 and Xw.data_ptr() == X.data_ptr()  # no copy
    for n, idx in enumerate(ds.usable_idx.tolist()):
        xi, yi = ds[idx]
        assert torch.equal(Xw[n], xi) and torch.equal(yw[n], yi)


def test_windowed_dataloader_shapes():
    X = torch.randn(100, 8)
    y = torch.randn(100)
    dl, ds, _ = util.make_WindowedDataloader(X, y, win_range=[-5, 5], batch_size=16)
    xb, yb = next(iter(dl))
    assert tuple(xb.shape) == (16, 10, 8) and tuple(yb.shape) == (16,)
    assert dl.sample_shape == [16, 10, 8]


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
