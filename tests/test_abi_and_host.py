"""CPU-side checks: the C-ABI library loads and exports every symbol the header declares, its
argument validation works without a GPU, and the host-side Python logic (Adam kwargs resolution,
softplus kwargs, quirk-compatible errors, the numpy pairwise-sum order restated in k_converge)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tensor_regression_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(tr_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_header_symbol():
    from tensor_regression_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(syms)
    assert lib.tr_abi_version() == _lib.TR_ABI_VERSION


def test_argument_validation_without_gpu():
    from tensor_regression_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    dims = (ctypes.c_int64 * 2)(8, 4)
    nn = (ctypes.c_int32 * 3)(0, 0, 0)
    # invalid arguments are rejected before any device call
    assert lib.tr_plan_create(ctypes.byref(h), 0, 0, 0, dims, 1, 2, 10, nn, 50.0, 1.0) == -1
    assert b"factors" in lib.tr_last_error()
    assert lib.tr_plan_create(ctypes.byref(h), 0, 0, 2, dims, 1, 0, 10, nn, 50.0, 1.0) == -1
    assert lib.tr_plan_create(ctypes.byref(h), 0, 0, 2, dims, 1, 1025, 10, nn, 50.0, 1.0) == -1  # rank > 1024
    assert lib.tr_plan_create(ctypes.byref(h), 0, 1, 2, dims, 0, 2, 10, nn, 50.0, 1.0) == -1  # no classes
    assert lib.tr_plan_create(ctypes.byref(h), 0, 7, 2, dims, 1, 2, 10, nn, 50.0, 1.0) == -1
    assert lib.tr_loss_grad(None, None, 0, None, None, 1.0, None, None, None, None, None, None) == -1
    assert lib.tr_adam_step(None, None, None, None, None, None, 0.0, 0.0, 0.9, 0.999, 1e-8, 0.0, 0, 1, None,
                            0, 0, 0, 0.0, None, None) == -1
    import torch
    if not torch.cuda.is_available():
        # a well-formed plan needs a device: the failure is reported, not hidden
        rc = lib.tr_plan_create(ctypes.byref(h), 0, 0, 2, dims, 1, 2, 10, nn, 50.0, 1.0)
        assert rc > 0 and lib.tr_last_error()


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle."""
    pkg = os.path.join(ROOT, "tensor_regression_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.sub(r"#.*", "", src).replace('"""', ""), f


def test_adam_kwargs_resolution():
    from tensor_regression_amd._engine import adam_hparams
    with pytest.raises(TypeError):
        adam_hparams(None)  # reference quirk Q1
    hp = adam_hparams({"lr": 0.01})
    assert hp == dict(lr=0.01, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, amsgrad=False)
    hp = adam_hparams({"lr": 0.02, "betas": (0.8, 0.99), "eps": 1e-6, "weight_decay": 0.1, "amsgrad": True})
    assert hp["beta1"] == 0.8 and hp["amsgrad"] is True and hp["weight_decay"] == 0.1
    with pytest.raises(TypeError):
        adam_hparams({"lr": 0.1, "bogus": 1})
    with pytest.raises(ValueError):
        adam_hparams({"lr": -1})
    with pytest.raises(NotImplementedError):
        adam_hparams({"lr": 0.1, "maximize": True})


def test_softplus_kwargs():
    from tensor_regression_amd._engine import softplus_params
    assert softplus_params(None) == (50.0, 1.0)
    assert softplus_params({"beta": 5}) == (5.0, 20.0)


def _pairwise(a):
    """numpy's DOUBLE_pairwise_sum order, as restated in k_converge (np_pairwise_sum_absdiff)."""
    n = len(a)
    if n < 8:
        res = -0.0
        for x in a:
            res += x
        return res
    if n <= 128:
        r = list(a[:8])
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pairwise(a[:n2]) + _pairwise(a[n2:])


@pytest.mark.parametrize("seed", range(5))
def test_plateau_sum_order_matches_numpy(seed):
    rng = np.random.default_rng(seed)
    for n in list(range(1, 40)) + [127, 128, 129, 300, 1000, 4097]:
        h = rng.standard_normal(n + 1) * 10 ** rng.uniform(-6, 2)
        d = np.abs(np.diff(h))
        assert _pairwise(list(d)) == np.sum(d)


def test_model_constructors_cpu_only():
    """Construction and init (RNG-identical to the reference) need no GPU."""
    import torch
    from tensor_regression_amd import CP_linear_regression, CP_logistic_regression
    torch.manual_seed(0)
    m = CP_linear_regression((10, 6, 4), rank=3, non_negative=True)
    assert [tuple(a.shape) for a in m.Bcp] == [(6, 3), (4, 3)] and m.non_negative == [True] * 3
    assert all(a.requires_grad for a in m.Bcp) and m.bias.requires_grad
    X = np.random.default_rng(0).standard_normal((20, 5, 3)).astype(np.float32)
    y = np.arange(20) % 4
    mm = CP_logistic_regression(X, y, rank=2)
    assert mm.n_classes == 4 and [tuple(a.shape) for a in mm.Bcp] == [(5, 2), (3, 2), (4, 2)]
    with pytest.raises(TypeError):
        m.fit_Adam(torch.zeros(10, 6, 4), torch.zeros(10))


def test_spectral_plan_validation_without_gpu():
    from tensor_regression_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    nn = (ctypes.c_int32 * 3)(0, 0, 0)
    # rank_normal + rank_spectral == 0, negative dims: argument errors
    assert lib.tr_plan_create_spectral(ctypes.byref(h), 0, 8, 5, 2, 0, 0, 2, 10, nn, 50.0, 1.0) == -1
    assert lib.tr_plan_create_spectral(ctypes.byref(h), 0, 0, 5, 2, 1, 1, 2, 10, nn, 50.0, 1.0) == -1
    # outside both spectral paths: K = 8 + 100*3 > 256; one sample's epilogue beyond LDS (D = 5000)
    assert lib.tr_plan_create_spectral(ctypes.byref(h), 0, 8, 5, 2, 8, 100, 3, 10, nn, 50.0, 1.0) == -2
    assert lib.tr_plan_create_spectral(ctypes.byref(h), 0, 8, 5000, 2, 4, 4, 2, 10, nn, 50.0, 1.0) == -2
    assert b"LDS" in lib.tr_last_error()


@pytest.mark.parametrize("name", ["spec_basic", "spec_nonneg_amsgrad_wd", "spec_cc1_softplus", "spec_rn0"])
def test_spectral_constructor_matches_reference_init(name):
    """CP_linear_regression.__init__ (spectral…py:425-539) draws the same factors for the same seed."""
    import json
    import torch
    from tensor_regression_amd.spectral_tensor_regression import CP_linear_regression
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz")))
    m = json.loads(str(d["meta"]))
    torch.manual_seed(m["seed"])
    X_shape = (len(d["y"]),) + tuple(m["shape"][1:])
    model = CP_linear_regression(X_shape, (len(d["y"]), m["n_out"]), rank_normal=m["rank_normal"],
                                 rank_spectral=m["rank_spectral"], non_negative=m["non_negative"],
                                 n_complex_dim=m["n_complex_dim"], softplus_kwargs=m["softplus_kwargs"])
    got_n = np.concatenate([a.detach().numpy().reshape(-1) for a in model.Bcp_n])
    got_c = np.concatenate([a.detach().numpy().reshape(-1) for a in model.Bcp_c])
    np.testing.assert_array_equal(got_n, d["Bcp_n0"])
    np.testing.assert_array_equal(got_c, d["Bcp_c0"])
    assert [tuple(a.shape) for a in model.Bcp_c] == [tuple(s) for s in m["factor_shapes_c"]]
    assert model.bias.shape == (m["n_out"],) and all(a.requires_grad for a in model.Bcp_n + model.Bcp_c)


def test_rccl_unique_id_bytes_roundtrip():
    """The gradient all-reduce's RCCL communicator is bootstrapped from an ncclUniqueId that rank 0
    broadcasts as raw bytes: ids with NUL bytes (binary) must survive the round trip whole."""
    from tensor_regression_amd import _engine
    raw = bytes([0, 7, 0, 255] * 32)
    uid = _engine.uid_from_bytes(raw)
    assert _engine.uid_to_bytes(uid) == raw
    assert _engine.uid_to_bytes(_engine.uid_from_bytes(bytearray(raw))) == raw
    with pytest.raises(ValueError):
        _engine.uid_from_bytes(raw[:127])


def test_gradient_allreduce_falls_back_to_torch_for_gloo():
    """gloo groups (the CPU multi-process tests) keep torch.distributed.all_reduce; the direct
    ncclAllReduce path is only taken for an NCCL (RCCL) group."""
    import socket
    import torch
    import torch.distributed as dist
    from tensor_regression_amd import _engine
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        ar = _engine.gradient_allreduce(dist.group.WORLD, 0)
        assert not isinstance(ar, _engine.RcclAllReduce)
        t = torch.arange(5, dtype=torch.float32)
        ar(t)
        assert torch.equal(t, torch.arange(5, dtype=torch.float32))
    finally:
        dist.destroy_process_group()


class _FakeClock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t

    def sleep(self, dt):
        self.t += 1.0  # every poll advances one "second"


class _FakeEvent:
    """completes once the fake clock reaches `at`"""

    def __init__(self, clock, at):
        self.clock, self.at = clock, at

    def query(self):
        return self.clock.t >= self.at


def test_watchdog_counts_time_without_progress():
    """A healthy but slow chunk (64 all-reduces, 10 s apart: 640 s in all) passes a 30 s
    watchdog, because every completed all-reduce restarts the clock (the bound used
    to cover the whole chunk); a stall of more than 30 s after the 5th all-reduce trips it."""
    from tensor_regression_amd._engine import wait_progress, _CollectiveTimeout, _CollectiveError
    clk = _FakeClock()
    evs = [_FakeEvent(clk, 10.0 * (k + 1)) for k in range(64)]
    wait_progress(evs, lambda: None, 30.0, clock=clk, sleep=clk.sleep)
    assert clk.t >= 640.0
    clk = _FakeClock()
    evs = [_FakeEvent(clk, 10.0 * (k + 1)) for k in range(5)] + [_FakeEvent(clk, 1e9)]
    with pytest.raises(_CollectiveTimeout, match="5 of the 6"):
        wait_progress(evs, lambda: None, 30.0, clock=clk, sleep=clk.sleep)
    assert 80.0 <= clk.t <= 82.0
    clk = _FakeClock()
    errs = iter([None, None, "remote process exited"])
    with pytest.raises(_CollectiveError, match="remote process"):
        wait_progress([_FakeEvent(clk, 1e9)], lambda: next(errs), 1e6, clock=clk, sleep=clk.sleep)


def _mnl_geometry(I, J, R, C=10):
    from tensor_regression_amd import _lib
    lib = _lib.load()
    out = (ctypes.c_int32 * 11)()
    rc = lib.tr_mnl_geometry(I, J, R, C, out, 11)
    keys = ["duo", "bsp", "waves", "wg_per_cu", "ring", "padded", "row_width", "row_blocks", "rank_cols",
            "lds_bytes", "fused_ok"]
    return rc, dict(zip(keys, list(out)))


# (I, J, R): expected (duo, bsp, waves, wg/CU, ring, padded, row width, row blocks, rank columns);
# the multinomial factored pass's envelope as DESIGN.md "Multinomial" describes it (no device needed:
# the plan may still fall back at creation when an instantiation spills)
MNL_GEOMETRY = [
    ((128, 64, 8), (1, 0, 4, 2, 2, 0, 64, 1, 8)),      # config 3: rank-block body
    ((128, 64, 3), (1, 1, 4, 2, 2, 0, 64, 1, 8)),      # rank <= 4: split body
    ((128, 64, 16), (1, 1, 4, 2, 2, 0, 64, 1, 16)),    # ranks 9..16: the 16-rank form
    ((64, 64, 8), (1, 1, 2, 4, 2, 0, 64, 1, 8)),
    ((160, 64, 8), (1, 1, 5, 1, 3, 0, 64, 1, 8)),      # ring of three at 5 / 6 waves
    ((96, 128, 12), (1, 1, 6, 1, 2, 0, 128, 1, 16)),   # (no ring of three for the 128-wide 16-rank form)
    ((100, 64, 8), (1, 1, 4, 2, 2, 1, 64, 1, 8)),      # padded rows
    ((128, 48, 8), (1, 1, 4, 2, 2, 1, 64, 1, 8)),      # padded width
    ((512, 64, 8), (1, 1, 8, 1, 2, 0, 64, 2, 8)),      # row blocks
    ((256, 128, 8), (1, 1, 8, 1, 2, 0, 128, 2, 8)),
    ((384, 64, 5), (1, 1, 6, 1, 2, 0, 64, 2, 8)),
    ((288, 128, 8), (1, 1, 6, 1, 2, 0, 128, 3, 8)),
    ((512, 48, 8), (1, 1, 8, 1, 2, 1, 64, 2, 8)),
    ((64, 32, 4), (1, 1, 2, 4, 3, 0, 32, 1, 8)),       # the 32-wide form, a ring of three
    ((256, 32, 8), (1, 1, 8, 1, 3, 0, 32, 1, 8)),
    ((192, 32, 8), (1, 1, 6, 1, 3, 0, 32, 1, 8)),
    ((100, 24, 4), (1, 1, 4, 2, 3, 1, 32, 1, 8)),      # padded rows and width
    ((64, 24, 8), (1, 1, 2, 4, 3, 1, 32, 1, 8)),
    ((128, 32, 12), (1, 1, 4, 2, 2, 1, 64, 1, 16)),    # rank > 8: the 64-wide 16-rank form
    ((512, 32, 4), (1, 1, 8, 1, 2, 1, 64, 2, 8)),      # > 256 rows: 64-wide row blocks
]
MNL_GEOMETRY_OUTSIDE = [(768, 64, 8), (300, 128, 8), (512, 128, 8), (256, 128, 12), (16, 64, 8), (64, 12, 8), (32, 20, 8), (64, 20, 8),
                        (128, 64, 17)]


@pytest.mark.parametrize("shape,want", MNL_GEOMETRY)
def test_mnl_geometry_envelope(shape, want, monkeypatch):
    for k in ("TR_MNL_DUO", "TR_DUO_SPLIT", "TR_DUO_ANYFILL"):
        monkeypatch.delenv(k, raising=False)
    rc, g = _mnl_geometry(*shape)
    assert rc == 0
    got = tuple(g[k] for k in ["duo", "bsp", "waves", "wg_per_cu", "ring", "padded", "row_width", "row_blocks",
                               "rank_cols"])
    assert got == want, g
    assert g["wg_per_cu"] * g["lds_bytes"] <= 160 * 1024, g


@pytest.mark.parametrize("shape", MNL_GEOMETRY_OUTSIDE)
def test_mnl_geometry_outside(shape, monkeypatch):
    """Outside the family: rows not whole blocks or four blocks (768, 64), (512, 128); rank > 8 with
    row blocks; a sample filling less than a third of its padded shape; J < 16; rank > 16."""
    for k in ("TR_MNL_DUO", "TR_DUO_SPLIT", "TR_DUO_ANYFILL"):
        monkeypatch.delenv(k, raising=False)
    rc, g = _mnl_geometry(*shape)
    assert rc == 0 and g["duo"] == 0, g


def test_mnl_geometry_switches(monkeypatch):
    for k in ("TR_MNL_DUO", "TR_DUO_SPLIT", "TR_DUO_ANYFILL"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("TR_DUO_SPLIT", "1")  # the split body at config 3's rank 8
    assert _mnl_geometry(128, 64, 8)[1]["bsp"] == 1
    monkeypatch.setenv("TR_DUO_SPLIT", "0")  # the rank-block body only
    assert _mnl_geometry(128, 64, 8)[1]["bsp"] == 0 and _mnl_geometry(64, 64, 8)[1]["duo"] == 0
    monkeypatch.delenv("TR_DUO_SPLIT")
    monkeypatch.setenv("TR_DUO_ANYFILL", "1")  # any fill of the padded shape (the tests' switch)
    assert _mnl_geometry(16, 64, 8)[1]["duo"] == 1
    monkeypatch.delenv("TR_DUO_ANYFILL")
    monkeypatch.setenv("TR_MNL_DUO", "0")
    assert _mnl_geometry(128, 64, 8)[1]["duo"] == 0
    from tensor_regression_amd import _lib
    lib = _lib.load()
    out = (ctypes.c_int32 * 11)()
    assert lib.tr_mnl_geometry(128, 64, 40, 10, out, 11) == -2  # rank beyond the factored kernels
    assert lib.tr_mnl_geometry(128, 64, 8, 10, None, 11) == -1
