"""The real HIP fit at world size 2 on one GPU (reference fit_Adam loops
standard_tensor_regression.py:458-470, multinomial_tensor_regression.py:453-465,
spectral_tensor_regression.py:714-741, which north_star shards over the sample axis).

Two fresh child processes (torch.multiprocessing spawn: the children, not the pytest process,
create their HIP contexts) both bind cuda:0 and form a gloo group.  gloo all-reduces and
broadcasts the device tensors themselves, so the start-of-fit replica broadcast of the device
arena, the per-iteration all-reduce of the gradient arena (with its device status slot) and the
multinomial class-set / class-weight reductions all run for real, around the production classes
and the gfx950 kernels.  Each rank fits its own sample shard:

  * linear, single-pass fused path          (k_linear_fused)
  * linear, wide rows                       (k_linear_cluster; two processes share the GPU, so
                                             its exchange may time out and the fit resume on the
                                             two-pass path — on BOTH ranks, at the same iteration;
                                             which path each rank ran is printed)
  * linear, wide rows, ranks in turns       (k_linear_cluster with each rank's gradient pass run
                                             while the other rank's queue is drained and parked at
                                             a barrier: the kernels never share the GPU in time, so
                                             the single pass must complete on both ranks)
  * multinomial, config-3 sample shape      (k_mnl_duo), model built WITHOUT Bcp_init: rank 1's
                                             shard misses the top class and a middle class and
                                             starts from another seed
  * spectral, config-5 sample shape         (k_spec_slice)

Pass: both ranks end bitwise identical, and equal to ONE process fitting the concatenated data
from the same initial point within 1e-5 (loss_running elementwise, factors normwise).
"""
import os
import socket
import warnings

import numpy as np
import pytest
import torch

from golden_util import normwise_rel

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
RTOL = 1e-5
ITERS = 20
CASES = ("linear_fused", "linear_cluster", "linear_cluster_turns", "mnl_duo", "spectral_slice")


def _data(case):
    """(X, y, split, init) on the CPU; init = the initial factors every fit starts from (None for
    the multinomial case: the models draw their own, see _make)."""
    g = torch.Generator().manual_seed(100 + CASES.index(case))
    if case == "linear_fused":
        X = torch.randn(3000, 64, 32, generator=g)
        y = torch.randn(3000, generator=g)
        init = [torch.randn(d, 6, generator=g) * 0.3 for d in (64, 32)]
        return X, y, 1300, init
    if case.startswith("linear_cluster"):
        X = torch.randn(600, 64, 64, 32, generator=g)
        y = torch.randn(600, generator=g)
        init = [torch.randn(d, 16, generator=g) * 0.3 for d in (64, 64, 32)]
        return X, y, 280, init
    if case == "mnl_duo":
        X = torch.randn(1500, 128, 64, generator=g)
        y = torch.randint(0, 10, (1500,), generator=g)
        y[:10] = torch.arange(10)
        # rank 1 (rows 700:) lacks class 9 (top) and class 4 (middle): its local class count is 8
        tail = y[700:]
        tail[(tail == 9) | (tail == 4)] = 0
        return X, y, 700, None
    X = torch.randn(600, 256, 129, generator=g)
    y = torch.randn(600, 2, generator=g)
    Bn = [torch.randn(256, 8, 1, generator=g) * 0.1, torch.randn(129, 8, 1, generator=g) * 0.1,
          torch.randn(2, 8, 1, generator=g)]
    Bc = [torch.randn(256, 8, 2, generator=g) * 0.1, torch.randn(129, 8, 1, generator=g) * 0.1,
          torch.randn(2, 8, 1, generator=g)]
    return X, y, 250, (Bn, Bc)


def _fit(case, X, y, init, seed, process_group=None):
    """Fit through the production class; returns (loss_running, factors as numpy, plan describe).
    The gradient arena of the first iteration, as the Adam step received it (after the all-reduce
    on a process group), is recorded in _FIRST_GRAD."""
    import tensor_regression_amd as tra
    from tensor_regression_amd import spectral_tensor_regression as SP
    Xd, yd = X.to(DEV), y.to(DEV)
    adam = {"lr": 0.01}
    if case.startswith("linear"):
        m = tra.CP_linear_regression(X.shape, rank=init[0].shape[1], device=DEV,
                                     Bcp_init=[a.clone().to(DEV).requires_grad_(True) for a in init], bias_init=0.1)
        m.fit_Adam(Xd, yd, lambda_L2=0.01, max_iter=ITERS, tol=0, patience=10, Adam_kwargs=adam,
                   process_group=process_group)
        facs = [a.detach().cpu().numpy() for a in m.Bcp] + [m.bias.detach().cpu().numpy()]
    elif case == "mnl_duo":
        torch.manual_seed(seed)
        m = tra.CP_logistic_regression(Xd, yd, rank=8, device=DEV)  # no Bcp_init: drawn from the local labels
        m.fit_Adam(lambda_L2=0.01, max_iter=ITERS, tol=0, patience=10, weights=np.linspace(0.5, 1.5, 10),
                   Adam_kwargs=adam, process_group=process_group)
        facs = [a.detach().cpu().numpy() for a in m.Bcp]
    else:
        Bn, Bc = init
        m = SP.CP_linear_regression(X.shape, y.shape, rank_normal=8, rank_spectral=8, n_complex_dim=1, device=DEV,
                                    Bcp_init=([a.clone().to(DEV).requires_grad_(True) for a in Bn],
                                              [a.clone().to(DEV).requires_grad_(True) for a in Bc]))
        m.fit_Adam(Xd, yd, lambda_L2=0.01, max_iter=ITERS, tol=0, patience=10, Adam_kwargs=adam,
                   process_group=process_group)
        facs = [a.detach().cpu().numpy() for a in list(m.Bcp_n) + list(m.Bcp_c)] + [m.bias.detach().cpu().numpy()]
    return list(m.loss_running), facs, m._plan.describe


_FIRST_GRAD = {}


def _record_first_grad():
    """Wrap the engine so the first iteration's gradient arena is kept: after the sharded fit's
    all-reduce (gradient_allreduce's callable), or after the local gradient without a group."""
    from tensor_regression_amd import _engine
    orig_ga, orig_lg = _engine.gradient_allreduce, _engine.loss_grad_any
    _FIRST_GRAD.clear()

    def ga(process_group, device_index):
        fn = orig_ga(process_group, device_index)

        def wrapped(g):
            fn(g)
            _FIRST_GRAD.setdefault("grad", g.detach().clone().cpu())
        _FIRST_GRAD["allreduce"] = True
        return wrapped

    def lg(plan, X, target, class_weight, norm, arena, weights, grad, **kw):
        orig_lg(plan, X, target, class_weight, norm, arena, weights, grad, **kw)
        if not _FIRST_GRAD.get("allreduce"):
            _FIRST_GRAD.setdefault("grad", grad.detach().clone().cpu())
    _engine.gradient_allreduce, _engine.loss_grad_any = ga, lg
    return lambda: (setattr(_engine, "gradient_allreduce", orig_ga), setattr(_engine, "loss_grad_any", orig_lg))


def _in_turns(fn, rank, world):
    """fn (a rank's gradient pass) run while every other rank's GPU queue is drained and the rank
    is parked at a barrier: the ranks' kernels never overlap in time."""
    import torch.distributed as dist

    def wrapped(*a, **k):
        torch.cuda.synchronize()
        for r in range(world):
            dist.barrier()
            if r == rank:
                fn(*a, **k)
                torch.cuda.synchronize()
        dist.barrier()
    return wrapped


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from tensor_regression_amd import _engine
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    res = {}
    for case in CASES:
        X, y, split, init = _data(case)
        lo, hi = (0, split) if rank == 0 else (split, X.shape[0])
        orig = _engine.loss_grad_any
        restore = _record_first_grad()
        if case.endswith("_turns"):
            _engine.loss_grad_any = _in_turns(_engine.loss_grad_any, rank, world)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            try:
                lr, facs, desc = _fit(case, X[lo:hi].contiguous(), y[lo:hi].contiguous(), init, seed=7 + 5 * rank,
                                      process_group=dist.group.WORLD)
            finally:
                restore()
                _engine.loss_grad_any = orig
        res[case] = {"loss_running": lr, "factors": [torch.from_numpy(np.ascontiguousarray(f)) for f in facs],
                     "describe": desc, "warnings": [str(x.message) for x in w], "grad0": _FIRST_GRAD["grad"]}
    torch.save(res, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def world2(tmp_path_factory):
    import torch.multiprocessing as mp
    out = str(tmp_path_factory.mktemp("world2") / "res")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    return [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]


def _single(case):
    X, y, split, init = _data(case)
    restore = _record_first_grad()
    try:
        out = _fit(case, X, y, init, seed=7)
    finally:
        restore()
    return out + (_FIRST_GRAD["grad"],)


@pytest.mark.parametrize("case", CASES)
def test_world2_fit_matches_single_process(world2, case, capsys):
    r0, r1 = world2[0][case], world2[1][case]
    paths = [("recovered on the two-pass path" if "recovered=2pass" in r["describe"] else "single pass completed")
             for r in (r0, r1)]
    with capsys.disabled():
        print(f"\n[world2 {case}] rank 0: {paths[0]}; rank 1: {paths[1]} ({r0['describe'].split(' path=')[1].split()[0]})")
    # the replicas are in lock-step: bitwise identical on both ranks
    assert r0["loss_running"] == r1["loss_running"]
    for a, b in zip(r0["factors"], r1["factors"]):
        assert torch.equal(a, b)
    # the kernel the case is about ran (the cluster pass may have recovered on the two-pass path:
    # two processes share the GPU, which is exactly what its status slot exists for)
    want = {"linear_fused": "fused-1pass", "linear_cluster": "cluster-1pass", "linear_cluster_turns": "cluster-1pass",
            "mnl_duo": " duo ", "spectral_slice": "slice-1pass"}[case]
    assert want in r0["describe"] and want in r1["describe"], (r0["describe"], r1["describe"])
    assert ("recovered=2pass" in r0["describe"]) == ("recovered=2pass" in r1["describe"])
    if case != "linear_cluster":
        # with the ranks' passes apart in time the cluster exchange has no co-tenant: it must
        # complete (no recovery, no warning) on both ranks
        assert "recovered=2pass" not in r0["describe"], r0["describe"]
        assert not r0["warnings"] and not r1["warnings"], (r0["warnings"], r1["warnings"])
    # and equal to one process fitting the concatenated shards from the same initial point
    lr, facs, _, g0 = _single(case)
    assert len(r0["loss_running"]) == len(lr) == ITERS
    # the all-reduced gradient arena of the first iteration (the data gradients, the bias entries and
    # the data-loss slot, each normalised by the GLOBAL sample count or class-weight total) equals
    # the single process's at the same point, element by element — Adam normalises each
    # coordinate's step by its own scale, so a gradient summed once too often would not show in
    # the trajectory (the multinomial ranks start from different local draws, synchronised to
    # rank 0's before the first iteration; the single process starts from seed 7 = rank 0's)
    assert torch.equal(r0["grad0"], r1["grad0"])
    a, b = r0["grad0"].double().numpy(), g0.double().numpy()
    assert a.shape == b.shape
    scale = np.abs(b).max()
    np.testing.assert_allclose(a, b, rtol=RTOL, atol=RTOL * 1e-2 * scale)
    np.testing.assert_allclose(r0["loss_running"], lr, rtol=RTOL)
    assert len(facs) == len(r0["factors"])
    for a, b in zip(r0["factors"], facs):
        assert a.shape == b.shape
        if a.numel() == 1:
            # the bias: it crosses zero during the fit (final value ~ -0.006 after 20 steps of
            # lr 0.01), and Adam normalises each coordinate's step by its own gradient scale, so
            # fp32 summation-order noise of a near-zero gradient moves it by a fraction of a step:
            # held to RTOL of the path length lr * ITERS instead of RTOL of its final value
            d = abs(float(a.reshape(-1)[0]) - float(np.asarray(b).reshape(-1)[0]))
            assert d <= RTOL * max(abs(float(np.asarray(b).reshape(-1)[0])), 0.01 * ITERS), (case, d)
            continue
        assert normwise_rel(a.numpy(), b) <= RTOL, (case, a.shape, normwise_rel(a.numpy(), b))
