"""Multi-rank fit loop on CPU (gloo, world_size 2).

`tensor_regression_amd._engine.run_adam_fit` is the production fit loop: per iteration it calls
the plan's data-gradient entry point, all-reduces the packed gradient arena, then the plan's
Adam step. Here the HIP plan is replaced by `OraclePlan`, a test double with the same interface
that computes shard gradients with the oracle. The real loop then runs sample-sharded over gloo
and is compared with the unsharded run. This covers the sharding, the global normalisation, the
all-reduce placement, the device-side history and stop-flag bookkeeping, the replica
lock-step, the start-of-fit replica synchronisation (ranks initialised differently) and the
recovery from a pass that failed on the device on one rank only, all without a GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import cp_oracle
from tensor_regression_amd import _lib
from tensor_regression_amd._engine import adam_hparams, run_adam_fit


class OraclePlan:
    """Same interface as _engine.Plan, computed on the CPU with the oracle (tests only)."""

    def __init__(self, model, shapes, non_negative, has_bias, fail_at=None):
        self.model = model
        self.fail_at = fail_at  # (simulated) device failure of the local pass at this Adam step
        self.step_seen = 0
        self.recovered = []
        self.shapes = shapes
        self.non_negative = non_negative
        self.has_bias = has_bias
        self.offsets = np.cumsum([0] + [a * b for a, b in shapes]).tolist()
        self.num_params = self.offsets[-1] + (1 if has_bias else 0)
        self.num_grads = self.num_params + 2  # + data loss + device status
        self.device_str = "cpu"

    def check_status(self):
        pass

    def recover(self, where):
        self.recovered.append(where)
        self.fail_at = None

    def factors(self, arena):
        return [arena[self.offsets[f]:self.offsets[f + 1]].view(s).clone() for f, s in enumerate(self.shapes)]

    def loss_grad(self, X, target, class_weight, norm, arena, weights, grad, yhat=None, stop=None):
        if stop is not None and int(stop.item()):
            return
        Bcp = [a.clone().requires_grad_(True) for a in self.factors(arena)]
        if self.model == "linear":
            b = arena[-1:].clone().requires_grad_(True)
            yh = cp_oracle.lin_model(X, Bcp, weights, self.non_negative, b)
            data = torch.sum((yh - target) ** 2) / norm
            data.backward()
            grad[:self.offsets[-1]] = torch.cat([a.grad.reshape(-1) for a in Bcp])
            grad[self.offsets[-1]] = b.grad[0]
        else:
            S = cp_oracle.mnl_model(X, Bcp, weights, self.non_negative)
            logq = torch.log_softmax(S, dim=1)
            cw = class_weight[target]
            data = torch.sum(-cw * logq[torch.arange(X.shape[0]), target]) / norm
            data.backward()
            grad[:self.offsets[-1]] = torch.cat([a.grad.reshape(-1) for a in Bcp])
        grad[self.num_params] = data.detach()
        self.step_seen += 1
        failed = self.fail_at is not None and self.step_seen == self.fail_at
        if failed:  # what k_linear_cluster leaves behind: NaN partials + the status slot
            grad[:self.num_params + 1] = float("nan")
        grad[self.num_params + 1] = 1.0 if failed else 0.0

    def adam_step(self, arena, grad, m, v, vmax, lam, hp, step, hist, base, it, patience, tol, stop):
        if int(stop.item()):
            return
        if float(grad[self.num_params + 1]) != 0.0:  # k_update: failed pass -> stop, apply nothing
            stop[0] = _lib.TR_STOP_DEVICE_ERROR - it
            return
        nfe = self.offsets[-1]
        norms = [torch.sqrt(torch.sum(arena[self.offsets[f]:self.offsets[f + 1]] ** 2))
                 for f in range(len(self.shapes))]
        g = grad[:self.num_params].clone()
        for f, n in enumerate(norms):
            sl = slice(self.offsets[f], self.offsets[f + 1])
            g[sl] += (lam / (2 * n)) * (2 * arena[sl])
        if hp["weight_decay"]:
            g = g + hp["weight_decay"] * arena[:self.num_params]
        m.lerp_(g, 1 - hp["beta1"])
        v.mul_(hp["beta2"]).addcmul_(g, g, value=1 - hp["beta2"])
        bc1 = 1 - hp["beta1"] ** step
        bc2 = 1 - hp["beta2"] ** step
        den_src = v
        if hp["amsgrad"]:
            torch.maximum(vmax, v, out=vmax)
            den_src = vmax
        denom = den_src.sqrt() / (bc2 ** 0.5) + hp["eps"]
        arena[:self.num_params].addcdiv_(m, denom, value=-hp["lr"] / bc1)
        total = float(grad[self.num_params]) + lam * float(sum(norms))
        hist[base + it] = total
        if it > patience and tol > 0:
            h = hist[it - patience: base + it + 1].numpy()
            if np.sum(np.abs(np.diff(h))) < tol:
                stop[0] = it + 1
        _ = nfe


def _problem(model):
    g = torch.Generator().manual_seed(7)
    N, dims, R = 96, (6, 5), 3
    X = torch.randn(N, *dims, generator=g)
    if model == "linear":
        shapes = [(d, R) for d in dims]
        y = torch.randn(N, generator=g)
        cw = None
        norm = float(N)
    else:
        C = 4
        shapes = [(d, R) for d in dims] + [(C, R)]
        y = torch.randint(0, C, (N,), generator=g)
        cw = torch.rand(C, generator=g) + 0.5
        norm = float(cw[y].double().sum())
    arena0 = torch.randn(sum(a * b for a, b in shapes) + (1 if model == "linear" else 0), generator=g) * 0.3
    return X, y, cw, norm, shapes, arena0


def _fit(model, X, y, cw, norm, shapes, arena0, process_group=None, iters=25, tol=0.0, patience=5, fail_at=None):
    plan = OraclePlan(model, shapes, [False] * len(shapes), model == "linear", fail_at=fail_at)
    arena = arena0.clone()
    loss_running = []
    hp = adam_hparams({"lr": 0.02, "amsgrad": model != "linear"})
    conv, n = run_adam_fit(plan, X, y, cw, norm, arena, torch.ones(shapes[0][1]), 0.01, iters, tol, patience, hp,
                           loss_running, process_group=process_group, sync_every=7)
    return arena, loss_running, conv, plan


def _worker(rank, world, port, model, tol, out_path, variant="plain"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    X, y, cw, norm, shapes, arena0 = _problem(model)
    if variant == "seeds" and rank == 1:  # a replica initialised differently: sync_replicas takes rank 0's
        arena0 = torch.randn(arena0.shape, generator=torch.Generator().manual_seed(123))
    fail_at = 10 if (variant == "fail" and rank == 1) else None  # rank 1's 10th pass fails on the "device"
    lo, hi = [(0, 40), (40, 96)][rank]  # uneven shards
    arena, lr_, conv, plan = _fit(model, X[lo:hi].contiguous(), y[lo:hi].contiguous(), cw, norm, shapes, arena0,
                                  process_group=dist.group.WORLD, tol=tol, fail_at=fail_at)
    torch.save({"arena": arena, "loss_running": lr_, "conv": conv, "recovered": plan.recovered}, f"{out_path}.{rank}")
    dist.destroy_process_group()


def _worker_mismatch(rank, world, port, out_path):
    """Rank 1's model has other feature shapes (a genuine mismatch: a class count that differs
    between shards is resolved before the fit, CP_logistic_regression._sync_class_set): every
    rank must raise instead of hanging in the per-iteration all-reduce."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, y, cw, norm, shapes, arena0 = _problem("multinomial")
    if rank == 1:
        shapes = [(shapes[0][0] - 1, shapes[0][1])] + shapes[1:]
        X = X[:, :-1]
        arena0 = arena0[:sum(a * b for a, b in shapes)]
    try:
        _fit("multinomial", X, y, cw, norm, shapes, arena0, process_group=dist.group.WORLD, iters=3)
        res = "no error"
    except ValueError as e:
        res = "ValueError" if "disagree" in str(e) else f"other: {e}"
    with open(f"{out_path}.{rank}", "w") as f:
        f.write(res)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,tol", [("linear", 0.0), ("multinomial", 0.0), ("linear", 0.05)])
def test_sharded_fit_matches_unsharded(tmp_path, model, tol):
    torch.set_num_threads(1)
    X, y, cw, norm, shapes, arena0 = _problem(model)
    ref_arena, ref_loss, ref_conv, _ = _fit(model, X, y, cw, norm, shapes, arena0, tol=tol)
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(2, _free_port(), model, tol, out), nprocs=2, join=True)
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    # replicas in lock-step: bitwise identical on both ranks
    assert torch.equal(r0["arena"], r1["arena"])
    assert r0["loss_running"] == r1["loss_running"]
    # and equal to the unsharded fit up to fp32 reduction order
    assert len(r0["loss_running"]) == len(ref_loss)
    assert bool(r0["conv"]) == bool(ref_conv)
    np.testing.assert_allclose(r0["loss_running"], ref_loss, rtol=2e-5)
    rel = float(torch.linalg.norm(r0["arena"] - ref_arena) / torch.linalg.norm(ref_arena))
    assert rel < 1e-4, rel


@pytest.mark.parametrize("variant", ["seeds", "fail"])
def test_sharded_fit_sync_and_device_failure(tmp_path, variant):
    """seeds: rank 1 starts from other parameters -> both ranks still reproduce the unsharded fit
    from rank 0's init (one broadcast at fit start).  fail: rank 1's local pass fails on the
    device at step 10 -> the all-reduced status slot stops BOTH ranks before that step, both
    recover at the same iteration, and the fit ends exactly where the failure-free fit ends."""
    torch.set_num_threads(1)
    model = "linear"
    X, y, cw, norm, shapes, arena0 = _problem(model)
    ref_arena, ref_loss, _, _ = _fit(model, X, y, cw, norm, shapes, arena0)
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(2, _free_port(), model, 0.0, out, variant), nprocs=2, join=True)
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    assert torch.equal(r0["arena"], r1["arena"])
    assert r0["loss_running"] == r1["loss_running"]
    assert len(r0["loss_running"]) == len(ref_loss)
    np.testing.assert_allclose(r0["loss_running"], ref_loss, rtol=2e-5)
    rel = float(torch.linalg.norm(r0["arena"] - ref_arena) / torch.linalg.norm(ref_arena))
    assert rel < 1e-4, rel
    if variant == "fail":
        assert r0["recovered"] == r1["recovered"] == ["iteration 9"]
        assert all(np.isfinite(r0["loss_running"]))
    else:
        assert r0["recovered"] == r1["recovered"] == []


def test_rank_mismatch_raises_everywhere(tmp_path):
    out = str(tmp_path / "mm")
    mp.spawn(_worker_mismatch, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        with open(f"{out}.{r}") as f:
            assert f.read() == "ValueError"


# ------------------------------------------------------------------------------------------------
# host logic of the sharded multinomial fit: the global class set (multinomial…py:279-280 takes
# n_classes = len(unique(y)) from the data it is given) and collective failure of local checks
# ------------------------------------------------------------------------------------------------
def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def _labels(variant, rank):
    """rank 0 / rank 1 label shards of a 10-class problem."""
    g = torch.Generator().manual_seed(3 + rank)
    y = torch.randint(0, 10, (60,), generator=g)
    if variant == "missing_middle_top":  # rank 1 lacks classes 4 and 9
        if rank == 0:
            y[:10] = torch.arange(10)
        else:
            y[(y == 4) | (y == 9)] = 0
    elif variant == "rank0_missing":  # rank 0 (whose parameters are broadcast) lacks class 9
        if rank == 0:
            y[y == 9] = 1
        else:
            y[:10] = torch.arange(10)
    elif variant == "union_gap":  # class 5 on no rank: the reference's IndexError, on every rank
        y[y == 5] = 6
        y[:1] = 9
    elif variant == "negative":
        if rank == 1:
            y[3] = -1
    elif variant == "empty_rank":
        y = y[:0] if rank == 1 else torch.cat([torch.arange(10), y])
    return y


def _worker_classes(rank, world, port, variant, out_path):
    from tensor_regression_amd import CP_logistic_regression
    _init(rank, world, port)
    y = _labels(variant, rank)
    X = torch.zeros(y.shape[0], 4, 3)
    torch.manual_seed(11 + rank)
    m = CP_logistic_regression(X, y, rank=2)
    res = {"local_C": int(m.Bcp[-1].shape[0])}
    try:
        m._sync_class_set(dist.group.WORLD)
        res.update(ok=True, C=int(m.Bcp[-1].shape[0]), n_classes=int(m.n_classes),
                   head=m.Bcp[-1].detach()[:res["local_C"]].clone(), requires_grad=bool(m.Bcp[-1].requires_grad))
    except IndexError as e:
        res.update(ok=False, err=str(e))
    torch.save(res, f"{out_path}.{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", ["missing_middle_top", "rank0_missing", "union_gap", "negative", "empty_rank"])
def test_sharded_class_set(tmp_path, variant):
    out = str(tmp_path / "cls")
    mp.spawn(_worker_classes, args=(2, _free_port(), variant, out), nprocs=2, join=True)
    r = [torch.load(f"{out}.{k}", weights_only=True) for k in range(2)]
    if variant in ("union_gap", "negative"):
        # the error a single process on the concatenated labels raises, on every rank
        want = "Target 9 is out of bounds." if variant == "union_gap" else "Target -1 is out of bounds."
        assert [x["ok"] for x in r] == [False, False] and [x["err"] for x in r] == [want, want]
        return
    assert all(x["ok"] for x in r)
    assert [x["C"] for x in r] == [10, 10] and [x["n_classes"] for x in r] == [10, 10]
    assert all(x["requires_grad"] for x in r)
    # the locally drawn rows are kept; only the missing class rows are appended
    assert all(x["head"].shape[0] == x["local_C"] for x in r)
    if variant == "missing_middle_top":
        assert [x["local_C"] for x in r] == [10, 8]
    if variant == "empty_rank":
        assert r[1]["local_C"] == 0


def _worker_agree(rank, world, port, out_path):
    """_engine.agree: a local check that fails on rank 1 only raises on both ranks (rank 1 its own
    error, rank 0 a RuntimeError), and the group stays usable; then the production fit_Adam on a
    host without a HIP device fails the same way on every rank instead of hanging."""
    from tensor_regression_amd import CP_logistic_regression, CP_linear_regression, _engine
    _init(rank, world, port)
    res = []

    def local():
        if rank == 1:
            raise ValueError("rank-1 only")
        return 5
    try:
        res.append(("agree", _engine.agree(dist.group.WORLD, local)))
    except Exception as e:
        res.append(("agree", type(e).__name__))
    t = torch.ones(1)
    dist.all_reduce(t)
    res.append(("after", float(t)))
    y = _labels("missing_middle_top", rank)
    m = CP_logistic_regression(torch.zeros(y.shape[0], 4, 3), y, rank=2)
    try:
        m.fit_Adam(max_iter=2, weights=np.ones(10), Adam_kwargs={"lr": 0.1}, process_group=dist.group.WORLD)
        res.append(("mnl", "no error"))
    except Exception as e:
        res.append(("mnl", type(e).__name__))
    lm = CP_linear_regression((8, 4, 3), rank=2)
    try:
        lm.fit_Adam(torch.zeros(8, 4, 3), torch.zeros(8), Adam_kwargs={"lr": 0.1}, process_group=dist.group.WORLD)
        res.append(("lin", "no error"))
    except Exception as e:
        res.append(("lin", type(e).__name__))
    with open(f"{out_path}.{rank}", "w") as f:
        f.write(repr(res))
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device failure path")
def test_local_failure_raises_on_every_rank(tmp_path):
    out = str(tmp_path / "agree")
    mp.spawn(_worker_agree, args=(2, _free_port(), out), nprocs=2, join=True)
    r = [eval(open(f"{out}.{k}").read()) for k in range(2)]
    assert r[0][0] == ("agree", "RuntimeError") and r[1][0] == ("agree", "ValueError")
    assert r[0][1] == r[1][1] == ("after", 2.0)
    for k in range(2):
        assert r[k][2] == ("mnl", "HipLibraryError") and r[k][3] == ("lin", "HipLibraryError"), r[k]


def _worker_fit_start(rank, world, port, out_path):
    """_engine.fit_start: one MAX all-reduce settles a sharded fit's start — the normaliser is the
    sum of every rank's value (negative values and an empty shard included), a failure on one rank
    raises on every rank, and unequal arena sizes raise ValueError on every rank."""
    from tensor_regression_amd import _engine
    _init(rank, world, port)
    res = []
    norms = [7.0, -2.5, 0.0][:world]
    out, tot = _engine.fit_start(dist.group.WORLD, lambda: ("ok", rank), lambda o: norms[rank], lambda o: 11)
    res.append(("sum", out, tot))

    def failing():
        if rank == world - 1:
            raise KeyError("last rank only")
        return 1
    try:
        _engine.fit_start(dist.group.WORLD, failing, lambda o: 1.0, lambda o: 3)
        res.append(("fail", "no error"))
    except Exception as e:
        res.append(("fail", type(e).__name__))
    try:
        _engine.fit_start(dist.group.WORLD, lambda: 0, lambda o: 1.0, lambda o: 10 + rank)
        res.append(("size", "no error"))
    except ValueError as e:
        res.append(("size", "ValueError" if "disagree" in str(e) else str(e)))
    t = torch.ones(1)
    dist.all_reduce(t)
    res.append(("after", float(t)))
    with open(f"{out_path}.{rank}", "w") as f:
        f.write(repr(res))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_fit_start_one_collective(tmp_path, world):
    out = str(tmp_path / "fs")
    mp.spawn(_worker_fit_start, args=(world, _free_port(), out), nprocs=world, join=True)
    r = [eval(open(f"{out}.{k}").read()) for k in range(world)]
    want = sum([7.0, -2.5, 0.0][:world])
    for k in range(world):
        assert r[k][0] == ("sum", ("ok", k), want), r[k]
        assert r[k][1] == ("fail", "KeyError" if k == world - 1 else "RuntimeError"), r[k]
        assert r[k][2] == ("size", "ValueError"), r[k]
        assert r[k][3] == ("after", float(world)), r[k]
