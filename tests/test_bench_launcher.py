"""bench.py --gpus N (CPU, no GPU needed): the run either measures N ranks or fails with a
non-zero exit code and no JSON line — it never prints n_gpus different from --gpus.

  * --gpus 2 with fewer than 2 visible devices: exit 2 before any rank starts;
  * --gpus 2 under a launcher that started a different WORLD_SIZE: exit 2;
  * the self-launch path (no launcher): N child ranks with torchrun's environment; one failing
    rank fails the whole run and rank 0's stdout is not passed through.
"""
import io
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(HERE, "bench.py")


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=300)


def test_gpus_beyond_visible_devices_fails_cleanly():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two devices visible: the launch would measure")
    r = _run(["--gpus", "2", "--no-cpu-baseline"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""
    assert "visible" in r.stderr


def test_gpus_must_match_launcher_world_size():
    r = _run(["--gpus", "2", "--no-cpu-baseline"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and r.stdout.strip() == ""
    assert "WORLD_SIZE=1" in r.stderr


def test_self_launch_propagates_a_failing_rank(monkeypatch):
    """launch_ranks with two 'visible' devices on a machine without a GPU: both children start
    with RANK / LOCAL_RANK / WORLD_SIZE = 2 / MASTER_ADDR 127.0.0.1 and fail at their device
    setup; the parent returns non-zero and writes nothing."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("needs a machine without a GPU (the children would measure)")
    sys.path.insert(0, HERE)
    import bench
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = io.StringIO()
    rc = bench.launch_ranks(2, ["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], out)
    assert rc != 0
    assert out.getvalue() == ""


def _bench():
    sys.path.insert(0, HERE)
    import bench
    return bench


def test_shard_rows_cover_the_total():
    bench = _bench()
    for total, world in ((131072, 8), (65536, 3), (32768, 8), (10, 4), (131072, 1)):
        spans = [bench.shard_rows(total, world, r) for r in range(world)]
        assert spans[0][0] == 0
        assert sum(n for _, n in spans) == total
        for (a0, n0), (a1, _) in zip(spans, spans[1:]):
            assert a0 + n0 == a1
        assert max(n for _, n in spans) - min(n for _, n in spans) <= 1


def test_two_rank_line_schema():
    """The N > 1 block of bench.py's JSON line from two stub ranks' numbers: what the driver's
    scaling run needs to read off the line itself."""
    import json
    bench = _bench()
    blk = bench.rank_summary(2, [65536, 65536], [0.0262, 0.0265], [1.262, 1.270], 20, 2,
                             [(0.031, 12352), (0.029, 12352), (0.035, 12352)], 12352, "weak")
    json.dumps(blk)  # serialisable
    assert blk["rccl_ranks"] == 2 and blk["world_size"] == 2 and blk["scaling"] == "weak"
    assert blk["rows_per_rank"] == [65536, 65536]
    assert abs(blk["allreduce_us_per_step"] - 31.0) < 1e-9 and blk["allreduce_samples"] == 3
    assert blk["allreduce_bytes"] == 12352
    assert blk["dominant_kernel_ms_min"] == 1.262 and blk["dominant_kernel_ms_max"] == 1.270
    assert len(blk["per_rank_samples_per_s"]) == 2
    assert abs(blk["per_rank_samples_per_s"][1] - 65536 * 20 / 0.0265) < 1e-6
    assert abs(blk["per_rank_ms_per_step"][0] - 1.31) < 1e-9
    nothing = bench.rank_summary(2, [8, 8], [1.0, 1.0], [0.1, 0.1], 1, None, [], 64, "strong")
    assert nothing["allreduce_us_per_step"] is None and nothing["allreduce_bytes"] == 64


def test_launch_timeout_ends_a_hung_run(monkeypatch):
    """A rank that never finishes (and ignores SIGTERM) cannot hang the self-launched run: past
    --launch-timeout the parent terminates, then kills, the ranks and fails with no JSON line."""
    import time
    import torch
    bench = _bench()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    stub = [sys.executable, "-c",
            "import signal, time; signal.signal(signal.SIGTERM, signal.SIG_IGN); print('{}', flush=True); "
            "time.sleep(600)"]
    out = io.StringIO()
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, [], out, timeout=1.0, cmd=stub, grace=1.0)
    assert rc != 0
    assert out.getvalue() == ""
    assert time.monotonic() - t0 < 30
