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
