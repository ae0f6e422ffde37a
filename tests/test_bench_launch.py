"""bench.py --gpus N starts its own N ranks: the
launcher's decision and command, and the N-rank plumbing end to end on the CPU
(--dry-run: gloo ranks, the all-gather and max over ranks the real bench uses,
one JSON line relayed from rank 0)."""

import json
import os
import subprocess
import sys
from types import SimpleNamespace

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_check_world_decides_launch_run_or_refuse():
    import bench
    assert bench.check_world(SimpleNamespace(gpus=1), {}) == "run"
    assert bench.check_world(SimpleNamespace(gpus=8), {}) == "launch"
    assert bench.check_world(SimpleNamespace(gpus=8), {"WORLD_SIZE": "8"}) == "run"
    assert bench.check_world(SimpleNamespace(gpus=1), {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 1"):
        bench.check_world(SimpleNamespace(gpus=1), {"WORLD_SIZE": "2"})


def test_launch_command_is_torchrun_on_this_script(monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    cmd = bench.launch_command(SimpleNamespace(gpus=4), 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "7"]


def test_bench_gpus_2_dry_run_spawns_two_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["AVDB_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["records_total"] == 200
    assert abs(out["ms_per_step"] - 2.0) < 1e-9  # the max over the two ranks' times
