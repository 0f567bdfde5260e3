"""bench.py's multi-rank launcher on the CPU: `--gpus N` alone starts N ranks (a child
torchrun, no exec), a rank's world size must equal --gpus on every path, and the launch-check
mode brings up a real gloo world of N ranks without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_argv_world_size():
    a1 = bench.parse(["--gpus", "1"])
    assert bench.launcher_argv(a1, [], {}) is None
    a8 = bench.parse(["--gpus", "8", "--steps", "5"])
    cmd = bench.launcher_argv(a8, ["--gpus", "8", "--steps", "5"], {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.abspath(bench.__file__)) + 1:] == ["--gpus", "8", "--steps",
                                                                    "5"]
    # already a rank (torchrun set WORLD_SIZE): run the benchmark, do not launch again
    assert bench.launcher_argv(a8, [], {"WORLD_SIZE": "8"}) is None


def test_init_dist_rejects_mismatched_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit):
        bench.init_dist(bench.parse(["--gpus", "2"]))
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit):
        bench.init_dist(bench.parse(["--gpus", "2"]))


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_alone_starts_n_ranks(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                          "--backend", "gloo", "--launch-check"], env=env, cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rep = json.loads(lines[0])
    assert rep["n_gpus"] == n and sorted(rep["ranks"]) == list(range(n))
