"""bench.py's launcher logic on the CPU (no GPU call): `--gpus N` without a launcher starts
N ranks under torch.distributed.run as a child process; under a launcher WORLD_SIZE must
equal --gpus (a plain `bench.py --gpus 8` used to run one rank and report
n_gpus 1)."""
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def _args(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.launch_ranks(_args("--gpus", "8"), [])
    assert bench.launch_ranks(_args("--gpus", "4"), []) is None      # agrees: run in this process


def test_one_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_ranks(_args(), []) is None
    assert bench.launch_ranks(_args("--gpus", "1"), []) is None


def test_gpus_n_starts_torchrun_child(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, cwd=None):
        seen["cmd"], seen["cwd"] = cmd, cwd
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    argv = ["--gpus", "8", "--config", "3", "--global-dates", "5000"]
    assert bench.launch_ranks(_args(*argv), argv) == 7               # the child's exit code
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")


def test_mismatch_fails_before_torch_import():
    """The check runs in a fresh interpreter before anything imports torch."""
    env = dict(os.environ, WORLD_SIZE="2")
    out = subprocess.run([sys.executable, "-c",
                          "import sys, runpy; sys.argv = ['bench.py', '--gpus', '8'];"
                          "runpy.run_path('bench.py', run_name='__main__')"],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=60)
    assert out.returncode != 0 and "must agree" in out.stderr
