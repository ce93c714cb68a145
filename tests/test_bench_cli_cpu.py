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


def test_other_configs_selection_and_record(monkeypatch):
    """The default cfg-2 run attaches configs 5 / 3 / 4 as child bench runs (in flight + single
    solve); 'none', another main config or a scan argument turns them off; a failing
    child is recorded, not raised."""
    import json as _json
    assert bench.other_configs(_args("--other-configs", "none")) is None
    assert bench.other_configs(_args("--config", "5")) is None
    assert bench.other_configs(_args("--dates-per-gpu", "500")) is None
    calls = []

    class R:
        def __init__(self, rc, out, err=""):
            self.returncode, self.stdout, self.stderr = rc, out, err

    def fake_run(cmd, capture_output, text, timeout):
        calls.append(cmd)
        cn = int(cmd[cmd.index("--config") + 1])
        if cn == 4:
            return R(1, "", "boom\n")
        line = {"value": 2.0e7 * cn, "unit": "VaR-dates/s", "ms_per_step": 0.2, "steps": 20, "var_checksum": -1.0,
                "single_solve": {"value": 1.0e7 * cn},
                "config": {"workload": f"cfg{cn}", "strategy": "compact", "global_dates": 5000, "inflight": 3},
                "roofline": {"avg_launch_us": 180.0, "frac": 0.14}, "e2e": {"value": 9.9e6} if cn == 5 else None}
        return R(0, "noise\n" + _json.dumps(line) + "\n")

    monkeypatch.setattr(subprocess, "run", fake_run)
    res = bench.other_configs(_args())
    assert set(res) == {"cfg5", "cfg3", "cfg4"}
    assert res["cfg5"]["single_solve"] == 5.0e7 and res["cfg5"]["e2e"] == 9.9e6 and res["cfg5"]["fp64_frac"] == 0.14
    assert res["cfg3"]["e2e"] is None
    assert "error" in res["cfg4"]
    assert all("--other-configs" in c and c[c.index("--other-configs") + 1] == "none" for c in calls)
    assert res["cfg5"]["in_flight"] == 1.0e8
    assert all("--inflight" not in c for c in calls)                  # the default batches in flight
