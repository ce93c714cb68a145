"""bench.py's multi-rank path on the GPU box: two ranks (torchrun, gloo process group,
both on the box's one MI355X) run the same code as the driver's N-GPU scaling bench --
per-rank plans over contiguous date blocks, device solve_local, ONE all-gather of the
packed blocks per solve, finalize on every rank -- and must reproduce the 1-rank VaR
vector bit for bit.  Only the transport differs from the 8-GPU run
(gloo instead of RCCL, which refuses two ranks on one device)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(args, nproc, self_launch=False):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    if self_launch:                                 # bench.py starts its own ranks (no launcher)
        env.pop("WORLD_SIZE", None)
        cmd = [sys.executable, "bench.py", "--gpus", str(nproc), "--backend", "gloo"]
    elif nproc == 1:
        cmd = [sys.executable, "bench.py"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(nproc),
               "--backend", "gloo"]
    out = subprocess.run(cmd + args, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


COMMON = ["--steps", "3", "--warmup", "1", "--cpu-baseline", "0", "--e2e", "0", "--single", "0", "--inflight", "2"]


def test_two_ranks_weak_and_strong_match_one_rank():
    one = _bench(COMMON + ["--dates-per-gpu", "240"], 1)
    weak = _bench(COMMON + ["--dates-per-gpu", "120"], 2)           # 2 x 120 dates of the same series
    strong = _bench(COMMON + ["--global-dates", "240", "--single", "1"], 2)   # 240 dates split 120 / 120
    assert one["var_nan"] == 0
    for r in (weak, strong):
        assert r["n_gpus"] == 2 and r["config"]["global_dates"] == 240
        assert r["var_checksum"] == one["var_checksum"], (r["var_checksum"], one["var_checksum"])
        assert r["value"] > 0
    assert weak["scaling"] == "weak" and strong["scaling"] == "strong"
    # the one-batch step split into the ranks' local solve and the all-gather + finalize
    ss = strong["single_solve"]
    assert 0 < ss["local_solve_ms"] <= ss["ms_per_step"] * 1.5
    assert ss["allgather_finalize_ms"] >= 0.0


def test_bench_gpus_flag_launches_its_own_ranks():
    """`python3 bench.py --gpus 2` with no external launcher runs two ranks:
    n_gpus 2 and the 1-rank VaR of the same 240 dates."""
    one = _bench(COMMON + ["--dates-per-gpu", "240"], 1)
    two = _bench(COMMON + ["--config", "2", "--dates-per-gpu", "120"], 2, self_launch=True)
    assert two["n_gpus"] == 2 and two["config"]["global_dates"] == 240
    assert two["var_checksum"] == one["var_checksum"], (two["var_checksum"], one["var_checksum"])
