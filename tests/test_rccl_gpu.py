"""The RCCL branch of the multi-GPU path, on the box's one MI355X.

The driver's 8-GPU scaling run takes init_process_group("nccl", device_id=...) (bench.py) and
distributed._gather's all_gather_into_tensor branch; the gloo tests never do.  A fresh child
process (tests/rccl_child.py) initialises a one-rank NCCL group on cuda:0 and runs the full
cfg 2 batch through device_sharded_var -- local solve, the all-gather over RCCL, the packed
finalize.  The VaR must equal tests/golden/fullbatch_cfg2.npz (the pinned oracle over the whole
batch) bit for bit, with the same global iteration count (Q2)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_nccl_world1_full_batch_matches_oracle():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_child.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"child exit {r.returncode}: {r.stderr[-2000:]}"
    out = json.loads(lines[-1])
    assert out["backend"] == "nccl", out
    assert out["gather_ok"], out
    assert out["var_equal"] and out["iterations_equal"], out
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
