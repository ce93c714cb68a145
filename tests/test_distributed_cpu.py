"""Date sharding + the one-shot collective (copula_var/distributed.py) on CPU gloo ranks.

The local solve and finalize steps are the oracle's CPU restatement of the
device kernels (oracle/sharded.py); what is under test is the sharding, the
header/snapshot exchange and the global Q2/Q4 resolution: the sharded VaR must
equal the reference's batch VaR bit-for-bit, including when a shard alone would
have stopped earlier (a shard of only (-3,-2]-class dates runs
fewer local iterations).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden

K = 30


def _problem(z, sl=slice(None)):
    from oracle.quadrature import Problem
    model = str(z["model"])
    per = (z["forecasts_by_states"][sl], z["forecasts"][sl]) if model == "msm" else z["sigma_forecasts"][sl]
    return Problem(model, str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                   z["combos"], z["weights"], z["copula_params"], per, z.get("unique_vol_states"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q, batches=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from copula_var.distributed import ShardedVaR, shard
        from oracle import sharded as S
        z = load_golden(case)
        T = int(z["var"].size)
        lo, hi, per = shard(T, rank, world)
        P = _problem(z, slice(lo, hi))
        ptf = float(z["ptf_mean"])

        def local(hdr, snaps):
            it, err, nz, sn = S.local_solve(P, ptf, K)
            hdr[0] = it | (err << 32)                     # int32 iters, int32 error
            hdr[1] = nz if nz < (1 << 63) else nz - (1 << 64)
            snaps[: sn.shape[0]] = torch.from_numpy(sn)

        def finalize(blocks, var):                        # the gathered [world, block_len] blocks
            hdr_all = blocks[:, s.hdr_off: s.hdr_off + 2].contiguous().view(torch.int64)
            snaps_all = blocks[:, : per * (K + 1)].reshape(world * per, K + 1)
            h = hdr_all.numpy().reshape(-1, 2)
            headers = [(int(a) & 0xFFFFFFFF, int(a) >> 32, int(b) & ((1 << 64) - 1)) for a, b in h]
            v, _, err = S.finalize(headers, snaps_all.numpy(), T, K, ptf)
            assert not err
            var.copy_(torch.from_numpy(v))

        if batches == 1:
            s = ShardedVaR(T, K + 1, local, finalize, torch.device("cpu"))
            var = s.solve().numpy().copy()
            q.put((rank, var))
        else:
            # bench.py's in-flight batches: one process group (communicator) per batch, the
            # batches' solves interleaved in step order i % batches
            groups = [dist.new_group(list(range(world))) for _ in range(batches)]
            shs = []
            for g in groups:
                s = ShardedVaR(T, K + 1, local, finalize, torch.device("cpu"), group=g)
                shs.append(s)
            out = []
            for i in range(2 * batches):
                out.append(shs[i % batches].solve().numpy().copy())
            q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(case, world, batches=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q, batches)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_shard_blocks():
    from copula_var.distributed import shard
    assert [shard(10, r, 4) for r in range(4)] == [(0, 3, 3), (3, 6, 3), (6, 9, 3), (9, 10, 3)]
    assert shard(3, 3, 4) == (3, 3, 1)
    with pytest.raises(ValueError):
        shard(10, 4, 4)


def test_single_shard_decomposition_matches_golden():
    from oracle import sharded as S
    z = load_golden("cfg1")
    P = _problem(z)
    it, err, nz, sn = S.local_solve(P, float(z["ptf_mean"]), K)
    var, kstop, e = S.finalize([(it, err, nz)], sn, P.T, K, float(z["ptf_mean"]))
    assert not e and kstop == int(z["n_calls"]) - 2
    assert np.array_equal(var, z["var"])


@pytest.mark.parametrize("case", ["cfg1", "q1_lowvol"])
def test_gloo_world2_sharded_var_is_bit_identical(case):
    z = load_golden(case)
    out = _run(case, 2)
    for r, var in out.items():
        assert np.array_equal(var, z["var"]), (case, r, np.max(np.abs(var - z["var"])))


def test_gloo_world3_uneven_blocks():
    """T = 10 over 3 ranks (blocks of 4, 4, 2): the last block is padded and
    finalize ignores the padding rows."""
    z = load_golden("msm_gauss_n64")
    assert z["var"].size % 3 != 0
    out = _run("msm_gauss_n64", 3)
    for var in out.values():
        assert np.array_equal(var, z["var"])


def test_gloo_world2_three_batches_own_groups():
    """Three in-flight batches (bench.py --inflight 3), each with its own process group, their
    all-gathers interleaved: every solve on every rank is bit-identical to the reference."""
    z = load_golden("cfg1")
    out = _run("cfg1", 2, batches=3)
    for r, vs in out.items():
        assert len(vs) == 6
        for var in vs:
            assert np.array_equal(var, z["var"])
