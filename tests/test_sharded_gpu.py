"""The device entry points of the sharded solve (cvq_solve_local / cvq_solve_finalize)
on one GPU: R plans each hold one contiguous date block, their headers and
snapshots are concatenated exactly as the all-gather lays them out, and every
"rank" finalises the full VaR vector -- which must equal the reference's batch
VaR bit-for-bit (Q2 / Q4 are global across the blocks)."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _plan(z, sl, strategy):
    from copula_var.engine import QuadraturePlan
    model = str(z["model"])
    p = QuadraturePlan(model, str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=z.get("unique_vol_states"),
                       strategy=strategy)
    p.set_stream(torch.cuda.current_stream().cuda_stream)      # order with the torch buffers
    if model == "msm":
        p.set_dates((z["forecasts_by_states"][sl], z["forecasts"][sl]))
    else:
        p.set_dates([z["sigma_forecasts"][sl]])
    return p


@pytest.mark.parametrize("strategy", ["compact", "direct", "prefix"])
@pytest.mark.parametrize("case,ranks", [("cfg1", 2), ("cfg1", 3), ("q1_lowvol", 4), ("cfg2_n64", 3),
                                        ("cfg3_n128", 2), ("cfg5_n64", 2)])
def test_sharded_device_solve(case, ranks, strategy):
    from copula_var import engine
    from copula_var.distributed import shard
    z = load_golden(case)
    T = z["var"].size
    args = engine.solve_args(float(z["ptf_mean"]))
    stride = engine.QuadraturePlan.snap_stride(args)
    dev = torch.device("cuda", 0)
    per = shard(T, 0, ranks)[2]
    hdr_all = torch.zeros(2 * ranks, dtype=torch.int64, device=dev)
    snaps_all = torch.full((ranks * per, stride), float("nan"), dtype=torch.float64, device=dev)
    plans = []
    try:
        for r in range(ranks):
            lo, hi, _ = shard(T, r, ranks)
            if hi <= lo:
                continue
            p = _plan(z, slice(lo, hi), strategy)
            plans.append(p)
            hdr = hdr_all[2 * r: 2 * r + 2]
            snaps = snaps_all[r * per: r * per + (hi - lo)]
            p.solve_local(args, hdr.data_ptr(), snaps.data_ptr())
        for p in plans:                      # every rank finalises the whole vector
            var = torch.empty(T, dtype=torch.float64, device=dev)
            p.solve_finalize(args, hdr_all.data_ptr(), ranks, snaps_all.data_ptr(), per, T, var.data_ptr())
            torch.cuda.synchronize()
            got = var.cpu().numpy()
            assert np.array_equal(got, z["var"]), (case, ranks, float(np.nanmax(np.abs(got - z["var"]))))
    finally:
        for p in plans:
            p.close()


@pytest.mark.parametrize("strategy", ["compact", "sorted"])
def test_device_sharded_var_orders_on_torch_stream(strategy):
    """device_sharded_var binds the plan to torch's current stream itself (no explicit
    set_stream): the snapshot buffer's NaN fill, the solve and the finalize are ordered."""
    from copula_var import engine
    from copula_var.distributed import device_sharded_var
    from copula_var.engine import QuadraturePlan
    z = load_golden("cfg2_n256")
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), 2, z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=z["unique_vol_states"],
                       strategy=strategy)
    try:
        p.set_dates((z["forecasts_by_states"], z["forecasts"]))
        args = engine.solve_args(float(z["ptf_mean"]))
        s = device_sharded_var(p, args, z["var"].size, torch.device("cuda", 0))
        for _ in range(3):
            got = s.solve().cpu().numpy()
            assert np.array_equal(got, z["var"])
        assert p.solve_status() == int(z["n_calls"]) - 2
    finally:
        p.close()


@pytest.mark.parametrize("strategy", ["compact", "direct", "prefix", "sorted"])
def test_non_dyadic_guesses_device_mode(strategy):
    """Non-dyadic guesses (K carries a margin): solve_device(check=True), the sharded
    path and the host path all agree with the oracle; solve_status reports the count."""
    from copula_var import engine
    from copula_var.distributed import device_sharded_var
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden("cfg2_n64")
    kw = dict(first_guess=-2.7, second_guess=(-3.3, -2.1))
    per = (z["forecasts_by_states"], z["forecasts"])
    cargs = (str(z["model"]), str(z["copula"]), 2, z["x_values"], z["step"], z["densities"], z["combos"],
             z["weights"], z["copula_params"])
    P = Problem(*cargs, per, z["unique_vol_states"])
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]), **kw)
    p = QuadraturePlan(*cargs, vol_states=z["unique_vol_states"], strategy=strategy)
    try:
        p.set_dates(per)
        host, it = p.calc_var(float(z["ptf_mean"]), **kw)
        assert it == ref_it and np.array_equal(host, ref)
        args = engine.solve_args(float(z["ptf_mean"]), **kw)
        p.set_stream(torch.cuda.current_stream().cuda_stream)
        var = torch.empty(P.T, dtype=torch.float64, device="cuda")
        assert p.solve_device(args, var.data_ptr(), check=True) == ref_it
        assert np.array_equal(var.cpu().numpy(), ref)
        p.solve_device(args, var.data_ptr())
        assert p.solve_status() == ref_it
        assert np.array_equal(var.cpu().numpy(), ref)
        s = device_sharded_var(p, args, P.T, torch.device("cuda", 0))
        assert np.array_equal(s.solve().cpu().numpy(), ref)
    finally:
        p.close()


@pytest.mark.parametrize("strategy", ["compact", "sorted"])
@pytest.mark.parametrize("case,ranks", [("cfg1", 3), ("cfg2_n64", 2), ("cfg4_k6_n16", 2)])
def test_packed_single_gather_layout(case, ranks, strategy):
    """cvq_solve_finalize_packed: every rank's snapshots + header in ONE block, the blocks
    concatenated as one all-gather lays them out; every rank's finalize gives the batch VaR."""
    from copula_var import engine
    from copula_var.distributed import shard
    from copula_var.engine import QuadraturePlan
    z = load_golden(case)
    if strategy == "compact" and int(z["dim"]) != 2:
        pytest.skip("COMPACT is built for dim == 2")
    T = z["var"].size
    args = engine.solve_args(float(z["ptf_mean"]))
    per = shard(T, 0, ranks)[2]
    ln, off = QuadraturePlan.packed_block_len(args, per)
    assert ln % 2 == 0 and off % 2 == 0 and off >= per * QuadraturePlan.snap_stride(args)
    blocks = torch.full((ranks, ln), float("nan"), dtype=torch.float64, device="cuda")
    plans = []
    try:
        for r in range(ranks):
            lo, hi, _ = shard(T, r, ranks)
            p = _plan(z, slice(lo, hi), strategy)
            plans.append(p)
            blk = blocks[r]
            blk[off: off + 2] = 0.0
            p.solve_local(args, blk[off:].data_ptr(), blk.data_ptr())
        for p in plans:
            var = torch.empty(T, dtype=torch.float64, device="cuda")
            p.solve_finalize_packed(args, blocks.data_ptr(), ranks, per, T, var.data_ptr())
            assert p.solve_status() == int(z["n_calls"]) - 2
            assert np.array_equal(var.cpu().numpy(), z["var"])
    finally:
        for p in plans:
            p.close()
