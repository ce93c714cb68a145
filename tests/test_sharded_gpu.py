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
