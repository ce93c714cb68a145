"""Dispatch order of the dates (cvq_plan_set_dispatch_order): with heavy-bracket dates
dispatched first (k_date_order at cvq_set_dates) every result must stay bit-identical --
full BASELINE batches against the oracle's fixtures, COMPACT's deferred generic dates,
the sharded solve + finalize, device-resident inputs, and NaN / degenerate scales (the
order must still be a permutation: a repeated or missing date would leave a VaR unsolved)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden_kwargs, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _cargs(z):
    return (str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
            z["combos"], z["weights"], z["copula_params"])


def _plan(z, strategy, order):
    from copula_var.engine import QuadraturePlan
    p = QuadraturePlan(*_cargs(z), vol_states=z.get("unique_vol_states"), strategy=strategy)
    p.set_stream(torch.cuda.current_stream().cuda_stream)
    p.set_dispatch_order(order)
    return p


def _dates(z, sl=slice(None)):
    if str(z["model"]) == "msm":
        return (z["forecasts_by_states"][sl], z["forecasts"][sl])
    return [z["sigma_forecasts"][sl]]


@pytest.mark.parametrize("cfg,strategy", [(2, "auto"), (5, "auto"), (5, "sorted"), (3, "auto")])
def test_full_batch_heavy_first_matches_oracle(cfg, strategy):
    z = dict(np.load(os.path.join(GOLDEN, f"fullbatch_cfg{cfg}.npz"), allow_pickle=False))
    p = _plan(z, strategy, True)
    try:
        p.set_dates(_dates(z))
        var, it = p.calc_var(float(z["ptf_mean"]))
    finally:
        p.close()
    assert it == int(z["iterations"])
    assert np.array_equal(var, z["var"])


@pytest.mark.parametrize("strategy", ["compact", "sorted"])
def test_heavy_first_with_generic_dates(strategy):
    """Every third date's pi is not rank 1 (COMPACT defers them to its generic kernel)."""
    from oracle.quadrature import Problem, calc_var
    z = load_golden("cfg2_n64")
    pi = z["forecasts"].copy()
    pi[::3] *= np.random.default_rng(11).uniform(0.9, 1.1, size=pi[::3].shape)
    P = Problem(*_cargs(z), (z["forecasts_by_states"], pi), z["unique_vol_states"])
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]))
    p = _plan(z, strategy, True)
    try:
        for _ in range(2):                                 # plan reuse: deferral reset under the order
            p.set_dates((z["forecasts_by_states"], pi))
            var, it = p.calc_var(float(z["ptf_mean"]))
            assert it == ref_it
            assert np.array_equal(var, ref)
    finally:
        p.close()


@pytest.mark.parametrize("case,ranks,strategy", [("cfg2_n64", 3, "compact"), ("cfg2_n64", 2, "sorted"),
                                                 ("cfg1", 2, "sorted")])
def test_heavy_first_sharded(case, ranks, strategy):
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
            p = _plan(z, strategy, True)
            plans.append(p)
            p.set_dates(_dates(z, slice(lo, hi)))
            p.solve_local(args, hdr_all[2 * r: 2 * r + 2].data_ptr(), snaps_all[r * per: r * per + hi - lo].data_ptr())
        var = torch.empty(T, dtype=torch.float64, device=dev)
        plans[0].solve_finalize(args, hdr_all.data_ptr(), ranks, snaps_all.data_ptr(), per, T, var.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(var.cpu().numpy(), z["var"])
    finally:
        for p in plans:
            p.close()


@pytest.mark.parametrize("order", [False, True])
@pytest.mark.parametrize("case", ["cfg2_n64", "cfg5_n64", "cfg1"])
def test_heavy_first_device_inputs(case, order):
    """set_dates_device (the bench's path): the order kernel reads the caller's buffers."""
    z = load_golden(case)
    T = z["var"].size
    dev = torch.device("cuda", 0)
    msm = str(z["model"]) == "msm"
    # C order: the goldens' arrays may be Fortran-ordered, and torch keeps a copy's strides
    a = torch.tensor(np.ascontiguousarray(z["forecasts_by_states"] if msm else z["sigma_forecasts"]),
                     dtype=torch.float64, device=dev).contiguous()
    b = torch.tensor(np.ascontiguousarray(z["forecasts"]), dtype=torch.float64, device=dev).contiguous() if msm else None
    p = _plan(z, "auto", order)
    try:
        p.set_dates_device(T, a.data_ptr(), b.data_ptr() if msm else None)
        var, _ = p.calc_var(float(z["ptf_mean"]), **golden_kwargs(z))
    finally:
        p.close()
    assert np.array_equal(var, z["var"])


def test_heavy_first_degenerate_scales():
    """Extreme, zero-weight-like and NaN scales land in the first / last order buckets; the
    order must stay a permutation, so every result equals index order's bit for bit (or both
    fail the same way)."""
    z = load_golden("cfg1")
    sig = z["sigma_forecasts"].copy()
    sig[3, 0] = 1e-6
    sig[5, :] = 1e3
    sig[7, 1] = np.nan
    out = {}
    for order in (False, True):
        p = _plan(z, "sorted", order)
        try:
            p.set_dates([sig])
            out[order] = p.calc_var(float(z["ptf_mean"]))
        except Exception as e:                             # noqa: BLE001 -- compared below
            out[order] = type(e)
        finally:
            p.close()
    if isinstance(out[False], type):
        assert out[True] is out[False]
    else:
        assert out[True][1] == out[False][1]
        np.testing.assert_array_equal(out[True][0], out[False][0])
