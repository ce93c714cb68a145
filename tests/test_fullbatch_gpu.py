"""Full BASELINE batches against the pinned oracle.

calc_var couples every date of a batch: the bisection runs max-over-dates iterations
(Q2, calc_var_class.py:278) and stops every date at the first all-zero iteration (Q4,
:293).  tests/golden/fullbatch_cfg{2,5,3}.npz hold the oracle's calc_var over the whole
1000- / 5000-date batch of configs 2, 5 and 3, fullbatch_cfg4.npz over the first 250 of cfg 4's
2000 dates (3 assets, 128^3, MSM k = 6; inputs from the oracle's host forecast stage;
tests/golden/gen_fullbatch.py).  Here the HIP solve of the same full batch must
give the same VaR vector bit for bit and the same global iteration count -- on one plan,
and split into 2 and 4 contiguous date blocks (plans) joined by the packed finalize
(cvq_solve_finalize_packed, the single all-gather's layout).  The strategy
is auto (COMPACT for cfg 2 / 5, SORTED for cfg 3 / 4); cfg 5 also runs SORTED."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

CASES = [(2, "auto"), (5, "auto"), (5, "sorted"), (3, "auto"), (4, "auto")]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _load(cfg):
    path = os.path.join(GOLDEN, f"fullbatch_cfg{cfg}.npz")
    return dict(np.load(path, allow_pickle=False))


def _plan(z, sl, strategy):
    from copula_var.engine import QuadraturePlan
    model = str(z["model"])
    p = QuadraturePlan(model, str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=z.get("unique_vol_states"),
                       strategy=strategy)
    p.set_stream(torch.cuda.current_stream().cuda_stream)
    if model == "msm":
        p.set_dates((z["forecasts_by_states"][sl], z["forecasts"][sl]))
    else:
        p.set_dates([z["sigma_forecasts"][sl]])
    return p


@pytest.mark.parametrize("cfg,strategy", CASES)
def test_full_batch_one_plan(cfg, strategy):
    z = _load(cfg)
    T = int(z["T"])
    p = _plan(z, slice(0, T), strategy)
    try:
        var, it = p.calc_var(float(z["ptf_mean"]))
    finally:
        p.close()
    assert not bool(z["broke"]) and int(np.isnan(z["var"]).sum()) == 0
    assert it == int(z["iterations"]), (it, int(z["iterations"]))
    assert np.array_equal(var, z["var"]), (cfg, int((var != z["var"]).sum()), float(np.max(np.abs(var - z["var"]))))


@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("cfg,strategy", CASES)
def test_full_batch_split_packed(cfg, strategy, ranks):
    from copula_var import engine
    from copula_var.distributed import shard
    from copula_var.engine import QuadraturePlan
    z = _load(cfg)
    T = int(z["T"])
    args = engine.solve_args(float(z["ptf_mean"]))
    per = shard(T, 0, ranks)[2]
    ln, off = QuadraturePlan.packed_block_len(args, per)
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
        for p in (plans[0], plans[-1]):
            var = torch.empty(T, dtype=torch.float64, device="cuda")
            p.solve_finalize_packed(args, blocks.data_ptr(), ranks, per, T, var.data_ptr())
            assert p.solve_status() == int(z["iterations"])
            got = var.cpu().numpy()
            assert np.array_equal(got, z["var"]), (cfg, ranks, int((got != z["var"]).sum()))
    finally:
        for p in plans:
            p.close()
