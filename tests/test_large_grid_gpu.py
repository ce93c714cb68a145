"""num_points above 512 (the reference's constructor takes any num_points,
calc_var_class.py:16, and main.py:50 suggests raising it for precision).

A 2-asset grid with 512 < n <= 1024 runs on SORTED's 1024-thread instance (engine.auto_strategy,
cvq_sorted.hip sorted_threads).  The grids are the reference's own (compute_normal_densities:
msm_estimation.py:300-328, garch_estimation.py:148-188) at n = 1024 and an odd n = 700, on the
first dates of the full-batch fixtures' per-date inputs; the VaR must equal the oracle's bit for
bit with the same iteration count, and compute_integral must match within 1e-10."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

T = 6


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _problem(cfg, n):
    from oracle import forecast as F
    from oracle.quadrature import Problem
    z = dict(np.load(os.path.join(GOLDEN, f"fullbatch_cfg{cfg}.npz"), allow_pickle=False))
    model = str(z["model"])
    x, step = F.x_grid(n, model)
    if model == "msm":
        uvs = z["unique_vol_states"]
        dens = F.msm_densities(uvs, x)
        per = (z["forecasts_by_states"][:T], z["forecasts"][:T])
        combos = z["combos"]
    else:
        uvs = None
        dens = np.ones((2, 1, n))
        per = z["sigma_forecasts"][:T]
        combos = np.zeros((1, 2))
    P = Problem(model, str(z["copula"]), 2, x, step, dens, combos, z["weights"], z["copula_params"], per, uvs)
    return z, P


@pytest.mark.parametrize("cfg,n", [(3, 1024), (2, 1024), (5, 700)])
def test_large_grid_matches_oracle(cfg, n):
    from copula_var.engine import QuadraturePlan, auto_strategy
    from oracle.quadrature import calc_var
    z, P = _problem(cfg, n)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]))
    assert auto_strategy(P.model, 2, n, P.copula, z["copula_params"]) == "sorted"
    p = QuadraturePlan(P.model, P.copula, 2, P.x, P.step, P.dens, P.combos, P.w, z["copula_params"],
                       vol_states=P.uvs if P.model == "msm" else None)
    try:
        assert p.strategy == "sorted"
        p.set_dates((P.fbs, P.pi) if P.model == "msm" else [P.sigma])
        var, it = p.calc_var(float(z["ptf_mean"]))
        b = np.column_stack((np.full(T, -100.0), np.full(T, -3.0)))
        slab = p.compute_integral(b)
        b2 = np.column_stack((np.full(T, -3.0), np.full(T, 0.5)))     # above v_cap: the SORTED sibling
        slab2 = p.compute_integral(b2)
    finally:
        p.close()
    assert it == ref_it
    assert np.array_equal(var, ref), (float(np.max(np.abs(var - ref))))
    np.testing.assert_allclose(slab, P.compute_integral(b), rtol=1e-10, atol=1e-15)
    np.testing.assert_allclose(slab2, P.compute_integral(b2), rtol=1e-10, atol=1e-15)


def test_num_points_limits():
    from copula_var.engine import QuadraturePlan
    from oracle import forecast as F
    x, step = F.x_grid(1025, "garch")
    with pytest.raises(ValueError, match="1024"):
        QuadraturePlan("garch", "plackett", 2, x, step, np.ones((2, 1, 1025)), np.zeros((1, 2)), [0.5, 0.5], [3.0])
    x, step = F.x_grid(600, "garch")
    with pytest.raises(ValueError, match="SORTED"):
        QuadraturePlan("garch", "plackett", 2, x, step, np.ones((2, 1, 600)), np.zeros((1, 2)), [0.5, 0.5], [3.0],
                       strategy="compact")
