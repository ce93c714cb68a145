"""Q4 zero-interval KAT on the device: F passes exactly through 0.0 after a
negative Q1 offset inside the solve kernels' tails (tests/q4_zero_case.py); every strategy
must break where the oracle does (calc_var_class.py:293) -- same VaR, same iteration count."""
import numpy as np
import pytest

from q4_zero_case import CASES, build

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


@pytest.mark.parametrize("strategy", ["compact", "sorted", "sweep", "direct", "prefix"])
@pytest.mark.parametrize("l22", sorted(CASES))
def test_zero_crossing_after_negative_offset(l22, strategy):
    from copula_var.engine import QuadraturePlan
    z = build(l22)
    var_ref, it_ref = CASES[l22]
    p = QuadraturePlan(z["model"], z["copula"], 2, z["x_values"], z["step"], z["densities"], z["combos"],
                       z["weights"], z["copula_params"], vol_states=z["unique_vol_states"], strategy=strategy)
    try:
        p.set_dates((z["forecasts_by_states"], z["forecasts"]))
        var, it = p.calc_var(z["ptf_mean"])
    finally:
        p.close()
    assert it == it_ref, (strategy, it, it_ref)
    np.testing.assert_array_equal(var, np.full(var.shape, var_ref))
