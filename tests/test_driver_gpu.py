"""The reference-shaped driver (copula_var.utils: factory -> adapter ->
ValueAtRiskCalcualtion) end to end on the GPU: returns + in-sample params in,
VaR out, bit-identical to the reference on every golden case (including the
patched-k MSM k=6 case the reference itself cannot run, Q8)."""
import numpy as np
import pytest

from conftest import GOLDEN_CASES, golden_kwargs, load_golden
from driver_util import inject

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _driver(z):
    from copula_var.utils.calc_var_class import ValueAtRiskCalcualtion
    from copula_var.utils.factory import ValueAtRiskCalculationFactory
    tickers, start, kw = inject(z)
    model = str(z["model"])
    copula = str(z["copula"])
    calc = ValueAtRiskCalculationFactory.create_var_calculator(copula_type=copula, estimation_type=model)
    return ValueAtRiskCalcualtion(tickers, start, int(z["n_in"]), calc, None, num_points=int(z["num_points"]),
                                  weights=z["weights"], copula_params=z["copula_params"], **kw)


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_driver_calc_var_bit_identical(case):
    z = load_golden(case)
    if str(z["model"]) == "mean_reverting" and str(z["copula"]) == "gaussian":
        pytest.skip("factory maps (mean_reverting, gaussian) to Plackett (Q17)")
    v = _driver(z)
    try:
        var = v.calc_var(**golden_kwargs(z))
        assert v.ptf_mean == float(z["ptf_mean"])
        assert v.out_sample_N == z["var"].size
    finally:
        v.close()
    assert np.array_equal(var, z["var"]), (case, float(np.max(np.abs(var - z["var"]))))


@pytest.mark.parametrize("case", ["cfg1", "q1_lowvol", "cfg2_n64"])
def test_driver_host_bisection_over_device_slabs(case):
    """bisection_algorithm / adjust_integral / compute_integral: the reference's own host
    control flow with device slabs gives the same VaR as the one-shot device solve."""
    z = load_golden(case)
    v = _driver(z)
    try:
        T = v.out_sample_N
        obj, fg, sg = 0.05, -3.0, (-3.5, -2.0)
        r0 = v.compute_integral(np.column_stack((np.full(T, -100.0), np.full(T, fg))))
        nl = np.where(r0 >= obj, sg[0], fg)
        nu = np.where(r0 < obj, sg[1], fg)
        b = np.column_stack((nl, nu))
        prev_upper = np.where(nl == sg[0], sg[0], fg)
        F = v.adjust_integral(v.compute_integral(b), r0, b, fg * np.ones(T))
        bb = np.full((T, 2), np.nan)
        bb[F > obj] = (-7.5, sg[0])
        bb[(F < obj) & (nu == fg)] = (sg[0], fg)
        bb[(F < obj) & (nu == sg[1])] = (sg[1], 0.0)
        bb[(F > obj) & (nu == sg[1])] = (fg, sg[1])
        upper_stack = ~np.isin(bb[:, 1], list(sg))
        host = v.bisection_algorithm(obj, bb, F, upper_stack, prev_upper) + v.ptf_mean
        dev = v.calc_var()
    finally:
        v.close()
    assert np.array_equal(host, z["var"])
    assert np.array_equal(dev, z["var"])


def test_copula_density_api_matches_reference_formula():
    """Adapters' copula_density (t.ppf / norm.ppf on the device) vs the oracle's
    restatement of student.py / gaussian.py / plackett.py."""
    from copula_var.utils.model_estimation.copula.gaussian_estimation import GaussianCopulaVaR
    from copula_var.utils.model_estimation.copula.plackett_estimation import PlackettCopulaVaR
    from copula_var.utils.model_estimation.copula.student_estimation import StudentCopulaVaR
    from oracle.joblib_port import _copula_scalar
    rng = np.random.default_rng(5)
    u = rng.uniform(1e-6, 1 - 1e-6, size=(400, 2))
    R = np.array([[1.0, 0.5], [0.5, 1.0]])
    # scipy's stdtrit (the oracle's t.ppf) is itself only ~1e-11 accurate
    np.testing.assert_allclose(StudentCopulaVaR.copula_density(cdf=u, nu=6.0, corr_matrix=R),
                               _copula_scalar("student", u, 6.0, R), rtol=1e-9)
    np.testing.assert_allclose(GaussianCopulaVaR.copula_density(cdf=u, corr_matrix=R),
                               _copula_scalar("gaussian", u, None, R), rtol=1e-12)
    np.testing.assert_allclose(PlackettCopulaVaR.copula_density(cdf=u, nu=3.0),
                               _copula_scalar("plackett", u, 3.0, None), rtol=1e-14)
