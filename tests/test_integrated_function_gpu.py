"""The adapters' integrated_function on the reference's own nested grids.

The plug-in surface keeps integrated_function: a caller that builds a nested
grid for bounds (a, b] (create_grids.py:6-240; here oracle.joblib_port.nested_grid, the
reference's node order and Delta-product matrix) and calls
adapter.integrated_function(grids, step_sizes, copula_params, integrations_params_i,
integrations_params_static, adapter.copula_density, adapter.unpack_copula_params) gets the
reference's per-combination (MSM, msm_integration_function.py:5-47) or per-node (GARCH / UKF,
garch_integration_function.py:5-52) values, erf and the copula quantiles on the GPU.  Checked on
golden dates against the oracle's restatement of the same formulas (scipy erf / quantiles,
the reference's scalar copula loop), and the sum of the values -- what multi_integral_function
returns (integration_algo.py:84) -- against the oracle's slab and the recorded
compute_integral result of the reference run."""
import numpy as np
import pytest

from conftest import golden_calls, load_golden

pytestmark = pytest.mark.gpu

# Student: the reference's t.ppf is scipy's stdtrit, only ~1e-11 accurate in places (SURVEY.md §8c;
# measured 8.8e-12 at p = 1e-7, 3.7e-13 at p = 0.3; the device t.ppf is within 7e-14 of mpmath).
# The 1e-12 comparison therefore takes the oracle's Student density at quantiles polished by two
# Newton steps on scipy's t CDF (stdtr, ~1e-16: lower tail directly, upper tail by symmetry), and
# the scipy-quantile oracle itself is held to 1e-9.
RTOL = {"gaussian": 1e-12, "plackett": 1e-12, "student": 1e-12}
RTOL_SCIPY_TPPF = 1e-9
CASES = ["cfg1", "cfg2_n64", "msm_gauss_n64", "msm_plackett_n64", "garch_student_n64", "ukf_plackett_n64",
         "cfg5_n64", "cfg4_k4_n16"]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _tppf_polished(u, nu):
    """t.ppf to ~1e-16: scipy's stdtrit, then two Newton steps on stdtr (p <= 1/2; p > 1/2 by symmetry)."""
    from scipy import special, stats
    u = np.asarray(u, dtype=np.float64)
    lo = np.where(u <= 0.5, u, 1.0 - u)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        z = stats.t.ppf(lo, nu)
        for _ in range(2):
            step = (special.stdtr(nu, z) - lo) / stats.t.pdf(z, nu)
            z = np.where(np.isfinite(z) & np.isfinite(step), z - step, z)
    return np.where(u <= 0.5, z, -z)


def _student_accurate(cdf, nu, R):
    """student.py:49-174 (the _copula_scalar formulas) at polished quantiles."""
    import math
    z = _tppf_polished(cdf, nu)
    d = cdf.shape[1]
    Ri, det = np.linalg.inv(R), np.linalg.det(R)
    term1 = math.gamma((nu + d) / 2) / (math.gamma(nu / 2) * ((nu * np.pi) ** (d / 2)) * np.sqrt(det))
    g = math.gamma((nu + 1) / 2) / (np.sqrt(nu * np.pi) * math.gamma(nu / 2))
    fin = np.all(np.isfinite(z), axis=1)
    zz = np.where(np.isfinite(z), z, 0.0)
    qf = np.array([np.dot(np.dot(r.T, Ri), r) for r in zz])
    mv = np.where(fin, term1 * (1 + qf / nu) ** (-(nu + d) / 2), 0.0)
    uni = np.where(np.isfinite(z), g * (1 + (zz ** 2 / nu)) ** (-(nu + 1) / 2), 0.0)
    with np.errstate(invalid="ignore", divide="ignore"):
        return mv / np.prod(uni, axis=1)


def _expected(P, t, grids, delta, accurate=False):
    """The reference's integrand restated with scipy (oracle/joblib_port._date_task, unsummed);
    accurate: the Student density at polished quantiles."""
    from oracle.joblib_port import _copula_scalar
    from oracle.quadrature import norm_cdf, norm_pdf
    dens = (lambda cdf: _student_accurate(cdf, P.nu, P.R)) if (accurate and P.copula == "student") \
        else (lambda cdf: _copula_scalar(P.copula, cdf, P.nu, P.R))
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        if P.model == "msm":
            x = grids[:, :, None] / P.uvs[None, :, :]
            cdf = np.sum(P.fbs[t] * norm_cdf(x), axis=2)
            c = dens(cdf)
            return np.sum(c[:, None] * delta, axis=0) * P.pi[t]
        x = grids / P.sigma[t]
        c = dens(norm_cdf(x))
        return np.nan_to_num((c * np.prod(norm_pdf(x) / P.sigma[t], axis=1))[:, None]) * delta


@pytest.mark.parametrize("case", CASES)
def test_integrated_function_matches_oracle(case):
    from copula_var.utils.factory import ValueAtRiskCalculationFactory
    from oracle.joblib_port import nested_grid
    from oracle.quadrature import Problem
    z = load_golden(case)
    model, copula = str(z["model"]), str(z["copula"])
    per = (z["forecasts_by_states"], z["forecasts"]) if model == "msm" else z["sigma_forecasts"]
    P = Problem(model, copula, int(z["dim"]), z["x_values"], z["step"], z["densities"], z["combos"], z["weights"],
                z["copula_params"], per, z.get("unique_vol_states"))
    adapter = ValueAtRiskCalculationFactory.create_var_calculator(copula, model)
    if copula == "gaussian" and model == "mean_reverting":
        pytest.skip("the factory maps (mean_reverting, gaussian) to Plackett (Q17)")
    bounds, results = golden_calls(z)[0]                    # the reference's first compute_integral call
    checked = 0
    for t in range(min(P.T, 3)):
        a, b = float(bounds[t, 0]), float(bounds[t, 1])
        grids, delta = nested_grid(P, a, b)
        if grids.shape[0] == 0:
            continue
        if model == "msm":
            params_i, static = [P.fbs[t], P.pi[t]], P.uvs
        else:
            params_i, static = P.sigma[t], None
        got = adapter.integrated_function(grids=grids, step_sizes=delta, copula_params=z["copula_params"],
                                          integrations_params_i=params_i, integrations_params_static=static,
                                          copula_density=adapter.copula_density,
                                          unpack_copula_params=adapter.unpack_copula_params)
        exp = _expected(P, t, grids, delta, accurate=True)
        assert got.shape == exp.shape
        np.testing.assert_allclose(got, exp, rtol=RTOL[copula], atol=1e-300)
        if copula == "student":
            np.testing.assert_allclose(got, _expected(P, t, grids, delta), rtol=RTOL_SCIPY_TPPF, atol=1e-300)
        total = float(np.sum(got))                          # multi_integral_function's np.sum
        np.testing.assert_allclose(total, P.slab(t, a, b), rtol=1e-10, atol=1e-15)
        np.testing.assert_allclose(total, results[t], rtol=1e-10, atol=1e-15)
        checked += 1
    assert checked >= 1
