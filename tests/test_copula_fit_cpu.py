"""Copula IFM fits (copula_var/optim/copula_fit.py) on the CPU: the product's vectorised
objectives, driven by scipy's quantiles, against the oracle's scalar-loop restatement
of copulas/{student,gaussian,plackett}/opti.py (oracle/copula_fit.py), and the
two-stage optimisers on seeded samples.

Parity unpinned against reference fits: the bars here are the oracle
objectives (1e-12 relative: summation order only) and recovery of the generating
parameters."""
import numpy as np
import pytest
from scipy.optimize import minimize
from scipy.stats import norm, t


def _tppf(u, nu):
    return t.ppf(u, nu)


@pytest.fixture(scope="module")
def sample2():
    from oracle.copula_fit import student_sample
    return student_sample(400, 2, 5.0, 0.5, seed=31)


@pytest.fixture(scope="module")
def sample3():
    from oracle.copula_fit import student_sample
    return student_sample(200, 3, 5.0, 0.4, seed=32)


@pytest.mark.parametrize("row", [[4.0, 0.3], [7.5, 0.6], [12.0, -0.2], [2.2, 0.95], [5.0, 1.0], [5.0, -1.2]])
def test_student_nll_matches_oracle(sample2, row):
    from oracle.copula_fit import student_nll
    from copula_var.optim.copula_fit import StudentCopulaOptimizer
    u, d = sample2
    opt = StudentCopulaOptimizer(u, d, tppf=_tppf)
    got, want = opt.negative_log_likelihood(np.array(row)), student_nll(u, d, row)
    if row[1] >= 1.0 or row[1] <= -1.0:
        assert got == want == 1e10                                  # opti.py:44-52
    else:
        np.testing.assert_allclose(got, want, rtol=1e-12)


def test_student_nll_3d_and_edges(sample3):
    from oracle.copula_fit import student_nll
    from copula_var.optim.copula_fit import StudentCopulaOptimizer
    u, d = sample3
    u = u.copy()
    u[3, 1] = 1.0                                                   # t.ppf = inf -> pdf 0/0 -> NaN (student.py:133-141)
    opt = StudentCopulaOptimizer(u, d, tppf=_tppf)
    for row in ([6.0, 0.4, 0.3, 0.5], [3.5, 0.1, -0.2, 0.2]):
        got, want = opt.negative_log_likelihood(np.array(row)), student_nll(u, d, row)
        assert np.isnan(got) and np.isnan(want)
    opt = StudentCopulaOptimizer(sample3[0], d, tppf=_tppf)
    for row in ([6.0, 0.4, 0.3, 0.5], [3.5, 0.1, -0.2, 0.2]):
        np.testing.assert_allclose(opt.negative_log_likelihood(np.array(row)), student_nll(sample3[0], d, row),
                                   rtol=1e-12)
    assert opt.construct_correlation_matrix([0.4, 0.3, 0.5])[2, 1] == 0.5
    with pytest.raises(ValueError):
        StudentCopulaOptimizer(u, d[:-1], tppf=_tppf)


def test_student_optimizer_two_stage(sample2):
    from oracle.copula_fit import student_nll
    from copula_var.optim.copula_fit import Optimizer
    u, d = sample2
    opt = Optimizer(u, d, nu_values=np.array([3.0, 8.0]), tppf=_tppf)
    res = opt.optimize()
    nu, rho = res["nu"][0], res["corr_matrix"][0, 1]
    assert 2.01 <= nu <= 50 and 2.5 < nu < 12.0 and 0.4 < rho < 0.6     # generated with nu 5, rho 0.5 (N = 400)
    np.testing.assert_allclose(res["nll"], student_nll(u, d, res["optimized_params"]), rtol=1e-12)
    assert res["optimized_params"].shape == (2,) and opt.launches > 0
    # the nu stage only moves nu: the correlations are the best of the sweep
    sweep = [minimize(lambda c: student_nll(u, d, np.hstack(([v], c))), x0=[0.5], method="L-BFGS-B",
                      bounds=[(-0.99, 0.99)], tol=1e-9).x for v in (3.0, 8.0)]
    assert min(abs(res["optimized_params"][1] - s[0]) for s in sweep) < 1e-5


def test_student_optimizer_all_nan_objective_raises(sample2):
    """A marginal at exactly 1 gives t.ppf = inf and a NaN objective for every nu; the
    reference then fails on best_corr_params None -- here a ValueError says why."""
    from copula_var.optim.copula_fit import Optimizer
    u, d = sample2
    u = u.copy()
    u[0, 0] = 1.0
    with pytest.raises(ValueError, match="NaN for every nu"):
        Optimizer(u, d, nu_values=np.array([4.0]), tppf=_tppf).optimize()


@pytest.mark.parametrize("rho", [0.2, 0.7, -0.5, 0.99, 1.0])
def test_gaussian_nll_matches_oracle(sample2, rho):
    from oracle.copula_fit import gaussian_nll
    from copula_var.optim.copula_fit import GaussianCopulaOptimizer
    u, d = sample2
    opt = GaussianCopulaOptimizer(u, d, ndtri=norm.ppf)
    np.testing.assert_allclose(opt.negative_log_likelihood([rho]), gaussian_nll(u, d, [rho]), rtol=1e-12)


def test_gaussian_optimizer(sample2):
    from oracle.copula_fit import gaussian_nll
    from copula_var.optim.copula_fit import GaussianCopulaOptimizer
    u, d = sample2
    opt = GaussianCopulaOptimizer(u, d, ndtri=norm.ppf)
    res = opt.optimize()
    ref = minimize(lambda c: gaussian_nll(u, d, c), x0=[0.5], method="L-BFGS-B", bounds=[(-0.99, 0.99)], tol=1e-9)
    np.testing.assert_allclose(res["optimized_params"], ref.x, rtol=1e-6)
    np.testing.assert_allclose(res["nll"], ref.fun, rtol=1e-12)
    assert opt.launches == 1                                        # quantiles computed once


@pytest.mark.parametrize("theta", [2.0, 7.0, 0.3, 1.0])
def test_plackett_nll_matches_oracle(sample2, theta):
    from oracle.copula_fit import plackett_nll
    from copula_var.optim.copula_fit import PlackettCopulaOptimizer
    u, d = sample2
    opt = PlackettCopulaOptimizer(u, d)
    np.testing.assert_allclose(opt.negative_log_likelihood(np.array([theta])), plackett_nll(u, d, [theta]),
                               rtol=1e-12)


def test_plackett_optimizer(sample2):
    from oracle.copula_fit import plackett_nll
    from copula_var.optim.copula_fit import PlackettCopulaOptimizer
    u, d = sample2
    res = PlackettCopulaOptimizer(u, d).optimize(theta_range=np.array([0.5, 5.0]))
    best = min((minimize(lambda th: plackett_nll(u, d, th), x0=[s], method="L-BFGS-B", bounds=[(0.1, None)],
                         tol=1e-9) for s in (0.5, 5.0)), key=lambda r: r.fun)
    np.testing.assert_allclose(res["theta"], best.x[0], rtol=1e-6)
    np.testing.assert_allclose(res["nll"], best.fun, rtol=1e-12)
    assert res["theta"] >= 0.1                 # (the Q11 density is not Plackett's: no sign check on theta - 1)
    with pytest.raises(ValueError):
        PlackettCopulaOptimizer(np.zeros((4, 3)) + 0.5, np.ones((4, 3)))
