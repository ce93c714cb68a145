"""Device likelihood kernels and the device-batched GarchOptimizer against the
reference's own results (tests/golden/gen_optim_golden.py) -- needs an MI355X.

Bars: log-likelihoods within 1e-12 relative (sequential vs numpy pairwise
summation over ~1,100 terms); the optimiser selects the same (p, q) and lands on
the same parameters within 1e-7 relative (finite-difference Hessians amplify the
1e-13 likelihood differences; Newton converges to the same point)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


@pytest.mark.parametrize("p,q", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_garch_loglik_pq_kernel(p, q):
    from copula_var import engine
    z = load_golden("optim_garch")
    sel = [i for i, (pp, qq) in enumerate(z["ll_pq"]) if (pp, qq) == (p, q)]
    rows = z["ll_rows"][sel][:, :1 + p + q]
    got = engine.garch_loglik_pq(z["returns"], p, q, rows)
    np.testing.assert_allclose(got, z["ll"][sel], rtol=1e-12)
    if (p, q) == (1, 1):                                       # the (1,1) entry point agrees
        np.testing.assert_allclose(engine.garch_loglik(z["returns"], rows), got, rtol=1e-15)


def test_garch_optimizer_on_device_matches_reference():
    from copula_var.optim.garch import GarchOptimizer
    z = load_golden("optim_garch")
    opt = GarchOptimizer(z["returns"], p_max=int(z["p_max"]), q_max=int(z["q_max"]))
    best_pq, best_params, best_nll, best_bic = opt.optimize()
    assert tuple(best_pq) == tuple(z["best_pq"])
    np.testing.assert_allclose(best_params, z["best_params"], rtol=1e-7)
    np.testing.assert_allclose(best_nll, float(z["best_nll"]), rtol=1e-10)
    np.testing.assert_allclose(best_bic, float(z["best_bic"]), rtol=1e-10)


def test_msm_loglik_kernel():
    from copula_var import engine
    z = load_golden("optim_msm_ll")
    got = engine.msm_loglik(z["returns"], int(z["k"]), z["rows"])
    np.testing.assert_allclose(got, z["ll"], rtol=1e-11)


def test_msm_optimizer_on_device_replays_the_cpu_chains():
    """Same seeded chains on the device likelihood and on the CPU oracle: the accept /
    reject path and the result agree (likelihoods agree to ~1e-13)."""
    from oracle.forecast import msm_loglik
    from copula_var import synthetic
    from copula_var.optim.msm import Optimizer
    cfg = synthetic.baseline_configs()[2].with_(T=1, n_in=399)
    x = synthetic.simulate_returns(cfg)[:, 0]
    r = x - x.mean()
    dev = Optimizer(r, 4, basin_iter=8, seed=5)
    cpu = Optimizer(r, 4, basin_iter=8, seed=5, loglik=lambda rows: np.array([msm_loglik(r, 4, *row) for row in rows]))
    np.testing.assert_allclose(dev.optimize(), cpu.optimize(), rtol=1e-9)


@pytest.mark.parametrize("dim,row", [(2, [4.0, 0.3]), (2, [7.5, 0.6]), (2, [2.2, 0.95]), (2, [30.0, -0.2]),
                                     (3, [6.0, 0.4, 0.3, 0.5]), (3, [3.5, 0.1, -0.2, 0.2])])
def test_student_copula_nll_device_quantiles(dim, row):
    """Device t.ppf (1e-13 relative) vs the oracle's scalar scipy loop (scipy's stdtrit
    is ~1e-11 accurate): the summed log-likelihood agrees to 1e-9 relative."""
    from oracle.copula_fit import student_nll, student_sample
    from copula_var.optim.copula_fit import StudentCopulaOptimizer
    u, d = student_sample(400 if dim == 2 else 200, dim, 5.0, 0.5 if dim == 2 else 0.4, seed=31 + dim)
    got = StudentCopulaOptimizer(u, d).negative_log_likelihood(np.array(row))
    np.testing.assert_allclose(got, student_nll(u, d, row), rtol=1e-9)


def test_student_copula_optimizer_on_device_matches_cpu():
    """Same two-stage L-BFGS-B run with device and scipy quantiles: same fit to 1e-5
    (finite-difference gradients see the 1e-11 quantile differences)."""
    from scipy.stats import t
    from oracle.copula_fit import student_sample
    from copula_var.optim.copula_fit import StudentCopulaOptimizer
    u, d = student_sample(400, 2, 5.0, 0.5, seed=31)
    dev = StudentCopulaOptimizer(u, d, nu_values=np.array([3.0, 8.0])).optimize()
    cpu = StudentCopulaOptimizer(u, d, nu_values=np.array([3.0, 8.0]), tppf=lambda x, nu: t.ppf(x, nu)).optimize()
    np.testing.assert_allclose(dev["optimized_params"], cpu["optimized_params"], rtol=1e-5)
    np.testing.assert_allclose(dev["nll"], cpu["nll"], rtol=1e-9)


def test_gaussian_copula_optimizer_on_device():
    from oracle.copula_fit import gaussian_nll, student_sample
    from copula_var.optim.copula_fit import GaussianCopulaOptimizer
    u, d = student_sample(400, 2, 5.0, 0.5, seed=31)
    opt = GaussianCopulaOptimizer(u, d)
    for rho in (0.2, 0.7, -0.5):
        np.testing.assert_allclose(opt.negative_log_likelihood([rho]), gaussian_nll(u, d, [rho]), rtol=1e-11)
    res = opt.optimize()
    assert 0.3 < res["optimized_params"][0] < 0.7 and opt.launches == 1
