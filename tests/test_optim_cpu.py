"""In-sample optimiser layer on the CPU: the oracle's likelihoods and the product's
GarchOptimizer host logic (driven by the oracle likelihood) against the reference's
own results (tests/golden/gen_optim_golden.py: garch/opti.py, garch/estimation.py,
markov_switching_multifractal/calc_prob.py run in the build container)."""
import numpy as np
import pytest

from conftest import load_golden


def _rows(z, p, q):
    sel = [i for i, (pp, qq) in enumerate(z["ll_pq"]) if (pp, qq) == (p, q)]
    return z["ll_rows"][sel][:, :1 + p + q], z["ll"][sel]


@pytest.mark.parametrize("p,q", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_oracle_garch_loglik_matches_reference(p, q):
    from oracle.optim import garch_loglik_batch
    z = load_golden("optim_garch")
    rows, ll = _rows(z, p, q)
    np.testing.assert_array_equal(garch_loglik_batch(z["returns"], rows, p, q), ll)   # same arithmetic


def test_garch_optimizer_host_logic_matches_reference():
    """opti.py's Newton-Raphson / FD stencils / BIC search with the oracle likelihood:
    the reference's exact path (bit-identical likelihoods -> identical iterates)."""
    from oracle.optim import garch_loglik_batch
    from copula_var.optim.garch import GarchOptimizer
    z = load_golden("optim_garch")
    r = z["returns"]
    opt = GarchOptimizer(r, p_max=int(z["p_max"]), q_max=int(z["q_max"]),
                         loglik=lambda rows, p, q: garch_loglik_batch(r, rows, p, q))
    best_pq, best_params, best_nll, best_bic = opt.optimize()
    assert tuple(best_pq) == tuple(z["best_pq"])
    np.testing.assert_allclose(best_params, z["best_params"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(best_nll, float(z["best_nll"]), rtol=1e-13)
    np.testing.assert_allclose(best_bic, float(z["best_bic"]), rtol=1e-13)
    # one batched likelihood call per Newton step (+ the final value), 1 + 2n rows each
    assert opt.launches > 0 and opt.evaluations >= 7 * (opt.launches - 4) // 2


def test_garch_optimizer_penalty_and_unpack():
    from copula_var.optim.garch import GarchOptimizer
    opt = GarchOptimizer(np.zeros(10), loglik=lambda rows, p, q: np.zeros(len(rows)))
    assert opt.negative_log_likelihood(np.array([0.1, 0.6, 0.5]), 1, 1) == 1e10        # opti.py:30-31
    with pytest.raises(ValueError):
        opt.negative_log_likelihood(np.array([0.0, 0.1, 0.1]), 1, 1)                 # estimation.py:33-34
    w, a, b = opt.unpack_garch_parameters(((2, 1), np.array([0.1, 0.2, 0.05, 0.6])))
    assert w == 0.1 and list(a) == [0.2, 0.05] and list(b) == [0.6]


def test_oracle_msm_loglik_matches_reference():
    from oracle.forecast import msm_loglik
    z = load_golden("optim_msm_ll")
    got = [msm_loglik(z["returns"], int(z["k"]), *row) for row in z["rows"]]
    np.testing.assert_allclose(got, z["ll"], rtol=1e-12)


def _msm_series(n=300):
    from copula_var import synthetic
    cfg = synthetic.baseline_configs()[2].with_(T=1, n_in=n - 1)
    x = synthetic.simulate_returns(cfg)[:, 0]
    return x - x.mean()


def test_msm_optimizer_host_logic_is_reproducible():
    """opti.py's basin hopping / b sweep driven by the oracle likelihood: seeded chains
    replay exactly, every proposal stays inside the bounds, one call per iteration."""
    from oracle.forecast import msm_loglik
    from copula_var.optim.msm import Optimizer
    r = _msm_series()
    ll = lambda rows: np.array([msm_loglik(r, 2, *row) for row in rows])
    runs = []
    for _ in range(2):
        opt = Optimizer(r, 2, basin_iter=6, seed=11, loglik=ll)
        runs.append((opt.optimize(), opt.launches))
    assert runs[0][0] == runs[1][0]
    m0, b, gamma, sigma = runs[0][0]
    assert 0.2 <= m0 <= 0.8 and 1.0 <= b <= 50.0 and 0.05 <= gamma <= 0.95
    np.testing.assert_allclose(sigma, np.sqrt(np.var(r)) / (m0 ** 2 - 2 * m0 + 2) ** (2 / 2), rtol=1e-15)
    assert runs[0][1] <= 6 + 2                                # <= one launch per iteration + start + final


def test_oracle_ukf_filter_matches_reference():
    """UKF E-step (kalman_mean_reverting/estimate.py:230-281, init (l, q) as forecast.py:9
    and optimize.py:31 call it): LL, state path and forecast mean vs the reference's own
    KalmanFilterVolEstimation (tests/golden/gen_optim_golden.py ukf_garch_pq)."""
    from oracle.optim import ukf_filter_batch
    from oracle.forecast import ukf_run
    z = load_golden("optim_ukf")
    ll, st = ukf_filter_batch(z["returns"], z["rows"])
    np.testing.assert_allclose(ll, z["ll"], rtol=1e-12)
    np.testing.assert_allclose(st, z["states"], rtol=1e-11, atol=1e-13)
    for i, (a, l, q) in enumerate(z["rows"]):
        f, _, _, failed = ukf_run(z["returns"][None, :], a, l, q)
        assert not failed[0]
        np.testing.assert_allclose(np.log(f[0]), z["forecast_mean"][i], rtol=1e-12)


def test_oracle_optim_garch_pq_matches_reference():
    """garch/forecast.py:5-19 for (p, q) != (1, 1): alpha_1 pairs with the oldest of the
    last p returns (Q13), beta_1 with the oldest of the last q variances."""
    from oracle.optim import garch_forecast_pq
    z = load_golden("optim_garch_pq")
    s, n_in = z["returns"], int(z["n_in"])
    for i, (p, q) in enumerate(z["orders"]):
        w = z["params"][i]
        got = [garch_forecast_pq(s[t:t + n_in], w[0], w[1:p + 1], w[p + 1:p + 1 + q])
               for t in range(z["forecasts"].shape[1])]
        np.testing.assert_allclose(got, z["forecasts"][i], rtol=1e-14)
