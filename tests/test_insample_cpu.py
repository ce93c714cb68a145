"""In-sample stage on the CPU: the host marginals (copula_var/insample.py) and the UKF EM
optimiser's control flow (copula_var/optim/ukf.py) driven by the oracle's E-step.

Pinning: the MSM filtered probabilities reproduce the reference's own calc_likelihood
values (optim_msm_ll.npz, calc_prob.py run here), and the GARCH variance recursion
reproduces numba_garch_log_likelihood (optim_garch.npz).  The EM fit has no reference
run (its draws are unseeded in the reference): seeded chains must replay exactly."""
import numpy as np
import pytest

from conftest import load_golden


def test_msm_filtered_probabilities_reproduce_reference_likelihood():
    from copula_var.insample import msm_state_probs, msm_transition
    z = load_golden("optim_msm_ll")
    k = int(z["k"])
    for (m0, sig, b, g), want in zip(z["rows"], z["ll"]):
        probs, cond, _ = msm_state_probs(z["returns"], k, m0, sig, b, g)
        A, _ = msm_transition(k, m0, b, g)
        ll = sum(np.log(np.dot(np.dot(A, probs[i - 1]), cond[i])) for i in range(1, len(probs)))  # calc_prob.py:36-47
        np.testing.assert_allclose(ll, want, rtol=1e-12)


def test_msm_marginals_shapes_and_ranges():
    from copula_var.insample import msm_marginals_densities
    z = load_golden("optim_msm_ll")
    m, d, vol = msm_marginals_densities(z["returns"], int(z["k"]), 0.45, 1.2, 3.0, 0.3)
    assert m.shape == d.shape == (z["returns"].size - 1,) and vol.shape == (2 ** int(z["k"]),)
    assert np.all((m > 0) & (m < 1)) and np.all(d > 0)


def test_msm_marginals_match_reference():
    """calc_marginals / calc_densities (calc_marginals.py:7-30) run by the reference itself
    (optim_msm_marg.npz).  The filter's A @ prev (BLAS) sums in another order than the
    reference's per-row loop (calc_prob.py:56-57), so the bar is relative, not bitwise."""
    from copula_var.insample import msm_marginals_densities
    z = load_golden("optim_msm_marg")
    for row, mw, dw, vw in zip(z["rows"], z["marginals"], z["densities"], z["vol_states"]):
        m, d, vol = msm_marginals_densities(z["returns"], int(z["k"]), *row)
        np.testing.assert_array_equal(vol, vw)
        np.testing.assert_allclose(m, mw, rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(d, dw, rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("p,q", [(1, 1), (2, 1), (2, 2)])
def test_garch_eps_reproduces_reference_variances(p, q):
    from copula_var.insample import garch_eps, garch_marginals_densities
    z = load_golden("optim_garch")
    r = z["returns"]
    sel = [i for i, (pp, qq) in enumerate(z["ll_pq"]) if (pp, qq) == (p, q)]
    for row, want in zip(z["ll_rows"][sel][:, :1 + p + q], z["ll"][sel]):
        eps = garch_eps(r, row[0], row[1:p + 1], row[p + 1:])
        s2 = (r / eps) ** 2
        m = max(p, q)
        ll = -0.5 * np.sum(np.log(2 * np.pi * s2[m:]) + r[m:] ** 2 / s2[m:])
        np.testing.assert_allclose(ll, want, rtol=1e-12)
        mg, dn = garch_marginals_densities(r, (p, q), row)
        assert np.all((mg >= 0) & (mg <= 1)) and np.all(dn >= 0)
    with pytest.raises(ValueError):
        garch_eps(r, 0.1, [0.6], [0.5])                         # estimation.py:36-38


def _mr_series(n=400, seed=21):
    from copula_var import synthetic
    cfg = [c for c in synthetic.baseline_configs().values() if c.model == "mean_reverting"][0]
    return synthetic.simulate_returns(cfg.with_(T=1, n_in=n - 1, seed=seed))


def test_ukf_em_replays_and_runs_in_lockstep():
    from oracle.optim import ukf_filter_batch
    from copula_var.optim.ukf import VolOptimizer, em_lockstep
    x = _mr_series()
    runs = []
    for _ in range(2):
        o = VolOptimizer(0.99, 0.5, 0.1, max_iter=25, tol=1e-6, seed=3, efilter=ukf_filter_batch)
        runs.append((o.em_algorithm(x[:, 0]), o.launches, o.passes))
    (p0, ll0), launches, passes = runs[0]
    assert np.array_equal(p0, runs[1][0][0]) and ll0 == runs[1][0][1]
    assert 0.5 <= p0[0] <= 0.999999 and p0[2] > 0 and np.isfinite(ll0)
    assert passes == launches and launches <= 2 * 25 + 5 * 25     # the duplicate E-steps are reused
    # two assets in lockstep: same per-chain result as one at a time, one launch per round
    a = VolOptimizer(0.99, 0.5, 0.1, max_iter=25, tol=1e-6, seed=3, efilter=ukf_filter_batch)
    b = VolOptimizer(0.99, 0.5, 0.1, max_iter=25, tol=1e-6, seed=4, efilter=ukf_filter_batch)
    (pa, lla), (pb, llb) = em_lockstep([a, b], [x[:, 0], x[:, 1]])
    assert np.array_equal(pa, p0) and lla == ll0
    single_b = VolOptimizer(0.99, 0.5, 0.1, max_iter=25, tol=1e-6, seed=4, efilter=ukf_filter_batch)
    pb1, llb1 = single_b.em_algorithm(x[:, 1])
    assert np.array_equal(pb, pb1) and llb == llb1


def test_ukf_em_m_step_pieces():
    """optimize.py:34-53, including update_l ignoring mu."""
    from copula_var.optim.ukf import VolOptimizer
    o = VolOptimizer(0.99, 0.5, 0.1)
    s = np.array([0.1, 0.3, 0.2, 0.4])
    y, x = s[1:] - 0.9 * 0.2, s[:-1] - 0.9 * 0.2
    assert o.update_a_with_ols(s, 0.9, 0.2) == np.sum(x * y) / np.sum(x ** 2)
    assert o.update_a_with_ols(np.full(4, 0.25), 0.5, 0.5) == 0.01     # zero denominator
    assert o.update_l(123.0, 0.2, 0.9) == o.update_l(-5.0, 0.2, 0.9) == 0.2 ** 2 / (2 * (1 - 0.81))
    assert o.update_q(0.9, s) == np.std(s) * np.sqrt(1 - 0.81)


def test_ukf_em_failed_passes_perturb_a():
    """A failed E-step (LL -1e10) triggers the perturbation retry loop (optimize.py:58-72)."""
    from copula_var.optim.ukf import VolOptimizer
    calls = []

    def efilter(R, P):
        calls.append(P.copy())
        ok = len(calls) > 2                                  # first two passes fail
        N = R.shape[1]
        return (np.array([-100.0 if ok else -1e10]),
                np.tile(np.linspace(0, 1, N), (1, 1)) if ok else np.full((1, N), np.nan))
    o = VolOptimizer(0.99, 0.5, 0.1, max_iter=1, seed=0, efilter=efilter)
    o.em_algorithm(np.ones(10))
    assert calls[1][0, 0] != calls[0][0, 0] and 0.5 <= calls[1][0, 0] <= 0.999999
