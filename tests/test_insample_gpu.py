"""In-sample stage on the MI355X: the UKF E-step kernel (cvq_ukf_filter), the GARCH(p, q)
forecast kernel (cvq_garch_forecast_pq), the device EM fit, and the reference pipeline
run end to end with NO injected parameters (optimiser -> in-sample marginals -> copula
fit -> forecasts -> VaR), as main.py runs it."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _mr_series(n=400, seed=21):
    from copula_var import synthetic
    cfg = [c for c in synthetic.baseline_configs().values() if c.model == "mean_reverting"][0]
    return synthetic.simulate_returns(cfg.with_(T=1, n_in=n - 1, seed=seed))


def test_msm_marginals_kernel_matches_reference():
    """cvq_msm_marginals (one device Hamilton-filter pass with the per-step state sums)
    against calc_marginals / calc_densities run by the reference itself (optim_msm_marg.npz,
    calc_marginals.py:7-30) and against the host restatement; the filter's transition
    product sums in another order than the reference's per-row loop, so the bar is
    relative.  Plus k = 1..6 on a longer series against the host restatement."""
    from copula_var import engine
    from copula_var.insample import msm_marginals_densities, msm_marginals_densities_device
    z = load_golden("optim_msm_marg")
    for row, mw, dw, vw in zip(z["rows"], z["marginals"], z["densities"], z["vol_states"]):
        m, d, vol = msm_marginals_densities_device(z["returns"], int(z["k"]), *row)
        np.testing.assert_array_equal(vol, vw)
        np.testing.assert_allclose(m, mw, rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(d, dw, rtol=1e-12, atol=1e-300)
    x = _mr_series(n=1136, seed=5)[:, 0]
    for k in range(1, 7):
        m, d = engine.msm_marginals(x, k, 0.6, float(np.std(x)), 2.5, 0.4)
        mh, dh, _ = msm_marginals_densities(x, k, 0.6, float(np.std(x)), 2.5, 0.4)
        np.testing.assert_allclose(m, mh, rtol=1e-12, atol=1e-300, err_msg=f"k {k}")
        np.testing.assert_allclose(d, dh, rtol=1e-12, atol=1e-300, err_msg=f"k {k}")


def test_ukf_filter_kernel_matches_oracle():
    from oracle.optim import ukf_filter_batch
    from copula_var import engine
    x = _mr_series()
    P = np.array([[0.97, 0.05, 0.15], [0.99, 0.5, 0.1], [0.6, -0.2, 0.3], [0.9, 0.1, 0.05], [0.999, 0.0, 0.02]])
    ll, st = engine.ukf_filter(x[:, 0], P)                             # one series for every row
    ll_o, st_o = ukf_filter_batch(x[:, 0], P)
    np.testing.assert_allclose(ll, ll_o, rtol=1e-12)
    np.testing.assert_allclose(st, st_o, rtol=1e-11, atol=1e-13)
    R = np.stack([x[:, 0], x[:, 1], x[:, 0], x[:, 1], x[:, 1]])       # one series per row
    ll2, st2 = engine.ukf_filter(R, P)
    ll2_o, st2_o = ukf_filter_batch(R, P)
    np.testing.assert_allclose(ll2, ll2_o, rtol=1e-12)
    np.testing.assert_allclose(st2, st2_o, rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(engine.ukf_loglik(x[:, 0], P), ll, rtol=1e-15)   # same pass as cvq_ukf_loglik


def test_ukf_em_on_device_replays_the_cpu_chain():
    from oracle.optim import ukf_filter_batch
    from copula_var.optim.ukf import VolOptimizer, em_lockstep
    x = _mr_series()
    dev = [VolOptimizer(0.99, 0.5, 0.1, max_iter=60, tol=1e-6, seed=s) for s in (3, 4)]
    cpu = [VolOptimizer(0.99, 0.5, 0.1, max_iter=60, tol=1e-6, seed=s, efilter=ukf_filter_batch) for s in (3, 4)]
    got = em_lockstep(dev, [x[:, 0], x[:, 1]])
    want = em_lockstep(cpu, [x[:, 0], x[:, 1]])
    for (pg, lg), (pw, lw) in zip(got, want):
        np.testing.assert_allclose(pg, pw, rtol=1e-9)
        np.testing.assert_allclose(lg, lw, rtol=1e-11)
    assert all(o.launches == o.passes for o in dev)           # one pass per chain per shared launch


@pytest.mark.parametrize("p,q", [(1, 1), (1, 2), (2, 1), (2, 2), (3, 3), (4, 1)])
def test_garch_forecast_pq_kernel(p, q):
    from oracle.optim import garch_forecast_pq
    from copula_var import engine
    r = load_golden("optim_garch")["returns"]
    rng = np.random.default_rng(p * 10 + q)
    prm = np.concatenate(([0.05], rng.uniform(0.02, 0.8 / (p + q), size=p + q)))
    n_in, T = 300, 40
    got = engine.garch_forecast_pq(r[:n_in + T - 1], n_in, p, q, prm)
    want = [garch_forecast_pq(r[t:t + n_in], prm[0], prm[1:p + 1], prm[p + 1:]) for t in range(T)]
    np.testing.assert_allclose(got, want, rtol=2e-16, atol=0)
    if (p, q) == (1, 1):
        np.testing.assert_array_equal(got, engine.garch_forecast(r[:n_in + T - 1], n_in, *prm))


@pytest.mark.parametrize("case", ["cfg1", "cfg2_n64", "cfg5_n64", "msm_gauss_n64", "ukf_plackett_n64"])
def test_pipeline_without_injected_parameters(case):
    """main.py's pipeline from returns alone: every in-sample stage runs (device
    optimisers, host/device marginals, copula fit) and the VaR is computed."""
    from driver_util import inject
    from copula_var.utils import calc_var_ABC as A
    from copula_var.utils.calc_var_class import ValueAtRiskCalcualtion
    from copula_var.utils.factory import ValueAtRiskCalculationFactory
    z = load_golden(case)
    tickers, start, kw = inject(z)
    for c in (A.SharedCacheCopulaMSMVaR, A.SharedCacheCopulaGarchVaR, A.SharedCacheCopulaMRVaR):
        c.cache.clear()                                          # returns only: no fitted parameters
    model, copula = str(z["model"]), str(z["copula"])
    calc = ValueAtRiskCalculationFactory.create_var_calculator(copula_type=copula, estimation_type=model)
    v = ValueAtRiskCalcualtion(tickers, start, int(z["n_in"]), calc, None, num_points=int(z["num_points"]),
                               weights=z["weights"], **kw)
    var = v.calc_var()
    assert var.shape == (v.out_sample_N,) and np.all(np.isfinite(var)) and np.all(var < 0)
    assert v.marginals.shape[1] == v.dim and np.all((v.marginals >= 0) & (v.marginals <= 1))
    if copula == "student":
        assert 2.01 <= v.copula_params[0] <= 50 and np.all(np.abs(v.copula_params[1:]) <= 0.99)
    elif copula == "gaussian":
        assert np.all(np.abs(v.copula_params) <= 0.99)
    else:
        assert float(np.asarray(v.copula_params).ravel()[0]) >= 0.1
    cache = {"msm": A.SharedCacheCopulaMSMVaR, "garch": A.SharedCacheCopulaGarchVaR,
             "mean_reverting": A.SharedCacheCopulaMRVaR}[model].cache
    assert all((tk, kw["k"]) in cache if model == "msm" else tk in cache for tk in tickers)


def test_ukf_kernels_match_reference_golden():
    """cvq_ukf_filter / cvq_ukf_loglik / cvq_ukf_forecast against the reference's own
    KalmanFilterVolEstimation(a, l, q, l, q, n, returns) (estimate.py:230-281; LL at :276,
    forecast mean at :258/:281, Q19) at fixed (a, l, q) rows (golden optim_ukf)."""
    from copula_var import engine
    z = load_golden("optim_ukf")
    r, P = z["returns"], z["rows"]
    ll, st = engine.ukf_filter(r, P)
    np.testing.assert_allclose(ll, z["ll"], rtol=1e-12)
    np.testing.assert_allclose(st, z["states"], rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(engine.ukf_loglik(r, P), z["ll"], rtol=1e-12)
    for i, (a, l, q) in enumerate(P):
        f = engine.ukf_forecast(r, r.size, a, l, q)          # one window = the whole series
        np.testing.assert_allclose(np.log(f[0]), z["forecast_mean"][i], rtol=1e-12)


def test_garch_forecast_pq_kernel_matches_reference_golden():
    """cvq_garch_forecast_pq against garch/forecast.py:5-19 run by the reference for
    (p, q) in {(2,1), (1,2), (2,2), (3,2)} (Q13 lag order), rolling windows."""
    from copula_var import engine
    z = load_golden("optim_garch_pq")
    s, n_in = z["returns"], int(z["n_in"])
    for i, (p, q) in enumerate(z["orders"]):
        w = z["params"][i][:1 + p + q]
        got = engine.garch_forecast_pq(s, n_in, int(p), int(q), w)
        np.testing.assert_allclose(got, z["forecasts"][i], rtol=1e-13, err_msg=f"GARCH({p},{q})")


@pytest.mark.parametrize("device", [0, 1])
def test_msm_adapter_marginals_run_on_its_device(device):
    """the MSM adapter's in-sample marginals run on the adapter's device
    (set_device), and the library restores the caller's current HIP device afterwards
    (torch shares it)."""
    import torch
    from copula_var.insample import msm_marginals_densities
    from copula_var.utils.calc_var_ABC import SharedCacheCopulaMSMVaR
    from copula_var.utils.model_estimation.model.msm_estimation import MSMEstimation
    if device >= torch.cuda.device_count():
        pytest.skip(f"needs {device + 1} GPUs")
    torch.cuda.set_device(0)
    x = _mr_series(n=600, seed=9)[:, 0]
    est = MSMEstimation()
    est.device = device
    prm = {"m_0": 0.6, "sig": float(np.std(x)), "b": 2.5, "gamma": 0.4}
    key = ("dev_probe", "marginals_3")
    SharedCacheCopulaMSMVaR.cache.pop(key, None)
    try:
        m, d, v = est.calculate_marginals_and_densities_in_sample({"dev_probe": x}, {"dev_probe": {"optimal_params": prm}}, 3)
    finally:
        SharedCacheCopulaMSMVaR.cache.pop(key, None)
    assert torch.cuda.current_device() == 0
    mh, dh, _ = msm_marginals_densities(x, 3, prm["m_0"], prm["sig"], prm["b"], prm["gamma"])
    np.testing.assert_allclose(m[:, 0], mh, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(d[:, 0], dh, rtol=1e-12, atol=1e-300)
