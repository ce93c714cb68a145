"""The reference-shaped host layer without a GPU: offline loader semantics
(load_data.py), the factory (incl. Q17), adapter parameter packing, and the
error behaviour of the out-of-scope in-sample stages."""
import numpy as np
import pandas as pd
import pytest

from conftest import load_golden
from driver_util import inject


def test_loader_matches_reference_split_and_windows():
    from copula_var.data_loader.load_data import IndexReturnsRetriever, centred_series
    from oracle.forecast import insample_split
    z = load_golden("cfg1")
    tickers, start, _ = inject(z)
    r = IndexReturnsRetriever(tickers, start, int(z["n_in"]), z["weights"])
    ins, rolling, mean, end, out, T, dim, ptf = r.get_insample_data()
    assert ptf == float(z["ptf_mean"]) and T == z["var"].size and dim == 2
    _, _, win = insample_split(z["returns"], int(z["n_in"]), z["weights"])
    keys = list(rolling.keys())
    assert len(keys) == T and keys[0] == end                      # first window ends at the in-sample end
    for i in (0, 7, T - 1):
        w = rolling[keys[i]]
        assert np.array_equal(np.column_stack([w[tk] for tk in tickers]), win[i])
    assert np.array_equal(ins[tickers[0]], win[0][:, 0])
    plain = {k: rolling[k] for k in keys}                          # a dict built like the reference's
    assert np.array_equal(centred_series(plain, tickers)[:-1], rolling.centred[:-1])


def test_loader_is_offline_and_checks_length():
    from copula_var.data_loader.load_data import IndexReturnsRetriever, SharedCacheIndexReturns
    SharedCacheIndexReturns.returns_cache.clear()
    with pytest.raises(RuntimeError, match="no network"):
        IndexReturnsRetriever(["A", "B"], "2001-01-01", 10, np.array([0.5, 0.5]))
    idx = pd.bdate_range("2001-01-01", periods=5)
    SharedCacheIndexReturns.returns_cache[(("A", "B"), "2001-01-01", None)] = pd.DataFrame(
        np.zeros((5, 2)), index=idx, columns=["A", "B"])
    r = IndexReturnsRetriever(["A", "B"], "2001-01-01", 10, np.array([0.5, 0.5]))
    with pytest.raises(ValueError, match="Not enough returns"):
        r.get_insample_data()


def test_returns_from_prices():
    from copula_var.data_loader.load_data import returns_from_prices
    p = pd.DataFrame({"A": [100.0, 101.0, 99.0]}, index=pd.bdate_range("2020-01-01", periods=3))
    r = returns_from_prices(p)
    assert r.shape == (2, 1)
    assert r.iloc[0, 0] == pytest.approx(np.log(1.01) * 100)


def test_factory_mapping_and_q17():
    from copula_var.utils.factory import ValueAtRiskCalculationFactory as F
    for model in ("msm", "garch", "mean_reverting"):
        for cop in ("student", "gaussian", "plackett"):
            c = F.create_var_calculator(copula_type=cop, estimation_type=model)
            want = "plackett" if (model, cop) == ("mean_reverting", "gaussian") else cop
            assert c.copula_kind == want and c.model_kind == model
    with pytest.raises(ValueError, match="Unsupported estimation type."):
        F.create_var_calculator(copula_type="clayton", estimation_type="msm")


def test_copula_parameter_packing():
    from copula_var.utils.model_estimation.copula.gaussian_estimation import GaussianCopulaVaR
    from copula_var.utils.model_estimation.copula.plackett_estimation import PlackettCopulaVaR
    from copula_var.utils.model_estimation.copula.student_estimation import StudentCopulaVaR
    R = np.array([[1.0, 0.5, 0.4], [0.5, 1.0, 0.3], [0.4, 0.3, 1.0]])
    p = StudentCopulaVaR.copula_integrations_params({"optimized_params": [6.0], "corr_matrix": R})
    assert np.array_equal(p, [6.0, 0.5, 0.4, 0.3])
    nu, R2 = StudentCopulaVaR.unpack_copula_params(p)
    assert nu == 6.0 and np.array_equal(R2, R)
    g = GaussianCopulaVaR.copula_integrations_params({"corr_matrix": R})
    assert GaussianCopulaVaR.unpack_copula_params(g)[0] is None
    assert np.array_equal(GaussianCopulaVaR.unpack_copula_params(g)[1], R)
    assert PlackettCopulaVaR.copula_integrations_params({"theta": 3.0}) == 3.0
    assert PlackettCopulaVaR.unpack_copula_params(3.0) == (3.0, None)


def test_insample_stages_use_the_caches_then_the_device():
    """model_params_insample: the reference's cache first (msm_estimation.py:35-38); a miss
    runs the device-batched optimiser, which fails loudly without a GPU.  The in-sample
    marginals (device filter, likewise) are cached under the reference's key."""
    from copula_var import _native as N
    from copula_var.utils.factory import ValueAtRiskCalculationFactory as F
    from copula_var.utils.calc_var_ABC import SharedCacheCopulaMSMVaR
    SharedCacheCopulaMSMVaR.cache.clear()
    c = F.create_var_calculator(copula_type="student", estimation_type="msm")
    if not _gpu():
        with pytest.raises(N.NativeError):
            c.model_params_insample({"A": np.linspace(-1, 1, 50)}, k=4)
    SharedCacheCopulaMSMVaR.cache[("A", 4)] = {"optimal_params": {"m_0": 0.45, "sig": 1.2, "b": 3.0, "gamma": 0.3}}
    r = np.linspace(-2, 2, 40)
    got = c.model_params_insample({"A": r}, k=4)
    if not _gpu():                                   # the device filter (cvq_msm_marginals) fails loudly
        with pytest.raises(N.NativeError):
            c.calculate_marginals_and_densities_in_sample({"A": r}, got, k=4)
        SharedCacheCopulaMSMVaR.cache.clear()
        return
    m, d, vsa = c.calculate_marginals_and_densities_in_sample({"A": r}, got, k=4)
    assert vsa.shape == (1, 16) and m.shape == d.shape == (39, 1)
    assert np.all((m > 0) & (m < 1)) and np.all(d > 0)
    assert ("A", "marginals_4") in SharedCacheCopulaMSMVaR.cache
    SharedCacheCopulaMSMVaR.cache.clear()


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
