"""Mean-reverting log-vol (UKF) model adapter
(utils/model_estimation/model/mean_reverting_estimation.py of the reference).

integration_params_retrieval (:135-147) returns ([sigma (T, dim)], None,
(ones, x_values, step, zeros)) with one device UKF pass per (asset, window)
(cvq_ukf_forecast; kalman_mean_reverting/forecast.py:5-12 + estimate.py:230-281,
including the Q19 prediction-step forecast).  A window whose UKF normaliser
falls below 1e-10 makes the reference return None and crash in np.exp
(forecast.py:12); here the call raises NativeError(CVQ_ERR_NUMERIC).
"""
from __future__ import annotations

from .... import tables
from ....data_loader.load_data import centred_series
from ...calc_var_ABC import SharedCacheCopulaMRVaR, VaRCalculationMethod
from .garch_estimation import GarchEstimation


class MeanRevertingEstimation(VaRCalculationMethod):
    model_kind = "mean_reverting"
    device = 0

    @staticmethod
    def model_params_insample(in_sample_dict):
        """mean_reverting_estimation.py:17-57: cached {'optimal_params': {'a','l','q'}} per
        ticker (the EM optimiser, kalman_mean_reverting/optimize.py, is out of scope)."""
        results = {}
        for ticker in in_sample_dict:
            if ticker not in SharedCacheCopulaMRVaR.cache:
                raise NotImplementedError(
                    f"no in-sample mean-reverting parameters for {ticker!r}: the in-sample optimiser is out "
                    "of scope; inject them into SharedCacheCopulaMRVaR.cache[ticker]")
            results[ticker] = SharedCacheCopulaMRVaR.cache[ticker]
        return results

    @staticmethod
    def calculate_marginals_and_densities_in_sample(in_sample_dict, in_sample_params):
        return None, None, None

    def copula_or_correl_params_insample(self, *args, **kwargs):
        raise NotImplementedError("the copula adapter fits the copula")

    compute_normal_densities = GarchEstimation.compute_normal_densities

    def integration_params_retrieval(self, dim, rolling_windows_dict, in_sample_params, num_points,
                                     vol_state_array):
        params = [{k: float(v) for k, v in p["optimal_params"].items()} for p in in_sample_params.values()]
        centred = centred_series(rolling_windows_dict, list(in_sample_params.keys()))
        n_in = centred.shape[0] - len(rolling_windows_dict)
        return tables.sigma_integration_params(centred, n_in, "mean_reverting", params, num_points, self.device)

    def integrated_function(self, *args, **kwargs):
        raise NotImplementedError("the integrand is evaluated inside the device quadrature (cvq_slab / cvq_solve)")
