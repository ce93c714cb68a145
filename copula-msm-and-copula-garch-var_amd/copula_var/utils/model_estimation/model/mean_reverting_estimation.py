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

import numpy as np

from .... import insample, integrand, tables
from ....data_loader.load_data import centred_series
from ...calc_var_ABC import SharedCacheCopulaMRVaR, VaRCalculationMethod
from .garch_estimation import GarchEstimation


class MeanRevertingEstimation(VaRCalculationMethod):
    model_kind = "mean_reverting"
    device = 0

    seed = 0

    def model_params_insample(self, in_sample_dict):
        """mean_reverting_estimation.py:17-57: {'optimal_params': {'a','l','q'}} per ticker
        from SharedCacheCopulaMRVaR.cache, else the EM fit (optim.ukf.VolOptimizer(0.99, 0.5,
        0.1, max_iter=1000, tol=1e-6), :41-47); the uncached tickers' chains run in lockstep,
        one device UKF launch per round for all of them.  Seeds: self.seed + i."""
        from ....optim.ukf import VolOptimizer, em_lockstep
        todo = [t for t in in_sample_dict if t not in SharedCacheCopulaMRVaR.cache]
        if todo:
            opts = [VolOptimizer(0.99, 0.5, 0.1, max_iter=1000, tol=1e-6, seed=self.seed + i, device=self.device)
                    for i in range(len(todo))]
            fits = em_lockstep(opts, [np.asarray(in_sample_dict[t], dtype=np.float64) for t in todo])
            for t, (params, _ll) in zip(todo, fits):
                SharedCacheCopulaMRVaR.cache[t] = {
                    "optimal_params": {"a": params[0], "l": params[1], "q": params[2]}}
        return {t: SharedCacheCopulaMRVaR.cache[t] for t in in_sample_dict}

    def calculate_marginals_and_densities_in_sample(self, in_sample_dict, in_sample_params):
        """mean_reverting_estimation.py:59-119: per ticker (cached under (ticker, 'marginals'))
        Phi / phi of eps = r / exp(UKF state path) (estimate.py:46-51), stacked (N, dim)."""
        marg, dens = [], []
        for ticker, params in in_sample_params.items():
            key = (ticker, "marginals")
            if key not in SharedCacheCopulaMRVaR.cache:
                op = params["optimal_params"]
                m, d = insample.mr_marginals_densities(np.asarray(in_sample_dict[ticker], dtype=np.float64),
                                                       op["a"], op["l"], op["q"], self.device)
                SharedCacheCopulaMRVaR.cache[key] = {"marginals": m, "densities": d}
            c = SharedCacheCopulaMRVaR.cache[key]
            marg.append(np.asarray(c["marginals"]).reshape(-1, 1))
            dens.append(np.asarray(c["densities"]).reshape(-1, 1))
        return np.hstack(marg), np.hstack(dens), None

    def copula_or_correl_params_insample(self, *args, **kwargs):
        raise NotImplementedError("the copula adapter fits the copula")

    compute_normal_densities = GarchEstimation.compute_normal_densities

    def integration_params_retrieval(self, dim, rolling_windows_dict, in_sample_params, num_points,
                                     vol_state_array):
        params = [{k: float(v) for k, v in p["optimal_params"].items()} for p in in_sample_params.values()]
        centred = centred_series(rolling_windows_dict, list(in_sample_params.keys()))
        n_in = centred.shape[0] - len(rolling_windows_dict)
        return tables.sigma_integration_params(centred, n_in, "mean_reverting", params, num_points, self.device)

    def integrated_function(self, grids, step_sizes, copula_params, integrations_params_i,
                            integrations_params_static, copula_density, unpack_copula_params):
        """garch_integration_function.py:5-52 (mean_reverting_estimation.py:235-253): the per-node integrand for a caller-built
        nested grid, erf / quantiles on this adapter's device (copula_var/integrand.py).  The VaR
        path does not use it: the device solve evaluates the integrand in its kernels."""
        return integrand.sigma_integrated_function(grids, step_sizes, copula_params, integrations_params_i,
                                                    integrations_params_static, copula_density,
                                                    unpack_copula_params, device=self.device)
