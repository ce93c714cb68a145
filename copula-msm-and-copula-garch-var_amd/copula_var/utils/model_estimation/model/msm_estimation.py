"""MSM model adapter (utils/model_estimation/model/msm_estimation.py of the reference).

The per-date forecast stage (forecasts_array -> sum_forecast_by_state ->
compute_normal_densities -> create_vol_combinations ->
compute_forecast_combinations, msm_estimation.py:123-418) runs with one
device Hamilton filter per (asset, window) batch (cvq_msm_filter) and returns
the reference's exact (integrations_params_t, integrations_params_static,
grids_generations_params) layout.

Deliberate difference: Q8.  The reference recovers k as
int(sqrt(2**k)) (msm_estimation.py:125), which is right only for
k in {1, 2, 4, 5} and raises IndexError otherwise.  Here k =
log2(states): identical results where the reference works, the evidently
intended ("patched-k") result where it crashes.
"""
from __future__ import annotations

import numpy as np

from .... import insample, integrand, tables
from ....data_loader.load_data import centred_series
from ...calc_var_ABC import SharedCacheCopulaMSMVaR, VaRCalculationMethod


class MSMEstimation(VaRCalculationMethod):
    model_kind = "msm"
    device = 0

    seed = 0

    def model_params_insample(self, in_sample_dict, k):
        """msm_estimation.py:17-52: params per (ticker, k) from SharedCacheCopulaMSMVaR.cache,
        else the basin-hopping fit (optim.msm.Optimizer: the 10 b-chains' proposals in one
        device launch per iteration; seeded, see optim/msm.py) and cached."""
        from ....optim.msm import Optimizer
        results = {}
        for ticker, returns in in_sample_dict.items():
            key = (ticker, k)
            if key not in SharedCacheCopulaMSMVaR.cache:
                p = Optimizer(np.asarray(returns, dtype=np.float64), k, seed=self.seed, device=self.device).optimize()
                SharedCacheCopulaMSMVaR.cache[key] = {
                    "optimal_params": {"m_0": p[0], "sig": p[3], "b": p[1], "gamma": p[2]}}   # :45-48
            results[ticker] = SharedCacheCopulaMSMVaR.cache[key]
        return results

    def calculate_marginals_and_densities_in_sample(self, in_sample_dict, in_sample_params, k):
        """msm_estimation.py:55-120: per ticker (cached under (ticker, 'marginals_k'))
        the filtered-probability-weighted normal cdf / pdf of the in-sample returns
        (calc_marginals.py:7-30; one device filter pass, cvq_msm_marginals, on this
        adapter's device -- set_device), stacked (N-1, dim), and the 2**k vol states.
        (The reference's is a staticmethod; here it reads the instance's device.)"""
        marg, dens, vs = [], [], []
        for ticker, params in in_sample_params.items():
            key = (ticker, f"marginals_{k}")
            if key not in SharedCacheCopulaMSMVaR.cache:
                op = params["optimal_params"]
                m, d, v = insample.msm_marginals_densities_device(
                    np.asarray(in_sample_dict[ticker], dtype=np.float64), k, op["m_0"], op["sig"], op["b"],
                    op["gamma"], self.device)
                SharedCacheCopulaMSMVaR.cache[key] = {"marginals": m, "densities": d, "vol_states": v}
            c = SharedCacheCopulaMSMVaR.cache[key]
            marg.append(np.asarray(c["marginals"]).reshape(-1, 1))
            dens.append(np.asarray(c["densities"]).reshape(-1, 1))
            vs.append(c["vol_states"])
        return np.hstack(marg), np.hstack(dens), np.array(vs)

    def copula_or_correl_params_insample(self, *args, **kwargs):
        raise NotImplementedError("the copula adapter fits the copula")

    def integration_params_retrieval(self, dim, rolling_windows_dict, in_sample_params, num_points,
                                     vol_state_array):
        """msm_estimation.py:123-137 with the filters on the device."""
        k = int(round(np.log2(vol_state_array.shape[1])))                        # Q8: true k
        if 1 << k != vol_state_array.shape[1]:
            raise ValueError("vol_state_array must have 2**k columns")
        params = [p["optimal_params"] for p in in_sample_params.values()]
        centred = centred_series(rolling_windows_dict, list(in_sample_params.keys()))
        n_in = centred.shape[0] - len(rolling_windows_dict)
        return tables.msm_integration_params(centred, n_in, params, k, num_points, self.device)

    # ---- reference helper names (msm_estimation.py:140-418), host / device pieces
    @staticmethod
    def sum_forecast_by_state(vol_state_array, forecasts_array):
        return tables.sum_forecast_by_state(vol_state_array, np.asarray(forecasts_array))

    @staticmethod
    def compute_normal_densities(unique_vol_states, num_points, x_min=-5, x_max=5):
        x, step = tables.x_grid(num_points, "msm", x_min, x_max)
        return tables.msm_densities(unique_vol_states, x), x, step

    @staticmethod
    def create_vol_combinations(unique_vol_states):
        return tables.vol_combinations(unique_vol_states.shape[0], unique_vol_states.shape[1])

    @staticmethod
    def compute_forecast_combinations(forecasts_by_states):
        return tables.forecast_combinations(np.asarray(forecasts_by_states))

    def integrated_function(self, grids, step_sizes, copula_params, integrations_params_i,
                            integrations_params_static, copula_density, unpack_copula_params):
        """msm_integration_function.py:5-47 (msm_estimation.py:445-454): the per-node integrand for a caller-built
        nested grid, erf / quantiles on this adapter's device (copula_var/integrand.py).  The VaR
        path does not use it: the device solve evaluates the integrand in its kernels."""
        return integrand.msm_integrated_function(grids, step_sizes, copula_params, integrations_params_i,
                                                    integrations_params_static, copula_density,
                                                    unpack_copula_params, device=self.device)
