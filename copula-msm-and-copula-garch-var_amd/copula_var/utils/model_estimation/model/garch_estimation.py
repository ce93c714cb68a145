"""GARCH model adapter (utils/model_estimation/model/garch_estimation.py of the reference).

integration_params_retrieval (garch_estimation.py:133-145) returns
([sigma (T, dim)], None, (ones (dim,1,n), x_values, step, zeros (1, dim))) with
the sigma forecasts computed by one device thread per (asset, window)
(cvq_garch_forecast; garch/forecast.py:5-19 + estimation.py:40-65).
"""
from __future__ import annotations

import numpy as np

from .... import insample, integrand, tables
from ....data_loader.load_data import centred_series
from ...calc_var_ABC import SharedCacheCopulaGarchVaR, VaRCalculationMethod


def _garch_params(p):
    """{'best_pq', 'best_params'} -> the device forecast's arguments: the (1, 1) kernel
    for (1, 1), the GARCH(p, q) kernel (1 <= p, q <= 4) otherwise."""
    op = p["optimal_params"]
    pq = tuple(int(v) for v in op["best_pq"])
    bp = np.asarray(op["best_params"], dtype=np.float64)
    if pq == (1, 1):
        return {"omega": float(bp[0]), "alpha": float(bp[1]), "beta": float(bp[2])}
    return {"pq": pq, "params": bp}


class GarchEstimation(VaRCalculationMethod):
    model_kind = "garch"
    device = 0

    def model_params_insample(self, in_sample_dict):
        """garch_estimation.py:17-54: params per ticker from SharedCacheCopulaGarchVaR.cache,
        else the Newton-Raphson / BIC order search (optim.garch.GarchOptimizer: each Newton
        step's stencil likelihoods in one device launch) and cached."""
        from ....optim.garch import GarchOptimizer
        results = {}
        for ticker, returns in in_sample_dict.items():
            if ticker not in SharedCacheCopulaGarchVaR.cache:
                best_pq, best_params, _, best_bic = GarchOptimizer(np.asarray(returns, dtype=np.float64),
                                                                   device=self.device).optimize()
                SharedCacheCopulaGarchVaR.cache[ticker] = {
                    "optimal_params": {"best_pq": best_pq, "best_params": best_params, "best_bic": best_bic}}
            results[ticker] = SharedCacheCopulaGarchVaR.cache[ticker]
        return results

    @staticmethod
    def calculate_marginals_and_densities_in_sample(in_sample_dict, in_sample_params):
        """garch_estimation.py:57-119: per ticker (cached under (ticker, 'marginals'))
        Phi / phi of eps_t = r_t / sigma_t (garch/estimation.py:76-89), stacked (N, dim)."""
        marg, dens = [], []
        for ticker, params in in_sample_params.items():
            key = (ticker, "marginals")
            if key not in SharedCacheCopulaGarchVaR.cache:
                op = params["optimal_params"]
                m, d = insample.garch_marginals_densities(np.asarray(in_sample_dict[ticker], dtype=np.float64),
                                                          op["best_pq"], op["best_params"])
                SharedCacheCopulaGarchVaR.cache[key] = {"marginals": m, "densities": d}
            c = SharedCacheCopulaGarchVaR.cache[key]
            marg.append(np.asarray(c["marginals"]).reshape(-1, 1))
            dens.append(np.asarray(c["densities"]).reshape(-1, 1))
        return np.hstack(marg), np.hstack(dens), None

    def copula_or_correl_params_insample(self, *args, **kwargs):
        raise NotImplementedError("the copula adapter fits the copula")

    @staticmethod
    def compute_normal_densities(dim, num_points, x_min=-5, x_max=5):
        """garch_estimation.py:148-188."""
        x, step = tables.x_grid(num_points, "garch", x_min, x_max)
        return np.ones((dim, 1, num_points)), x, step

    def integration_params_retrieval(self, dim, rolling_windows_dict, in_sample_params, num_points,
                                     vol_state_array):
        params = [_garch_params(p) for p in in_sample_params.values()]
        centred = centred_series(rolling_windows_dict, list(in_sample_params.keys()))
        n_in = centred.shape[0] - len(rolling_windows_dict)
        return tables.sigma_integration_params(centred, n_in, "garch", params, num_points, self.device)

    def integrated_function(self, grids, step_sizes, copula_params, integrations_params_i,
                            integrations_params_static, copula_density, unpack_copula_params):
        """garch_integration_function.py:5-52 (garch_estimation.py:234-252): the per-node integrand for a caller-built
        nested grid, erf / quantiles on this adapter's device (copula_var/integrand.py).  The VaR
        path does not use it: the device solve evaluates the integrand in its kernels."""
        return integrand.sigma_integrated_function(grids, step_sizes, copula_params, integrations_params_i,
                                                    integrations_params_static, copula_density,
                                                    unpack_copula_params, device=self.device)
