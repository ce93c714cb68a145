"""GARCH model adapter (utils/model_estimation/model/garch_estimation.py of the reference).

integration_params_retrieval (garch_estimation.py:133-145) returns
([sigma (T, dim)], None, (ones (dim,1,n), x_values, step, zeros (1, dim))) with
the sigma forecasts computed by one device thread per (asset, window)
(cvq_garch_forecast; garch/forecast.py:5-19 + estimation.py:40-65).
"""
from __future__ import annotations

import numpy as np

from .... import tables
from ....data_loader.load_data import centred_series
from ...calc_var_ABC import SharedCacheCopulaGarchVaR, VaRCalculationMethod


def _garch11(p):
    op = p["optimal_params"]
    pq = tuple(op["best_pq"])
    if pq != (1, 1):
        raise NotImplementedError(f"device GARCH forecast supports (p, q) = (1, 1); got {pq}")
    bp = np.asarray(op["best_params"], dtype=np.float64)
    return {"omega": float(bp[0]), "alpha": float(bp[1]), "beta": float(bp[2])}


class GarchEstimation(VaRCalculationMethod):
    model_kind = "garch"
    device = 0

    @staticmethod
    def model_params_insample(in_sample_dict):
        """garch_estimation.py:17-54: cached params per ticker.  The Newton-Raphson / BIC
        optimiser (garch/opti.py) is out of scope: inject
        {'optimal_params': {'best_pq': (1, 1), 'best_params': [omega, alpha, beta]}}."""
        results = {}
        for ticker in in_sample_dict:
            if ticker not in SharedCacheCopulaGarchVaR.cache:
                raise NotImplementedError(
                    f"no in-sample GARCH parameters for {ticker!r}: the in-sample optimiser is out of scope; "
                    "inject them into SharedCacheCopulaGarchVaR.cache[ticker]")
            results[ticker] = SharedCacheCopulaGarchVaR.cache[ticker]
        return results

    @staticmethod
    def calculate_marginals_and_densities_in_sample(in_sample_dict, in_sample_params):
        """garch_estimation.py:57-115 (in-sample marginals feed the copula fit: out of scope)."""
        return None, None, None

    def copula_or_correl_params_insample(self, *args, **kwargs):
        raise NotImplementedError("the copula adapter fits the copula")

    @staticmethod
    def compute_normal_densities(dim, num_points, x_min=-5, x_max=5):
        """garch_estimation.py:148-188."""
        x, step = tables.x_grid(num_points, "garch", x_min, x_max)
        return np.ones((dim, 1, num_points)), x, step

    def integration_params_retrieval(self, dim, rolling_windows_dict, in_sample_params, num_points,
                                     vol_state_array):
        params = [_garch11(p) for p in in_sample_params.values()]
        centred = centred_series(rolling_windows_dict, list(in_sample_params.keys()))
        n_in = centred.shape[0] - len(rolling_windows_dict)
        return tables.sigma_integration_params(centred, n_in, "garch", params, num_points, self.device)

    def integrated_function(self, *args, **kwargs):
        raise NotImplementedError("the integrand is evaluated inside the device quadrature (cvq_slab / cvq_solve)")
