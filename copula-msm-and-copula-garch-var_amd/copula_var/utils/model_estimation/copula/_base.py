"""Shared forwarding of the copula adapters to their model (estimation) object.

The reference's three adapters (utils/model_estimation/copula/*_estimation.py)
each forward the model-side methods to ``self.estimation_method``; this base
class does that once.
"""
from __future__ import annotations

from ...calc_var_ABC import VaRCalculationMethod


class CopulaAdapter(VaRCalculationMethod):
    copula_kind = ""

    def __init__(self, estimation_method):
        self.estimation_method = estimation_method

    @property
    def device(self) -> int:
        return int(getattr(self.estimation_method, "device", 0))

    @property
    def model_kind(self) -> str:
        return self.estimation_method.model_kind

    def set_device(self, device: int) -> None:
        self.estimation_method.device = int(device)

    def model_params_insample(self, *args, **kwargs):
        return self.estimation_method.model_params_insample(*args, **kwargs)

    def calculate_marginals_and_densities_in_sample(self, *args, **kwargs):
        return self.estimation_method.calculate_marginals_and_densities_in_sample(*args, **kwargs)

    def integration_params_retrieval(self, *args, **kwargs):
        return self.estimation_method.integration_params_retrieval(*args, **kwargs)

    def integrated_function(self, *args, **kwargs):
        return self.estimation_method.integrated_function(*args, **kwargs)

    def compute_normal_densities(self, *args, **kwargs):
        return self.estimation_method.compute_normal_densities(*args, **kwargs)

    def __getattr__(self, name):
        # remaining reference helpers (sum_forecast_by_state, create_vol_combinations, ...)
        if name == "estimation_method":
            raise AttributeError(name)
        return getattr(self.estimation_method, name)
