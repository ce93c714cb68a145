"""Plugin surface of the reference (utils/calc_var_ABC.py:1-111), unchanged in shape.

A (copula x model) adapter implements these four methods; the driver
(utils/calc_var_class.py) calls them in this order, then hands the
integration parameters to the device engine instead of the reference's
numba/joblib quadrature.
"""
from abc import ABC, abstractmethod


class SharedCacheCopulaMSMVaR:
    """In-sample MSM params per (ticker, k) -- calc_var_ABC.py:4-8."""
    cache = {}


class SharedCacheCopulaGarchVaR:
    """In-sample GARCH params per ticker -- calc_var_ABC.py:11-15."""
    cache = {}


class SharedCacheCopulaMRVaR:
    """In-sample mean-reverting (UKF) params per ticker -- calc_var_ABC.py:18-22."""
    cache = {}


class VaRCalculationMethod(ABC):
    """calc_var_ABC.py:25-111."""

    @abstractmethod
    def model_params_insample(self, *args, **kwargs):
        """In-sample model parameters per ticker ({ticker: {'optimal_params': ...}})."""

    @abstractmethod
    def calculate_marginals_and_densities_in_sample(self, *args, **kwargs):
        """(marginals, densities, vol_states_array) of the in-sample returns."""

    @abstractmethod
    def copula_or_correl_params_insample(self, *args, **kwargs):
        """Best-fit copula / correlation parameters from the in-sample marginals."""

    @abstractmethod
    def integration_params_retrieval(self, *args, **kwargs):
        """(integrations_params_t, integrations_params_static, grids_generations_params)."""
