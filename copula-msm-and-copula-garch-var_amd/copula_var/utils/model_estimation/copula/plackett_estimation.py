"""Plackett copula adapter (utils/model_estimation/copula/plackett_estimation.py:6-71).

2-D only: the reference raises only in its IFM class (plackett.py:20-21) and
silently uses columns 0 and 1 on the integrand path; the device plan rejects
dim != 2 with CVQ_ERR_UNSUPPORTED."""
from __future__ import annotations

from .... import copulas
from ._base import CopulaAdapter


class PlackettCopulaVaR(CopulaAdapter):
    copula_kind = "plackett"

    @staticmethod
    def unpack_copula_params(copula_params):
        """(theta, None) (plackett_estimation.py:12-16)."""
        return copula_params, None

    @staticmethod
    def copula_or_correl_params_insample(marginals, densities):
        """plackett_estimation.py:18-26: the IFM fit (closed-form density)."""
        from ....optim.copula_fit import PlackettCopulaOptimizer
        return PlackettCopulaOptimizer(marginals, densities).optimize()

    @staticmethod
    def copula_integrations_params(best_p_params):
        """theta (plackett_estimation.py:29-37)."""
        return best_p_params["theta"]

    @staticmethod
    def copula_density(cdf, nu, **kwargs):
        return copulas.plackett(cdf, nu)
