"""Gaussian copula adapter (utils/model_estimation/copula/gaussian_estimation.py:7-79)."""
from __future__ import annotations

import numpy as np

from .... import copulas
from ._base import CopulaAdapter


class GaussianCopulaVaR(CopulaAdapter):
    copula_kind = "gaussian"

    @staticmethod
    def unpack_copula_params(copula_params):
        """(None, corr_matrix) from the packed upper triangle (gaussian_estimation.py:13-23)."""
        rho = copula_params
        n = int((1 + np.sqrt(1 + 8 * len(rho))) / 2)
        corr = np.eye(n)
        corr[np.triu_indices(n, k=1)] = rho
        corr[np.tril_indices(n, k=-1)] = rho
        return None, corr

    def copula_or_correl_params_insample(self, marginals, densities):
        """gaussian_estimation.py:25-33: the IFM fit with device norm.ppf quantiles."""
        from ....optim.copula_fit import GaussianCopulaOptimizer
        return GaussianCopulaOptimizer(marginals, densities, device=self.device).optimize()

    @staticmethod
    def copula_integrations_params(best_g_params):
        """rho upper triangle (gaussian_estimation.py:36-44)."""
        corr = np.asarray(best_g_params["corr_matrix"])
        return corr[np.triu_indices_from(corr, k=1)]

    @staticmethod
    def copula_density(cdf, corr_matrix, **kwargs):
        return copulas.gaussian(cdf, corr_matrix)
