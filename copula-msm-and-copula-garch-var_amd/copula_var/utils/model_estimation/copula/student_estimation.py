"""Student-t copula adapter (utils/model_estimation/copula/student_estimation.py:7-91)."""
from __future__ import annotations

import numpy as np

from .... import copulas
from ._base import CopulaAdapter


class StudentCopulaVaR(CopulaAdapter):
    copula_kind = "student"

    def copula_or_correl_params_insample(self, marginals, densities):
        """student_estimation.py:12-20: copulas/student/opti.py's IFM fit, each objective's
        t.ppf quantiles in one device launch (optim.copula_fit)."""
        from ....optim.copula_fit import StudentCopulaOptimizer
        return StudentCopulaOptimizer(marginals, densities, device=self.device).optimize()

    @staticmethod
    def copula_integrations_params(best_t_params):
        """[nu, rho upper triangle...] (student_estimation.py:23-37)."""
        nu = best_t_params["optimized_params"][0]
        corr = np.asarray(best_t_params["corr_matrix"])
        return np.concatenate((np.array([nu]), corr[np.triu_indices_from(corr, k=1)]))

    @staticmethod
    def unpack_copula_params(copula_params):
        """(nu, corr_matrix) (student_estimation.py:40-56)."""
        nu, rho = copula_params[0], copula_params[1:]
        n = int((1 + np.sqrt(1 + 8 * len(rho))) / 2)
        corr = np.eye(n)
        corr[np.triu_indices(n, k=1)] = rho
        corr[np.tril_indices(n, k=-1)] = rho
        return nu, corr

    @staticmethod
    def copula_density(cdf, nu, corr_matrix, **kwargs):
        return copulas.student(cdf, nu, corr_matrix)
