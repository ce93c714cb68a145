"""Copula fits by inference for margins (copulas/{student,gaussian,plackett}/opti.py)
with the quantile transforms on the device.

The reference's Student objective (student/opti.py:34-64 -> inference_for_margins.py:38-55
-> student.py:49-174) spends most of its time in a scalar ``scipy.stats.t.ppf`` loop
over the N x dim marginals (student.py:96-102).  Here one device
launch (cvq_special "tppf", the VaR path's stdtrit) returns all N x dim quantiles
of a candidate nu; Gaussian uses the device ``ndtri`` the same way.  The densities
and the log-sums follow the reference's formulas (copula_var.copulas).  The
optimiser control flow (L-BFGS-B sweeps, bounds, starting points, result dicts)
is the reference's, on scipy.optimize.minimize.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
from scipy.linalg import cholesky
from scipy.optimize import minimize

from .. import _native as N
from ..copulas import gaussian_from_quantiles, plackett, student_from_quantiles


def construct_correlation_matrix(dim, corr_params):
    """student/opti.py:66-85 == gaussian/opti.py:58-77 (lower triangle, row by row)."""
    corr_matrix = np.eye(dim)
    idx = 0
    for i in range(dim):
        for j in range(i):
            corr_matrix[i, j] = corr_params[idx]
            corr_matrix[j, i] = corr_params[idx]
            idx += 1
    return corr_matrix


def _invalid(corr_matrix) -> bool:
    """1e10 guard of student/opti.py:44-52, gaussian/opti.py:37-45."""
    if np.isnan(corr_matrix).any() or np.isinf(corr_matrix).any():
        return True
    try:
        cholesky(corr_matrix)
    except np.linalg.LinAlgError:
        return True
    return False


class _IFM:
    def __init__(self, marginals, densities, tol, max_iter, device):
        self.marginals = np.array(marginals, dtype=np.float64)
        self.densities = np.array(densities, dtype=np.float64)
        if len(self.marginals) != len(self.densities):               # inference_for_margins.py verify_sizes
            raise ValueError("Marginals and densities must have the same length.")
        self.N = self.marginals.shape[0]
        self.dim = self.marginals.shape[1]
        self.tol = tol
        self.max_iter = max_iter
        self.device = device
        self._log_dens = np.sum(np.sum(np.log(self.densities)))
        self.launches = 0

    def construct_correlation_matrix(self, corr_params):
        return construct_correlation_matrix(self.dim, corr_params)


class StudentCopulaOptimizer(_IFM):
    """student/opti.py:Optimizer (same constructor, objective and two-stage optimize)
    with the quantiles of each candidate nu from one device launch.

    tppf(u, nu) -> Student-t quantiles of u (any shape); default the device kernel.
    Tests pass scipy's t.ppf to replay the reference on the CPU.
    """

    def __init__(self, marginals, densities, nu_values=np.linspace(2.1, 30, 10), tol=1e-9, max_iter=5000,
                 device: int = 0, tppf: Optional[Callable] = None, verbose: bool = False):
        super().__init__(marginals, densities, tol, max_iter, device)
        self.nu_values = nu_values
        self.verbose = verbose
        self._tppf = tppf or (lambda u, nu: N.special("tppf", u, nu=nu, device=self.device))

    def negative_log_likelihood(self, params):
        """student/opti.py:34-64 -> inference_for_margins.py:38-55."""
        params = np.asarray(params, dtype=np.float64).ravel()
        nu = float(params[0])
        corr_matrix = self.construct_correlation_matrix(params[1:])
        if _invalid(corr_matrix):
            return 1e10
        z = np.asarray(self._tppf(self.marginals, nu), dtype=np.float64)   # student.py:96-102, one launch
        self.launches += 1
        with np.errstate(divide="ignore", invalid="ignore"):
            total = self._log_dens + np.sum(np.log(student_from_quantiles(z, nu, corr_matrix)))
        return -total

    def optimize(self, initial_corr=None, method="L-BFGS-B"):
        """student/opti.py:87-184: correlations by `method` for each nu in nu_values
        (bounds (-0.99, 0.99)), then nu from 10 (bounds (2.01, 50)) with the best ones."""
        best_nll, best_corr_params = np.inf, None
        n_corr = (self.dim * (self.dim - 1)) // 2
        if initial_corr is None:
            initial_corr = np.full(n_corr, 0.5)
        corr_bounds = [(-0.99, 0.99)] * n_corr
        nu_bounds = [(2.01, 50)]
        for nu in self.nu_values:
            res_corr = minimize(fun=lambda c: self.negative_log_likelihood(np.hstack(([nu], c))), x0=initial_corr,
                                method=method, bounds=corr_bounds, tol=self.tol, options={"maxiter": self.max_iter})
            nll_corr = self.negative_log_likelihood(np.hstack(([nu], res_corr.x)))
            if self.verbose:
                print(f"Negative Log-Likelihood for nu={nu}: {nll_corr}")
            if nll_corr < best_nll:
                best_nll, best_corr_params = nll_corr, res_corr.x
        if best_corr_params is None:
            # the reference goes on with None and fails in np.hstack / construct_correlation_matrix
            raise ValueError("Student copula fit: the negative log-likelihood is NaN for every nu "
                             "(a marginal at exactly 0 or 1 has an infinite t quantile, student.py:133-172)")
        res_nu = minimize(fun=lambda v: self.negative_log_likelihood(np.hstack((v, best_corr_params))), x0=[10],
                          method=method, bounds=nu_bounds, tol=self.tol, options={"maxiter": self.max_iter})
        optimized_nu = np.array([res_nu.x[0]])
        final_nll = self.negative_log_likelihood(np.hstack((optimized_nu, best_corr_params)))
        return {"nu": optimized_nu, "corr_matrix": self.construct_correlation_matrix(best_corr_params),
                "nll": final_nll, "optimized_params": np.hstack((optimized_nu, best_corr_params))}


Optimizer = StudentCopulaOptimizer          # the reference's class name (copulas/student/opti.py:8)


class GaussianCopulaOptimizer(_IFM):
    """gaussian/opti.py:GaussianCopulaOptimizer; the norm.ppf quantiles (gaussian.py:43-44)
    are computed once on the device -- they do not depend on the correlations."""

    def __init__(self, marginals, densities, tol=1e-9, max_iter=5000, device: int = 0,
                 ndtri: Optional[Callable] = None):
        super().__init__(marginals, densities, tol, max_iter, device)
        self._ndtri = ndtri or (lambda u: N.special("ndtri", u, device=self.device))
        self._z = None

    def negative_log_likelihood(self, corr_params):
        """gaussian/opti.py:30-56 -> inference_for_margins.py:34-53 (copula pdf floored at 1e-10)."""
        corr_matrix = self.construct_correlation_matrix(np.asarray(corr_params, dtype=np.float64).ravel())
        if _invalid(corr_matrix):
            return 1e10
        if self._z is None:
            self._z = np.asarray(self._ndtri(self.marginals), dtype=np.float64)
            self.launches += 1
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            copula_pdf = np.maximum(gaussian_from_quantiles(self._z, corr_matrix), 1e-10)
            total = self._log_dens + np.sum(np.log(copula_pdf))
        return -total

    def optimize(self, initial_corr=None, method="L-BFGS-B"):
        """gaussian/opti.py:79-128."""
        n_corr = (self.dim * (self.dim - 1)) // 2
        if initial_corr is None:
            initial_corr = np.full(n_corr, 0.5)
        res_corr = minimize(fun=self.negative_log_likelihood, x0=initial_corr, method=method,
                            bounds=[(-0.99, 0.99)] * n_corr, tol=self.tol, options={"maxiter": self.max_iter})
        optimized_corr_params = res_corr.x
        final_nll = self.negative_log_likelihood(optimized_corr_params)
        return {"corr_matrix": self.construct_correlation_matrix(optimized_corr_params), "nll": final_nll,
                "optimized_params": optimized_corr_params}


class PlackettCopulaOptimizer(_IFM):
    """plackett/opti.py:PlackettCopulaOptimizer (closed-form density, Q11 formula; no
    quantile transform, so nothing to put on the device)."""

    def __init__(self, marginals, densities, tol=1e-9, max_iter=5000):
        super().__init__(marginals, densities, tol, max_iter, device=0)
        if self.dim != 2:                                              # plackett inference_for_margins.py:29-30
            raise ValueError("Plackett copula is only defined for 2-dimensional marginals.")
        self._log_dens = np.sum(np.log(self.densities))

    def negative_log_likelihood(self, theta):
        """plackett/opti.py:28-42 -> inference_for_margins.py:32-49."""
        with np.errstate(divide="ignore", invalid="ignore"):
            total = self._log_dens + np.sum(np.log(plackett(self.marginals, theta)))
        return -total

    def optimize(self, theta_range=None, method="L-BFGS-B"):
        """plackett/opti.py:44-97: one L-BFGS-B run per starting theta (bounds (0.1, None))."""
        if theta_range is None:
            theta_range = np.linspace(0.5, 50, 10)
        best_nll, best_theta = np.inf, None
        for initial_theta in theta_range:
            res = minimize(fun=self.negative_log_likelihood, x0=[initial_theta], method=method,
                           bounds=[(0.1, None)], tol=self.tol, options={"maxiter": self.max_iter})
            if res.fun < best_nll:
                best_nll, best_theta = res.fun, res.x[0]
        return {"theta": best_theta, "nll": best_nll, "optimized_params": best_theta}
