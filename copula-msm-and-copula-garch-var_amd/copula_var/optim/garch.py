"""GARCH(p, q) order search + Newton-Raphson fit (garch/opti.py:7-208) with the
likelihoods on the device.

The reference evaluates the negative log-likelihood point by point in Python
(garch/opti.py:20-37 -> garch/estimation.py:91-125): per Newton step the
central-difference gradient and its finite-difference "Hessian" (opti.py:39-87)
need 2n + 3n + 4 n(n-1)/2 evaluations at n = 1 + p + q parameters.  Every one of
them is the likelihood at the current point or at one coordinate moved by
+-epsilon (the mixed "derivatives" of opti.py:79-85 reuse single-coordinate
moves), so a step needs only the 1 + 2n distinct values: they are computed by
ONE batched launch (cvq_garch_loglik_pq, one thread per parameter row) and the
gradient / Hessian are assembled on the host exactly as opti.py does.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from .. import engine


class GarchOptimizer:
    """garch/opti.py:GarchOptimizer with the same constructor, methods and results.

    loglik(rows, p, q) -> log-likelihoods of parameter rows (B, 1 + p + q); default:
    the device kernel.  Tests pass the CPU oracle here to check the host logic alone.
    """

    def __init__(self, returns, p_max=3, q_max=3, tol=1e-10, max_iter=1000, epsilon=1e-5, device: int = 0,
                 loglik: Optional[Callable] = None, verbose: bool = False):
        self.returns = np.ascontiguousarray(returns, dtype=np.float64)
        self.p_max = p_max
        self.q_max = q_max
        self.best_pq = None
        self.best_params = None
        self.best_result = None
        self.best_bic = None
        self.tol = tol
        self.max_iter = max_iter
        self.epsilon = epsilon
        self.device = device
        self.verbose = verbose
        self._loglik = loglik or (lambda rows, p, q: engine.garch_loglik_pq(self.returns, p, q, rows, self.device))
        self.evaluations = 0          # likelihood rows evaluated
        self.launches = 0             # batched likelihood calls

    # -- likelihood ------------------------------------------------------------------
    def _nll_rows(self, rows: np.ndarray, p: int, q: int) -> np.ndarray:
        """negative_log_likelihood (opti.py:20-37) of every row; one batched call."""
        rows = np.atleast_2d(np.asarray(rows, dtype=np.float64))
        out = np.full(rows.shape[0], 1e10)
        ok = np.array([np.sum(r[1:p + 1]) + np.sum(r[p + 1:]) < 1 for r in rows])   # :30-31 penalty
        if ok.any():
            live = rows[ok]
            # ProbEstimation.verify_params (garch/estimation.py:22-38) raises on these
            if (live[:, 0] <= 0).any() or (live[:, 1:] <= 0).any():
                raise ValueError("GARCH parameters must be positive (garch/estimation.py:29-34)")
            out[ok] = -np.asarray(self._loglik(live, p, q), dtype=np.float64)
            self.evaluations += int(ok.sum())
            self.launches += 1
        return out

    def negative_log_likelihood(self, params, p, q):
        return float(self._nll_rows(np.asarray(params, dtype=np.float64)[None, :], p, q)[0])

    def _stencil(self, params, p, q):
        """f(x), f(x + eps e_i), f(x - eps e_i) for all i, from one launch."""
        n = len(params)
        rows = np.repeat(np.asarray(params, dtype=np.float64)[None, :], 1 + 2 * n, axis=0)
        for i in range(n):
            rows[1 + i, i] += self.epsilon                                  # params_step_up[i] += eps
            rows[1 + n + i, i] -= self.epsilon                              # params_step_down[i] -= eps
        f = self._nll_rows(rows, p, q)
        return f[0], f[1:1 + n], f[1 + n:]

    def numerical_gradient(self, params, p, q):
        """opti.py:39-53."""
        _, up, dn = self._stencil(params, p, q)
        return (up - dn) / (2 * self.epsilon)

    def _grad_hess(self, params, p, q):
        f0, up, dn = self._stencil(params, p, q)
        n = len(params)
        grad = np.zeros_like(np.asarray(params, dtype=np.float64))
        for i in range(n):
            grad[i] = (up[i] - dn[i]) / (2 * self.epsilon)                  # opti.py:50-51
        hess = np.zeros((n, n))
        for i in range(n):                                                  # opti.py:59-85
            for j in range(i, n):
                if i == j:
                    hess[i, i] = (up[i] - 2 * f0 + dn[i]) / (self.epsilon ** 2)
                else:
                    hess[i, j] = hess[j, i] = (up[i] - up[j] - dn[i] + dn[j]) / (4 * self.epsilon ** 2)
        return grad, hess

    def numerical_hessian(self, params, p, q):
        return self._grad_hess(params, p, q)[1]

    # -- optimiser -------------------------------------------------------------------
    def newton_raphson(self, initial_params, p, q):
        """opti.py:139-172."""
        params = np.array(initial_params)
        for _ in range(self.max_iter):
            grad, hess = self._grad_hess(params, p, q)
            try:
                hess_inv = np.linalg.pinv(hess)
            except np.linalg.LinAlgError:
                return None, None
            delta_params = -hess_inv @ grad
            params += delta_params
            sum_rest = np.sum(params[1:])
            if sum_rest > 1:
                params[1:] = params[1:] / sum_rest
            params = np.maximum(params, self.epsilon + 1e-7)
            if np.linalg.norm(delta_params) < self.tol:
                break
        return params, self.negative_log_likelihood(params, p, q)

    def bic(self, log_likelihood, n_obs, num_params):
        """opti.py:174-181."""
        return -2 * log_likelihood + num_params * np.log(n_obs)

    def optimize(self):
        """opti.py:89-137: Newton-Raphson per (p, q), lowest BIC wins (first on ties)."""
        best_result = best_params = best_pq = best_bic = None
        n_obs = len(self.returns)
        for p in range(1, self.p_max + 1):
            for q in range(1, self.q_max + 1):
                alpha_beta_sum = 0.5 / (p + q)
                initial_guess = [0.1] + [alpha_beta_sum] * p + [alpha_beta_sum] * q
                params, neg_log_likelihood = self.newton_raphson(initial_guess, p, q)
                if params is None:
                    if self.verbose:
                        print(f"Failed to converge for p={p}, q={q}")
                    continue
                current_bic = self.bic(-neg_log_likelihood, n_obs, 1 + p + q)
                if best_result is None or current_bic < best_bic:
                    best_result, best_params, best_pq, best_bic = neg_log_likelihood, params, (p, q), current_bic
                if self.verbose:
                    print(f"p = {p}, q = {q}, -Log-Likelihood = {neg_log_likelihood}, BIC = {current_bic}")
        self.best_pq, self.best_params, self.best_result, self.best_bic = best_pq, best_params, best_result, best_bic
        return self.best_pq, self.best_params, self.best_result, self.best_bic

    def unpack_garch_parameters(self, result):
        """opti.py:183-208."""
        (p, q), params = result[0], result[1]
        return params[0], np.array(params[1:p + 1]), np.array(params[p + 1:p + 1 + q])
