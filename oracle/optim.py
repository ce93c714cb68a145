"""CPU restatement of the in-sample optimiser layer -- TEST INFRASTRUCTURE ONLY.

* garch_loglik_pq: numba_garch_log_likelihood (garch/estimation.py:91-125) for any
  (p, q), including the chopped max(p, q) prefix and np.sum's summation order.
* ukf_filter_batch: the VolOptimizer E-step (UKF LL + state path) per parameter row.
* the optimiser logic itself is the product's (copula_var/optim/garch.py); the
  tests drive it with this CPU likelihood as well as with the device one, and pin
  both against the reference's own GarchOptimizer results (tests/golden/
  gen_optim_golden.py).
"""
from __future__ import annotations

import numpy as np


def garch_loglik_pq(returns: np.ndarray, omega: float, alpha, beta, epsilon: float = 1e-7) -> float:
    """garch/estimation.py:91-125, line by line (sigma2[0] unclamped, max(., eps) after)."""
    r = np.asarray(returns, dtype=np.float64)
    alpha, beta = np.asarray(alpha, dtype=np.float64), np.asarray(beta, dtype=np.float64)
    n, p, q = r.size, alpha.size, beta.size
    m = max(p, q)
    s2 = np.zeros(n)
    s2[0] = omega / (1 - np.sum(alpha) - np.sum(beta))                      # :106
    for t in range(1, n):                                                  # :109-116
        v = omega
        for i in range(min(p, t)):
            v += alpha[i] * (r[t - i - 1] ** 2)
        for j in range(min(q, t)):
            v += beta[j] * s2[t - j - 1]
        s2[t] = max(v, epsilon)
    rc, sc = r[m:], s2[m:]                                                 # :119-121
    return float(-0.5 * np.sum(np.log(2 * np.pi * sc) + (rc ** 2) / sc))  # :124


def garch_loglik_batch(returns: np.ndarray, params: np.ndarray, p: int, q: int) -> np.ndarray:
    P = np.atleast_2d(np.asarray(params, dtype=np.float64))
    return np.array([garch_loglik_pq(returns, row[0], row[1:p + 1], row[p + 1:p + 1 + q]) for row in P])


def garch_forecast_pq(window: np.ndarray, omega: float, alpha, beta, epsilon: float = 1e-7) -> float:
    """garch/forecast.py:5-19 (calc_forecast) for any (p, q): estimation.py:40-65 variances,
    then sqrt(omega + sum(alpha * returns[-p:]**2) + sum(beta * sigma2[-q:]))."""
    r = np.asarray(window, dtype=np.float64)
    alpha, beta = np.asarray(alpha, dtype=np.float64), np.asarray(beta, dtype=np.float64)
    p, q = alpha.size, beta.size
    s2 = np.zeros(r.size)
    s2[0] = omega / (1 - sum(alpha) - sum(beta))
    for t in range(1, r.size):
        s2[t] = omega
        for i in range(min(p, t)):
            s2[t] += alpha[i] * (r[t - i - 1] ** 2)
        for j in range(min(q, t)):
            s2[t] += beta[j] * s2[t - j - 1]
        s2[t] = max(s2[t], epsilon)
    return float(np.sqrt(omega + np.sum(alpha * r[-p:] ** 2) + np.sum(beta * s2[-q:])))


def ukf_filter_batch(returns: np.ndarray, params: np.ndarray):
    """VolOptimizer.e_step (kalman_mean_reverting/optimize.py:28-32 -> estimate.py:230-281,
    init (l, q)) per row: returns (B, N) or (N,), params (B, 3) -> (LL with -1e10 on
    failure, state paths (B, N) NaN on failure), the layout of engine.ukf_filter."""
    from .forecast import ukf_run
    P = np.atleast_2d(np.asarray(params, dtype=np.float64))
    R = np.asarray(returns, dtype=np.float64)
    R = np.broadcast_to(R, (P.shape[0], R.shape[-1]))
    ll, st = np.empty(P.shape[0]), np.empty((P.shape[0], R.shape[1]))
    for b, (a, l, q) in enumerate(P):
        _, LL, state, failed = ukf_run(R[b][None, :], a, l, q)
        ll[b] = -1e10 if failed[0] else LL[0]
        st[b] = np.nan if failed[0] else state[0]
    return ll, st
