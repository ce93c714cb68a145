"""CPU restatement of the in-sample optimiser layer -- TEST INFRASTRUCTURE ONLY.

* garch_loglik_pq: numba_garch_log_likelihood (garch/estimation.py:91-125) for any
  (p, q), including the chopped max(p, q) prefix and np.sum's summation order.
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
