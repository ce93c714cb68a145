"""CPU restatement of the copula IFM objectives -- TEST INFRASTRUCTURE ONLY.

Scalar loops in the reference's own structure, so the product's vectorised,
device-quantile version (copula_var/optim/copula_fit.py) has an independent check:

* student_nll: copulas/student/opti.py:34-64 -> inference_for_margins.py:38-55 ->
  student.py:49-174 (scalar scipy t.ppf per entry, per-sample quadratic form, 0 pdf
  for non-finite quantiles).
* gaussian_nll: copulas/gaussian/opti.py:30-56 -> inference_for_margins.py:34-53 ->
  gaussian.py:43-117 (pdf floored at 1e-10).
* plackett_nll: copulas/plackett/opti.py:28-42 -> inference_for_margins.py:32-49 ->
  plackett.py:35-71.

PARITY UNPINNED for the fits themselves: running the reference's copula optimisers
in the build container to record golden fits was refused, so these
restatements are checked against the product on seeded samples, not against
reference outputs.  The copula densities they use are the ones the VaR goldens pin
(oracle/quadrature.py evaluates the same formulas inside the integrand).
"""
from __future__ import annotations

from math import gamma

import numpy as np
from scipy.linalg import cholesky
from scipy.stats import norm, t


def _corr(dim, corr_params):
    """student/opti.py:66-85."""
    c = np.eye(dim)
    idx = 0
    for i in range(dim):
        for j in range(i):
            c[i, j] = c[j, i] = corr_params[idx]
            idx += 1
    return c


def _bad(c) -> bool:
    if np.isnan(c).any() or np.isinf(c).any():
        return True
    try:
        cholesky(c)
    except np.linalg.LinAlgError:
        return True
    return False


def student_nll(marginals, densities, params) -> float:
    u, dens = np.asarray(marginals, dtype=np.float64), np.asarray(densities, dtype=np.float64)
    n, d = u.shape
    nu, c = float(params[0]), _corr(d, params[1:])
    if _bad(c):
        return 1e10
    z = np.zeros((n, d))
    for i in range(n):                                              # student.py:100-102
        for j in range(d):
            z[i, j] = t.ppf(u[i, j], df=nu)
    inv, det = np.linalg.inv(c), np.linalg.det(c)
    term1 = gamma((nu + d) / 2) / (gamma(nu / 2) * ((nu * np.pi) ** (d / 2)) * np.sqrt(det))
    g = gamma((nu + 1) / 2) / (np.sqrt(nu * np.pi) * gamma(nu / 2))
    logc = np.zeros(n)
    with np.errstate(divide="ignore", invalid="ignore"):
        for i in range(n):
            x = z[i]
            mv = 0.0 if not np.all(np.isfinite(x)) else term1 * (1 + np.dot(np.dot(x, inv), x) / nu) ** (-(nu + d) / 2)
            prod = 1.0
            for j in range(d):
                prod *= 0.0 if not np.isfinite(x[j]) else g * (1 + x[j] ** 2 / nu) ** (-(nu + 1) / 2)
            logc[i] = np.log(np.float64(mv) / np.float64(prod))
        return -(np.sum(np.sum(np.log(dens))) + np.sum(logc))


def gaussian_nll(marginals, densities, corr_params) -> float:
    u, dens = np.asarray(marginals, dtype=np.float64), np.asarray(densities, dtype=np.float64)
    n, d = u.shape
    c = _corr(d, corr_params)
    if _bad(c):
        return 1e10
    z = norm.ppf(u)                                                 # gaussian.py:43-44
    inv, det = np.linalg.inv(c), np.linalg.det(c)
    pdf = np.zeros(n)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        for i in range(n):
            x = z[i]
            mv = (1 / np.sqrt((2 * np.pi) ** d * det)) * np.exp(-0.5 * np.dot(np.dot(x, inv), x))
            prod = 1.0
            for j in range(d):
                prod *= (1 / np.sqrt(2 * np.pi)) * np.exp(-0.5 * x[j] ** 2)
            pdf[i] = mv / prod
        pdf = np.maximum(pdf, 1e-10)                                # inference_for_margins.py:48
        return -(np.sum(np.sum(np.log(dens))) + np.sum(np.log(pdf)))


def plackett_nll(marginals, densities, theta) -> float:
    u, dens = np.asarray(marginals, dtype=np.float64), np.asarray(densities, dtype=np.float64)
    th = float(np.asarray(theta).reshape(-1)[0])
    pdf = np.zeros(u.shape[0])
    with np.errstate(divide="ignore", invalid="ignore"):
        for i in range(u.shape[0]):                                 # plackett.py:65-69
            a, b = u[i, 0], u[i, 1]
            num = th * (1 + (th - 1) * (a + b - 2 * a * b))
            den = ((1 + (th - 1) * (a + b)) * (1 + (th - 1) * (1 - a - b))) ** 2
            pdf[i] = num / den
        return -(np.sum(np.log(dens)) + np.sum(np.log(pdf)))


def student_sample(n, dim, nu, rho, seed):
    """Seeded Student-t copula sample: u = t.cdf(x, nu), densities = t.pdf(x, nu)."""
    rng = np.random.default_rng(seed)
    R = np.full((dim, dim), rho) + (1 - rho) * np.eye(dim)
    g = rng.standard_normal((n, dim)) @ np.linalg.cholesky(R).T
    x = g / np.sqrt(rng.chisquare(nu, size=(n, 1)) / nu)
    return t.cdf(x, nu), t.pdf(x, nu)
