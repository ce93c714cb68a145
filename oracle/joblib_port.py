"""CPU joblib path -- a structural port of the reference quadrature, for bench.py's
``cpu_baseline`` leg (kind "port") and as a second, independent oracle.

Test/baseline infrastructure only (see oracle/__init__.py).  Unlike
oracle/quadrature.py (which exploits separability), this follows the
reference's own algorithm and cost structure:

* ``np.unique`` of the bounds rows (calc_var_class.py:192);
* one nested grid + Delta-product matrix per unique row (create_grids.py:6-240;
  built vectorised, standing in for the reference's numba recursion);
* one joblib task per date per quadrature call (calc_integral.py:174-225), each
  evaluating the integrand node by node with the copula's own special-function
  calls -- for Student a scalar ``scipy.stats.t.ppf`` loop (student.py:100-102).
"""
from __future__ import annotations

import math

import numpy as np
from joblib import Parallel, delayed
from scipy import special, stats

from .quadrature import BOX_LO, Problem, calc_var, norm_cdf, norm_pdf


def nested_grid(P: Problem, a: float, b: float):
    """Grid points (P_nodes, dim) and Delta-product matrix (P_nodes, Q) for bounds (a, b]."""
    mask = P.inner_mask(a, b)
    idx = np.argwhere(mask)                                   # row-major = the reference's order
    grids = P.x[idx]
    Q = P.combos.shape[0]
    delta = np.ones((idx.shape[0], Q))
    d = P.dim
    for l in range(Q):
        for c in range(d):
            f = P.dens[(c - 1) % d, P.combos[l, c], idx[:, c]] * P.step[idx[:, c]]
            if d == 3 and c == 0:
                f = np.where(idx[:, 1] == 0, f, 1.0)          # Q6
            delta[:, l] *= f
    return grids, delta


def _copula_scalar(copula, cdf, nu, R):
    """copula_density with the reference's per-element special-function calls."""
    if copula == "plackett":
        u, v = cdf[:, 0], cdf[:, 1]
        th = nu
        return th * (1 + (th - 1) * (u + v - 2 * u * v)) / ((1 + (th - 1) * (u + v)) * (1 + (th - 1) * (1 - u - v))) ** 2
    N, d = cdf.shape
    z = np.zeros((N, d))
    if copula == "student":
        for i in range(N):                                     # student.py:100-102
            for j in range(d):
                z[i, j] = stats.t.ppf(cdf[i, j], df=nu)
    else:
        z = stats.norm.ppf(cdf)                                 # gaussian.py:44
    Ri, det = np.linalg.inv(R), np.linalg.det(R)
    mv = np.zeros(N)
    if copula == "student":
        term1 = math.gamma((nu + d) / 2) / (math.gamma(nu / 2) * ((nu * np.pi) ** (d / 2)) * np.sqrt(det))
        g = math.gamma((nu + 1) / 2) / (np.sqrt(nu * np.pi) * math.gamma(nu / 2))
        uni = np.zeros((N, d))
        for i in range(N):
            x = z[i]
            if np.all(np.isfinite(x)):
                mv[i] = term1 * (1 + np.dot(np.dot(x.T, Ri), x) / nu) ** (-(nu + d) / 2)
            for j in range(d):
                uni[i, j] = g * (1 + (z[i, j] ** 2 / nu)) ** (-(nu + 1) / 2) if np.isfinite(z[i, j]) else 0.0
    else:
        term1 = 1 / (np.sqrt((2 * np.pi) ** d * det))
        for i in range(N):
            x = z[i]
            mv[i] = term1 * np.exp(-0.5 * np.dot(np.dot(x.T, Ri), x))
        uni = (1 / np.sqrt(2 * np.pi)) * np.exp(-0.5 * z ** 2)
    with np.errstate(invalid="ignore", divide="ignore"):
        return mv / np.prod(uni, axis=1)


def _date_task(model, copula, nu, R, grids, delta, params_i, uvs):
    """calculate_result_for_i (calc_integral.py:122-171) -> integrated_function."""
    if grids.shape[0] == 0:
        return 0.0
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        if model == "msm":
            fbs, pi = params_i
            x = grids[:, :, None] / uvs[None, :, :]
            cdf = np.sum(fbs * norm_cdf(x), axis=2)
            c = _copula_scalar(copula, cdf, nu, R)
            return float(np.sum(np.sum(c[:, None] * delta, axis=0) * pi))
        sig = params_i
        x = grids / sig
        cdf = norm_cdf(x)
        pdf = norm_pdf(x) / sig
        c = _copula_scalar(copula, cdf, nu, R)
        return float(np.sum(np.nan_to_num((c * np.prod(pdf, axis=1))[:, None]) * delta))


class JoblibPath:
    """compute_integral / calc_var over a Problem with the reference's joblib structure."""

    def __init__(self, P: Problem, n_jobs: int = -1):
        self.P = P
        self.n_jobs = n_jobs
        self._pool = Parallel(n_jobs=n_jobs)

    def compute_integral(self, bounds):
        P = self.P
        uniq, inv = np.unique(bounds, axis=0, return_inverse=True)
        inv = np.asarray(inv).reshape(-1)
        built = [nested_grid(P, a, b) for a, b in uniq]
        if P.model == "msm":
            par = [(P.fbs[t], P.pi[t]) for t in range(P.T)]
        else:
            par = [P.sigma[t] for t in range(P.T)]
        uvs = P.uvs if P.model == "msm" else None
        res = self._pool(delayed(_date_task)(P.model, P.copula, P.nu, P.R, built[inv[t]][0], built[inv[t]][1],
                                             par[t], uvs) for t in range(P.T))
        return np.array(res)

    def calc_var(self, ptf_mean, **kw):
        return calc_var(self.compute_integral, self.P.T, ptf_mean, **kw)
