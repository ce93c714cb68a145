"""Pointwise copula densities c(u) for the adapters' ``copula_density`` API.

The VaR path never calls these: the device quadrature evaluates the copula
inside its kernels.  They exist so code written against the reference's
adapters (``StudentCopulaVaR.copula_density(cdf=, nu=, corr_matrix=)`` etc.)
keeps working.  The quantile transforms (t.ppf / norm.ppf, the expensive part,
student.py:100-102, gaussian.py:43-44) run on the GPU through cvq_special; the
closed-form density around them is a few numpy array expressions.

Semantics follow the reference, including its edge behaviour: Student density
0 when a quantile is non-finite, so c = 0/0 = NaN at u in {0, 1}
(student.py:133-141, 164-172); Gaussian has no guard (gaussian.py:105-113);
Plackett uses the reference's non-standard formula (Q11, plackett.py:66-69).
"""
from __future__ import annotations

import math

import numpy as np

from . import _native as N


def student(cdf, nu, corr_matrix):
    """copulas/student/student.py:49-174."""
    u = np.asarray(cdf, dtype=np.float64)
    return student_from_quantiles(N.special("tppf", u, nu=float(nu)), nu, corr_matrix)


def student_from_quantiles(z, nu, corr_matrix):
    """student.py:66-79 after the t.ppf step: the multivariate t pdf of the
    quantiles z (P, d) over the product of the univariate t pdfs."""
    P, d = z.shape
    Ri, det = np.linalg.inv(corr_matrix), np.linalg.det(corr_matrix)
    term1 = math.gamma((nu + d) / 2) / (math.gamma(nu / 2) * ((nu * np.pi) ** (d / 2)) * np.sqrt(det))
    g = math.gamma((nu + 1) / 2) / (np.sqrt(nu * np.pi) * math.gamma(nu / 2))
    fin_row = np.all(np.isfinite(z), axis=1)
    zz = np.where(np.isfinite(z), z, 0.0)
    qf = np.einsum("pi,ij,pj->p", zz, Ri, zz)
    mv = np.where(fin_row, term1 * (1 + qf / nu) ** (-(nu + d) / 2), 0.0)
    uni = np.where(np.isfinite(z), g * (1 + zz ** 2 / nu) ** (-(nu + 1) / 2), 0.0)
    with np.errstate(invalid="ignore", divide="ignore"):
        return mv / np.prod(uni, axis=1)


def gaussian(cdf, corr_matrix):
    """copulas/gaussian/gaussian.py:43-117."""
    u = np.asarray(cdf, dtype=np.float64)
    return gaussian_from_quantiles(N.special("ndtri", u), corr_matrix)


def gaussian_from_quantiles(z, corr_matrix):
    """gaussian.py:52-61 after the norm.ppf step."""
    P, d = z.shape
    Ri, det = np.linalg.inv(corr_matrix), np.linalg.det(corr_matrix)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        qf = np.einsum("pi,ij,pj->p", z, Ri, z)
        mv = (1 / np.sqrt((2 * np.pi) ** d * det)) * np.exp(-0.5 * qf)
        uni = (1 / np.sqrt(2 * np.pi)) * np.exp(-0.5 * z ** 2)
        return mv / np.prod(uni, axis=1)


def plackett(cdf, theta):
    """copulas/plackett/plackett.py:35-71 (Q11 formula, columns 0 and 1)."""
    c = np.asarray(cdf, dtype=np.float64)
    u, v = c[:, 0], c[:, 1]
    th = float(np.asarray(theta).reshape(-1)[0])
    num = th * (1 + (th - 1) * (u + v - 2 * u * v))
    den = ((1 + (th - 1) * (u + v)) * (1 + (th - 1) * (1 - u - v))) ** 2
    with np.errstate(invalid="ignore", divide="ignore"):
        return num / den
