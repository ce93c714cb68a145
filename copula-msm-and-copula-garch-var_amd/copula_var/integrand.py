"""The reference's per-node integrands, ``integrated_function`` of the model adapters.

The VaR path never calls these: the device solve evaluates the integrand inside its kernels
(k_compact / k_sorted / k_direct).  They keep the plug-in surface so code
written against the reference's adapters -- a custom quadrature driving
``adapter.integrated_function(grids, step_sizes, copula_params, integrations_params_i,
integrations_params_static, copula_density, unpack_copula_params)`` over its own nested grid
-- keeps working, with the same arguments, shapes and semantics:

* MSM   (utils/calc_integral/integration_functions/msm_integration_function.py:5-47):
  u_d = sum_s f[d, s] Phi(x_d / sigma~[d, s]); c = copula_density(cdf=u, nu=, corr_matrix=);
  returns sum_P c * step_sizes (P, Q) over the nodes, times the forecast combinations (Q,)
  -- the reference sums over the nodes first, then over the combinations (its caller,
  multi_integral_function, integration_algo.py:84, takes np.sum of the result);
* GARCH / UKF (garch_integration_function.py:5-52): u_d = Phi(x_d / sigma_d),
  returns nan_to_num(c * prod_d phi(x_d / sigma_d) / sigma_d) (P, 1) * step_sizes.

Phi is the reference's erf form (utils/utils.py:4-22, Q16) with erf evaluated on the GPU
(cvq_special), like the quantile transforms inside ``copula_density`` (copulas.py); the rest
is a few numpy array expressions around those device calls.
"""
from __future__ import annotations

import numpy as np

from . import _native as N


def norm_cdf(x, device: int = 0):
    """norm_cdf_array (utils/utils.py:4-22): 0.5 (1 + erf(z / sqrt 2)), erf on the device."""
    z = np.asarray(x, dtype=np.float64)
    return 0.5 * (1 + N.special("erf", z / np.sqrt(2), device=device))


def norm_pdf(x):
    """norm_pdf_array (utils/utils.py:24-42)."""
    z = np.asarray(x, dtype=np.float64)
    return (1 / (1 * np.sqrt(2 * np.pi))) * np.exp(-0.5 * z ** 2)


def _column(c, P):
    """manual_reshape(c, (P, 1)) (utils/utils.py:45-69): the first P values as a column."""
    return np.asarray(c, dtype=np.float64).reshape(-1)[:P].reshape(P, 1)


def msm_integrated_function(grids, step_sizes, copula_params, integrations_params_i, integrations_params_static,
                            copula_density, unpack_copula_params, device: int = 0):
    """msm_integration_function.py:5-47.  grids (P, dim); step_sizes (P, Q) Delta products;
    integrations_params_i = [forecasts_by_states (dim, q), forecasts (Q,)];
    integrations_params_static = unique_vol_states (dim, q).  Returns (Q,)."""
    forecasts_by_states = np.asarray(integrations_params_i[0], dtype=np.float64)
    forecasts = np.asarray(integrations_params_i[1], dtype=np.float64)
    nu, corr_matrix = unpack_copula_params(copula_params)
    g = np.asarray(grids, dtype=np.float64)
    num_points = g.shape[0]
    uvs = np.asarray(integrations_params_static, dtype=np.float64)
    x = g[:, :, np.newaxis] / uvs[np.newaxis, :, :]
    cdf = np.sum(forecasts_by_states * norm_cdf(x, device), axis=2)
    dens = copula_density(cdf=cdf, nu=nu, corr_matrix=corr_matrix)
    return np.sum(_column(dens, num_points) * np.asarray(step_sizes, dtype=np.float64), axis=0) * forecasts


def sigma_integrated_function(grids, step_sizes, copula_params, integrations_params_i, integrations_params_static,
                              copula_density, unpack_copula_params, device: int = 0):
    """garch_integration_function.py:5-52 (GARCH and UKF).  grids (P, dim); step_sizes (P, 1);
    integrations_params_i = sigma forecasts (dim,).  Returns (P, 1)."""
    forecasted_vol = np.asarray(integrations_params_i, dtype=np.float64)
    nu, corr_matrix = unpack_copula_params(copula_params)
    g = np.asarray(grids, dtype=np.float64)
    num_points = g.shape[0]
    x = g / forecasted_vol
    cdf = norm_cdf(x, device)
    pdf = norm_pdf(x) / forecasted_vol
    density_prod = np.prod(pdf, axis=1)
    dens = copula_density(cdf=cdf, nu=nu, corr_matrix=corr_matrix)
    with np.errstate(invalid="ignore", over="ignore"):
        density_func = np.nan_to_num(_column(np.asarray(dens) * density_prod, num_points))
    return density_func * np.asarray(step_sizes, dtype=np.float64)
