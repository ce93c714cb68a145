"""Static quadrature tables and per-date table assembly (host side, O(T*S)).

These are the small, non-iterative pieces of the reference's
``integration_params_retrieval`` (msm_estimation.py:123-137,
garch_estimation.py:133-145, mean_reverting_estimation.py:135-147).  The heavy
part -- one filter run per (date, asset) window -- runs on the GPU
(``engine.msm_filter`` / ``garch_forecast`` / ``ukf_forecast``).
"""
from __future__ import annotations

import itertools
from typing import List, Sequence, Tuple

import numpy as np

from . import engine


def insample_split(returns: np.ndarray, n_in: int, weights: np.ndarray):
    """load_data.py:105-137: in-sample column means (pandas: contiguous pairwise sum /
    count), ptf_mean, centred series.  Returns (mean (dim,), ptf_mean, centred
    (n_in + T, dim), T).  Window t is centred[t : t + n_in]."""
    r = np.asarray(returns, dtype=np.float64)
    T = r.shape[0] - n_in
    if T <= 0:
        raise ValueError(f"Not enough returns after the start date for in-sample estimation. "
                         f"Required: {n_in}, Available: {r.shape[0]}")
    mean = np.array([np.ascontiguousarray(r[:n_in, d]).sum() / n_in for d in range(r.shape[1])])
    ptf_mean = float(np.sum(mean * np.asarray(weights)))
    return mean, ptf_mean, r - mean, T


def x_grid(num_points: int, model: str, x_min=-5, x_max=5) -> Tuple[np.ndarray, np.ndarray]:
    """compute_normal_densities grids (msm_estimation.py:300-319; garch_estimation.py:166-183)."""
    if model == "msm":
        outer, middle = num_points // 4, num_points // 7
    else:
        outer, middle = num_points // 8, num_points // 5
    central = num_points - 2 * outer - 2 * middle
    x = np.concatenate([
        np.linspace(x_min, -2.5, outer, endpoint=False),
        np.linspace(-2.5, -1, middle, endpoint=False),
        np.linspace(-1, 1, central, endpoint=False),
        np.linspace(1, 2.5, middle, endpoint=False),
        np.linspace(2.5, x_max, outer, endpoint=True),
    ])
    step = np.diff(x, prepend=x[0])
    step[0] = step[1]                                                     # Q18
    return x, step


def msm_vol_states(k: int, m0: float, sig: float) -> np.ndarray:
    """sqrt(prod M_s) * sigma for the 2**k states (calc_prob.py:86-89, 103-108)."""
    M = np.array(list(itertools.product([m0, 2 - m0], repeat=k)))
    return np.array([np.sqrt(np.prod(M[i])) * sig for i in range(M.shape[0])])


def unique_vol_map(vol_state_array: np.ndarray, tol: float = 1e-6):
    """The state -> unique-vol index map of sum_forecast_by_state (msm_estimation.py:228-235):
    (state_map (dim, S) int32, unique_vol_states (dim, q))."""
    maps, uniq = [], []
    for i in range(vol_state_array.shape[0]):
        rounded = np.round(vol_state_array[i, :] / tol) * tol
        u, inv = np.unique(rounded, return_inverse=True)
        maps.append(inv.astype(np.int32))
        uniq.append(u)
    return np.array(maps), np.array(uniq)


def sum_forecast_by_state(vol_state_array: np.ndarray, filtered: np.ndarray, tol: float = 1e-6):
    """msm_estimation.py:205-248: collapse states with equal (1e-6-rounded) vol (Q14).
    filtered (dim, T, S) -> forecasts_by_states (T, dim, q), unique_vol_states (dim, q)."""
    summed, uniq = [], []
    for i in range(vol_state_array.shape[0]):
        rounded = np.round(vol_state_array[i, :] / tol) * tol
        u, inv = np.unique(rounded, return_inverse=True)
        summed.append(np.stack([filtered[i][:, inv == j].sum(axis=1) for j in range(len(u))], axis=1))
        uniq.append(u)
    return np.array(summed).transpose(1, 0, 2), np.array(uniq)


def vol_combinations(dim: int, q: int) -> np.ndarray:
    """create_vol_combinations (msm_estimation.py:369-389), ij order."""
    g = np.meshgrid(*[np.arange(q) for _ in range(dim)], indexing="ij")
    return np.stack(g, axis=-1).reshape(-1, dim)


def forecast_combinations(fbs: np.ndarray) -> np.ndarray:
    """compute_forecast_combinations (msm_estimation.py:392-418), vectorised over T with
    the reference's xy-meshgrid product order (2-D matches the combos; 3-D is permuted, Q7)."""
    T, dim, q = fbs.shape
    grids = np.meshgrid(*[np.arange(q) for _ in range(dim)])             # xy indexing, as :413
    idx = np.array(grids).T.reshape(-1, dim)                              # combination -> per-axis index
    out = fbs[:, 0, idx[:, 0]]
    for d in range(1, dim):
        out = out * fbs[:, d, idx[:, d]]
    return out


def msm_densities(unique_vol_states: np.ndarray, x: np.ndarray) -> np.ndarray:
    """densities[i, j, :] (msm_estimation.py:322-328)."""
    dim, q = unique_vol_states.shape
    d = np.zeros((dim, q, x.size))
    for i in range(dim):
        for j in range(q):
            s = unique_vol_states[i, j]
            d[i, j, :] = (1 / (np.sqrt(2 * np.pi) * s)) * np.exp(-0.5 * (x / s) ** 2)
    return d


def msm_integration_params(centred: np.ndarray, n_in: int, params: Sequence[dict], k: int, num_points: int,
                           device: int = 0):
    """MSMEstimation.integration_params_retrieval with the Hamilton filters on the GPU.

    centred (n_in + T, dim).  Returns (integrations_params_t, integrations_params_static,
    grids_generations_params) exactly as the reference lays them out."""
    dim = centred.shape[1]
    filt = np.array([engine.msm_filter(centred[:-1, d], n_in, k, p["m_0"], p["sig"], p["b"], p["gamma"], device)
                     for d, p in enumerate(params)])                      # (dim, T, S)
    vsa = np.array([msm_vol_states(k, p["m_0"], p["sig"]) for p in params])
    fbs, uvs = sum_forecast_by_state(vsa, filt)
    x, step = x_grid(num_points, "msm")
    dens = msm_densities(uvs, x)
    combos = vol_combinations(dim, uvs.shape[1])
    pi = forecast_combinations(fbs)
    return (fbs, pi), uvs, (dens, x, step, combos)


def sigma_integration_params(centred: np.ndarray, n_in: int, model: str, params: Sequence[dict],
                             num_points: int, device: int = 0):
    """Garch/MeanRevertingEstimation.integration_params_retrieval with device filters."""
    dim = centred.shape[1]
    sig = np.empty((centred.shape[0] - n_in, dim))
    for d, p in enumerate(params):
        if model == "garch" and "pq" in p:
            sig[:, d] = engine.garch_forecast_pq(centred[:-1, d], n_in, p["pq"][0], p["pq"][1], p["params"], device)
        elif model == "garch":
            sig[:, d] = engine.garch_forecast(centred[:-1, d], n_in, p["omega"], p["alpha"], p["beta"], device)
        else:
            sig[:, d] = engine.ukf_forecast(centred[:-1, d], n_in, p["a"], p["l"], p["q"], device)
    x, step = x_grid(num_points, model)
    dens = np.ones((dim, 1, num_points))
    combos = np.zeros((1, dim))
    return [sig], None, (dens, x, step, combos)
