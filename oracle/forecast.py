"""Oracle: per-date forecast stage, numpy.

Test infrastructure only (see oracle/__init__.py).  Each window is processed
exactly as the reference processes it -- a fresh filter run over the centred
rolling window -- but all T windows are advanced together as a batch.
"""
from __future__ import annotations

import itertools
import math

import numpy as np

SQRT_2PI = np.sqrt(2 * np.pi)


# --------------------------------------------------------------------------- data
def insample_split(returns: np.ndarray, n_in: int, weights: np.ndarray):
    """Mean / centring / rolling windows of data_loader/load_data.py:105-137.

    returns (n_in + T, dim).  The in-sample mean is pandas' column mean
    (load_data.py:111), i.e. a contiguous pairwise sum divided by the count.
    Returns (mean (dim,), ptf_mean, windows (T, n_in, dim) centred)."""
    r = np.asarray(returns, dtype=np.float64)
    T = r.shape[0] - n_in
    if T <= 0:
        raise ValueError("Not enough returns after the start date for in-sample estimation.")
    mean = np.array([np.ascontiguousarray(r[:n_in, d]).sum() / n_in for d in range(r.shape[1])])
    ptf_mean = float(np.sum(mean * weights))                        # load_data.py:113
    centred = r - mean                                               # load_data.py:133
    idx = np.arange(T)[:, None] + np.arange(n_in)[None, :]           # windows i:i+N (:132)
    return mean, ptf_mean, centred[idx]


# --------------------------------------------------------------------------- MSM
def msm_states(k: int, m0: float):
    """itertools.product([m0, 2-m0], repeat=k)  (calc_prob.py:86-89)."""
    return np.array(list(itertools.product([m0, 2 - m0], repeat=k)))


def msm_transition(k: int, m0: float, b: float, gamma: float):
    """A[i,j] = prod_c (M_ic == M_jc ? p_c : q_c)  (calc_prob.py:91-101)."""
    M = msm_states(k, m0)
    gamma_k = 1 - (1 - gamma) ** (b ** np.arange(M.shape[1]))
    p = 1 - gamma_k / 2
    qv = 1 - p
    return np.prod(np.where(M[:, None, :] == M[None, :, :], p, qv), axis=2)


def msm_vol_states(k: int, m0: float, sig: float):
    """sqrt(prod M_s) * sigma  (calc_prob.py:103-108)."""
    M = msm_states(k, m0)
    return np.array([np.sqrt(np.prod(M[i])) * sig for i in range(M.shape[0])])


def msm_filtered_probs(windows: np.ndarray, k: int, m0: float, sig: float, b: float, gamma: float):
    """Filtered state probabilities at each window's last step
    (calc_marginals.py:33-38 -> calc_prob.py:8-32, 51-69, 110-120).

    windows (T, N).  Returns (T, 2**k)."""
    A = msm_transition(k, m0, b, gamma)
    vs = msm_vol_states(k, m0, sig)
    S = vs.size
    T, N = windows.shape
    prev = np.full((T, S), 1 / S)
    for i in range(N):
        r = windows[:, i][:, None]
        cond = (1 / (vs[None, :] * np.sqrt(2 * np.pi))) * np.exp(-0.5 * (r / vs[None, :]) ** 2)
        tp = prev @ A.T                                              # calc_prob.py:56-57
        prob = tp * cond
        scale = prob.sum(axis=1, keepdims=True)
        if np.any(scale == 0):
            raise FloatingPointError("MSM Bayes update normaliser is 0 (calc_prob.py:64-65)")
        prev = prob / scale
    return prev


def sum_forecast_by_state(vol_state_array: np.ndarray, filtered: np.ndarray, tol: float = 1e-6):
    """msm_estimation.py:205-248.  vol_state_array (dim, S); filtered (dim, T, S).
    Returns forecasts_by_states (T, dim, q) and unique_vol_states (dim, q)."""
    dim = vol_state_array.shape[0]
    summed, uniq = [], []
    for i in range(dim):
        rounded = np.round(vol_state_array[i, :] / tol) * tol                # :228
        u, inv = np.unique(rounded, return_inverse=True)                      # :229
        s = np.stack([filtered[i][:, inv == j].sum(axis=1) for j in range(len(u))], axis=1)
        summed.append(s)
        uniq.append(u)
    return np.array(summed).transpose(1, 0, 2), np.array(uniq)


def forecast_combinations(fbs: np.ndarray):
    """compute_forecast_combinations (msm_estimation.py:392-418): xy-meshgrid
    product order (2-D: l = a*q + b -> f0[a] f1[b]; 3-D permuted, Q7)."""
    T, dim, q = fbs.shape
    out = np.zeros((T, q ** dim))
    for n in range(T):
        rows = [fbs[n, d, :] for d in range(dim)]
        comb = np.array(np.meshgrid(*rows)).T.reshape(-1, dim)
        out[n] = np.prod(comb, axis=1)
    return out


def vol_combinations(dim: int, q: int):
    """create_vol_combinations (msm_estimation.py:369-389): ij order."""
    g = np.meshgrid(*[np.arange(q) for _ in range(dim)], indexing="ij")
    return np.stack(g, axis=-1).reshape(-1, dim)


# --------------------------------------------------------------------------- grids
def x_grid(num_points: int, model: str, x_min=-5, x_max=5):
    """x_values / step of compute_normal_densities: MSM splits n//4, n//7
    (msm_estimation.py:300-319); GARCH/UKF n//8, n//5 (garch_estimation.py:166-183)."""
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
    step[0] = step[1]                                                # Q18
    return x, step


def msm_densities(unique_vol_states: np.ndarray, x: np.ndarray):
    """densities[i, j, :] (msm_estimation.py:322-328)."""
    dim, q = unique_vol_states.shape
    d = np.zeros((dim, q, x.size))
    for i in range(dim):
        for j in range(q):
            s = unique_vol_states[i, j]
            d[i, j, :] = (1 / (np.sqrt(2 * np.pi) * s)) * np.exp(-0.5 * (x / s) ** 2)
    return d


def msm_integration_params(windows: np.ndarray, params: list, k: int, num_points: int):
    """MSMEstimation.integration_params_retrieval (msm_estimation.py:123-137) with
    the true k (the reference's int(sqrt(2**k)) is wrong for k not in {1,2,4,5}, Q8).

    windows (T, N, dim); params per asset {'m_0','sig','b','gamma'}."""
    dim = windows.shape[2]
    filt = np.array([msm_filtered_probs(windows[:, :, d], k, p["m_0"], p["sig"], p["b"], p["gamma"])
                     for d, p in enumerate(params)])                          # (dim, T, S)
    vsa = np.array([msm_vol_states(k, p["m_0"], p["sig"]) for p in params])
    fbs, uvs = sum_forecast_by_state(vsa, filt)
    x, step = x_grid(num_points, "msm")
    dens = msm_densities(uvs, x)
    combos = vol_combinations(dim, uvs.shape[1])
    pi = forecast_combinations(fbs)
    return dict(filtered=filt, vol_states_array=vsa, forecasts_by_states=fbs, forecasts=pi,
                unique_vol_states=uvs, densities=dens, x_values=x, step=step, combos=combos)


# --------------------------------------------------------------------------- GARCH
def garch_sigma2(window: np.ndarray, omega, alpha, beta):
    """calculate_conditional_variances (garch/estimation.py:40-65), GARCH(1,1),
    batched over the leading axis of window (.., N)."""
    w = np.asarray(window)
    s2 = np.zeros(w.shape)
    s2[..., 0] = omega / (1 - alpha - beta)
    for t in range(1, w.shape[-1]):
        v = omega + alpha * (w[..., t - 1] ** 2)
        v = v + beta * s2[..., t - 1]
        s2[..., t] = np.maximum(v, 1e-7)
    return s2


def garch_forecast(windows: np.ndarray, omega, alpha, beta):
    """garch/forecast.py:5-19 for (p,q)=(1,1): sqrt(w + a r[-1]^2 + b s2[-1])."""
    s2 = garch_sigma2(windows, omega, alpha, beta)
    f = omega + alpha * windows[..., -1] ** 2 + beta * s2[..., -1]
    return np.sqrt(f)


def garch_loglik(returns: np.ndarray, omega, alpha, beta):
    """numba_garch_log_likelihood (garch/estimation.py:91-125), p=q=1."""
    s2 = garch_sigma2(returns, omega, alpha, beta)
    r, s = returns[1:], s2[..., 1:]
    return -0.5 * np.sum(np.log(2 * np.pi * s) + (r ** 2) / s, axis=-1)


# --------------------------------------------------------------------------- UKF
def ukf_run(windows: np.ndarray, a, l, q, alpha=1.6, beta=2.0, kappa=1.75):
    """calculate_loglikelihood (kalman_mean_reverting/estimate.py:230-281), batched
    over windows (B, N) with init (l, q) as forecast.py:9 passes.  Returns
    (forecast = exp(last prediction mean) (Q19), LL, state (B,N), failed (B,))."""
    w = np.atleast_2d(np.asarray(windows, dtype=np.float64))
    B, N = w.shape
    L = 2
    lam = (alpha ** 2) * (L + kappa) - L
    wm = np.full(2 * L + 1, 1 / (2 * (L + lam)))
    wc = np.full(2 * L + 1, 1 / (2 * (L + lam)))
    wm[0] = lam / (L + lam)
    wc[0] = wm[0] + (1 - alpha ** 2 + beta)
    wm2 = np.full(L + 1, 1 / (2 * (L + lam)))
    wm2[0] = lam / (L + lam)
    phi = np.sqrt(L + lam)
    x = np.full(B, float(l))
    var = np.full(B, float(q))
    LL = np.zeros(B)
    failed = np.zeros(B, dtype=bool)
    state = np.zeros((B, N))
    xmean = np.zeros(B)
    for t in range(N):
        d = np.where(var <= 0, var + 1e-8, var)
        c0 = np.sqrt(d)                                     # custom_cholesky :54-78
        X10 = np.stack([x, x + phi * c0, x + phi * 0.0, x - phi * c0, x - phi * 0.0], axis=1)
        X11 = np.array([0.0, 0.0 + phi * 0.0, 0.0 + phi * 1.0, 0.0 - phi * 0.0, 0.0 - phi * 1.0])
        X = a * (X10 - l) + l + q * X11[None, :]            # f_vectorized :141
        xmean = X @ wm
        diff = X - xmean[:, None]
        P = (diff * wc[None, :] * diff).sum(axis=1)
        sP = np.sqrt(P)
        X2 = np.stack([xmean, xmean + phi * sP, xmean - phi * sP], axis=1)
        eta = w[:, t][:, None] / np.exp(X2)
        h = ((1 / np.sqrt(2 * np.pi)) * np.exp(-0.5 * eta ** 2)) * np.abs(eta)
        Z = (wm2[None, :] * h).sum(axis=1)
        bad = (Z <= 0) | (Z < 1e-10)
        failed |= bad
        Zs = np.where(bad, 1.0, Z)
        mean = ((wm2[None, :] * X2 * h) / Zs[:, None]).sum(axis=1)
        var = (wm2[None, :] * ((h / Zs[:, None]) * (X2 - mean[:, None]) ** 2)).sum(axis=1)
        state[:, t] = mean
        LL += np.log(np.abs(Zs))
        x = mean
    return np.exp(xmean), LL, state, failed


def sigma_forecasts(windows: np.ndarray, model: str, params: list):
    """(T, dim) sigma forecasts for GARCH (garch_estimation.py:190-231) or
    UKF (mean_reverting_estimation.py:192-232)."""
    out = np.zeros((windows.shape[0], windows.shape[2]))
    for d, p in enumerate(params):
        wd = windows[:, :, d]
        if model == "garch":
            out[:, d] = garch_forecast(wd, p["omega"], p["alpha"], p["beta"])
        else:
            f, _, _, failed = ukf_run(wd, p["a"], p["l"], p["q"])
            if failed.any():
                raise FloatingPointError("UKF normaliser Z < 1e-10 (estimate.py:219-220, Q19)")
            out[:, d] = f
    return out


def msm_loglik(returns: np.ndarray, k, m0, sig, b, gamma):
    """ProbEstimation.calc_likelihood (calc_prob.py:134-142 -> :36-47)."""
    A = msm_transition(k, m0, b, gamma)
    vs = msm_vol_states(k, m0, sig)
    S = vs.size
    r = np.asarray(returns, dtype=np.float64)
    cond = (1 / (vs[None, :] * np.sqrt(2 * np.pi))) * np.exp(-0.5 * (r[:, None] / vs[None, :]) ** 2)
    prev = np.full(S, 1 / S)
    probs = np.zeros((r.size, S))
    for i in range(r.size):
        pr = (A @ prev) * cond[i]
        sc = pr.sum()
        if sc == 0:
            raise FloatingPointError("normaliser 0")
        prev = pr / sc
        probs[i] = prev
    L = 0.0
    for i in range(1, r.size):
        term = np.dot(A @ probs[i - 1], cond[i])
        if term <= 0:
            return -math.inf
        L += math.log(term)
    return L
