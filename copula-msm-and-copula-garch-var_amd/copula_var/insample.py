"""In-sample marginals and densities that feed the copula fit
(calculate_marginals_and_densities_in_sample of the three model adapters).

One pass over the N in-sample returns per asset, once per fit: the MSM marginals come
from the device filter (cvq_msm_marginals; msm_marginals_densities is its host
restatement, kept for the CPU tests), the UKF state path from the device filter
(cvq_ukf_filter, the kernel the EM fit uses); the GARCH variance recursion is an O(N)
host loop.
"""
from __future__ import annotations

import itertools

import numpy as np
from scipy.special import erf
from scipy.stats import norm

from . import engine


def norm_cdf_array(x):
    """utils/utils.py:4-22 (erf form)."""
    return 0.5 * (1 + erf(np.asarray(x) / np.sqrt(2)))


def norm_pdf_array(x):
    """utils/utils.py:24-42."""
    return (1 / (1 * np.sqrt(2 * np.pi))) * np.exp(-0.5 * np.asarray(x) ** 2)


def msm_transition(k, m0, b, gamma):
    """calc_prob.py:86-101: the 2^k x 2^k transition matrix and the state multipliers."""
    M = np.array(list(itertools.product([m0, 2 - m0], repeat=k)))
    gamma_k = 1 - (1 - gamma) ** (b ** np.arange(M.shape[1]))
    p_values = 1 - gamma_k / 2
    q_values = 1 - p_values
    A = np.prod(np.where(M[:, None, :] == M[None, :, :], p_values, q_values), axis=2)
    return A, M


def msm_state_probs(returns, k, m0, sig, b, gamma):
    """calc_prob.py:7-32, 110-120: filtered state probabilities (N, 2^k), the
    conditional normal pdfs (N, 2^k) and the vol states (2^k,)."""
    r = np.asarray(returns, dtype=np.float64)
    A, M = msm_transition(k, m0, b, gamma)
    S = A.shape[0]
    vol = np.array([np.sqrt(np.prod(M[i])) * sig for i in range(S)])          # :103-108
    cond = (1 / (vol[None, :] * np.sqrt(2 * np.pi))) * np.exp(-0.5 * (r[:, None] / vol[None, :]) ** 2)
    probs = np.zeros((r.size, S))
    prev = np.full(S, 1 / S)
    for i in range(r.size):
        trans = A @ prev                                                        # :56-57
        p = trans * cond[i]
        scale = np.sum(p)
        if scale == 0:
            raise FloatingPointError(f"MSM filter: zero likelihood at step {i} (calc_prob.py:64-65)")
        prev = p / scale
        probs[i] = prev
    return probs, cond, vol


def msm_marginals_densities(returns, k, m0, sig, b, gamma):
    """calc_marginals.py:7-30: marginals, densities (N-1,) and vol states."""
    r = np.asarray(returns, dtype=np.float64)
    probs, cond, vol = msm_state_probs(r, k, m0, sig, b, gamma)
    cond_marg = norm.cdf(r[:, None] / vol[None, :])                            # calc_prob.py:122-132
    marginals = np.sum(probs[1:, :] * cond_marg[:-1, :], axis=1)
    densities = np.sum(probs[1:, :] * cond[:-1, :], axis=1)
    return marginals, densities, vol


def msm_marginals_densities_device(returns, k, m0, sig, b, gamma, device: int = 0):
    """msm_marginals_densities on the device (cvq_msm_marginals: one Hamilton-filter pass,
    the state sums per step in the same kernel); the vol states from the host transition
    (calc_prob.py:103-108, exact)."""
    m, d = engine.msm_marginals(returns, k, m0, sig, b, gamma, device)
    _, M = msm_transition(k, m0, b, gamma)
    vol = np.array([np.sqrt(np.prod(M[i])) * sig for i in range(M.shape[0])])
    return m, d, vol


def garch_eps(returns, omega, alpha, beta, epsilon=1e-7):
    """garch/estimation.py:22-38 (parameter checks), 40-65, 76-89: eps_t = r_t / sigma_t."""
    r = np.asarray(returns, dtype=np.float64)
    alpha, beta = np.atleast_1d(np.asarray(alpha, dtype=np.float64)), np.atleast_1d(np.asarray(beta, dtype=np.float64))
    if not all(a > 0 for a in alpha):
        raise ValueError("All elements of alpha_vect must be positive.")
    if not all(b_ > 0 for b_ in beta):
        raise ValueError("All elements of beta_vect must be positive.")
    if omega <= 0:
        raise ValueError("Omega must be positive.")
    if sum(alpha) + sum(beta) >= 1:
        raise ValueError("The sum of alpha_vect and beta_vect must be less than 1.")
    p, q = alpha.size, beta.size
    s2 = np.zeros(r.size)
    s2[0] = omega / (1 - sum(alpha) - sum(beta))
    for t in range(1, r.size):
        v = omega
        for i in range(min(p, t)):
            v += alpha[i] * (r[t - i - 1] ** 2)
        for j in range(min(q, t)):
            v += beta[j] * s2[t - j - 1]
        s2[t] = max(v, epsilon)
    return r / np.sqrt(s2)


def garch_marginals_densities(returns, best_pq, best_params):
    """garch_estimation.py:92-104."""
    bp = np.asarray(best_params, dtype=np.float64)
    p = int(best_pq[0])
    eps = garch_eps(returns, bp[0], bp[1:p + 1], bp[p + 1:])
    return norm_cdf_array(eps), norm_pdf_array(eps)


def mr_marginals_densities(returns, a, l, q, device: int = 0):
    """mean_reverting_estimation.py:97-104: eps = r / exp(state path) of the UKF with
    init (l, q) (estimate.py:46-51), on the device."""
    r = np.asarray(returns, dtype=np.float64)
    ll, states = engine.ukf_filter(r, np.array([[a, l, q]]), device)
    if ll[0] == -1e10:
        raise FloatingPointError("UKF failed on the in-sample series (estimate.py:270-271: state_estimation None)")
    eps = r / np.exp(states[0])
    return norm_cdf_array(eps), norm_pdf_array(eps)
