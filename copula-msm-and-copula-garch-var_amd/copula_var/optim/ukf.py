"""Mean-reverting log-vol EM fit (kalman_mean_reverting/optimize.py:6-167) with the
UKF E-step on the device.

Each E-step is one KalmanFilterVolEstimation pass (estimate.py:7-51, 230-281): a
sequential recursion over the N in-sample returns that yields the log-likelihood
and the filtered state path.  On the device that is ``cvq_ukf_filter`` (one lane
per chain).  A single chain is a chain of dependent passes, so the batching axis is
the assets: ``em_lockstep`` runs one EM chain per asset and hands every chain's
pending E-step to ONE launch (returns one series per lane).  Each chain's control
flow is the reference's, written as a generator that yields the parameters it
needs filtered.

Kept exactly (they change the result):
* the M-step uses the INITIAL a (optimize.py:83 binds a, l, q once; :141-149);
* update_l ignores mu (:46-48);
* random_perturbation writes the perturbed a into the array it is given, which is
  self.best_params on a restart or a stalled a (:61-62, :119, :153);
* the E-step at :135 repeats the one at :95 with the same parameters (and :120
  repeats the pass random_perturbation just made): the last pass is reused.
Randomness: the reference draws from numpy's global state (unseeded); each chain
here owns RandomState(seed) with the same draw sequence (one uniform per
perturbation attempt).  The reference's retry loop (:58-70) is unbounded; here it
raises after ``max_retries`` failed attempts.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np

from .. import engine


class _Pass:
    """What e_step returns (the KalmanFilterVolEstimation attributes used)."""
    __slots__ = ("LL", "state_estimation")

    def __init__(self, LL, state_estimation):
        self.LL = LL
        self.state_estimation = state_estimation


class VolOptimizer:
    """optimize.py:VolOptimizer; same constructor arguments plus seed / device /
    efilter (efilter(returns (B, N), params (B, 3)) -> (LL (B,), states (B, N)),
    default the device kernel; tests pass the CPU oracle)."""

    def __init__(self, a, l, q, max_iter=1000, tol=1e-7, perturb_scale=0.05, restart_attempts=5, seed: int = 0,
                 device: int = 0, efilter: Optional[Callable] = None, max_retries: int = 100000):
        self.a = a
        self.l = l
        self.q = q
        self.max_iter = max_iter
        self.tol = tol
        self.perturb_scale = perturb_scale
        self.restart_attempts = restart_attempts
        self.best_LL = -np.inf
        self.best_params = np.array([a, l, q])
        self.n_steps = None
        self.rng = np.random.RandomState(seed)
        self.device = device
        self.max_retries = max_retries
        self._efilter = efilter or (lambda R, P: engine.ukf_filter(R, P, self.device))
        self._last = None
        self.launches = 0
        self.passes = 0

    # ------------------------------------------------------------ M-step pieces
    def update_a_with_ols(self, state_estimates, a, l):
        """optimize.py:34-44."""
        y = state_estimates[1:] - a * l
        x = state_estimates[:-1] - a * l
        numerator = np.sum(x * y)
        denominator = np.sum(x ** 2)
        if denominator == 0:
            return 0.01
        return numerator / denominator

    def update_l(self, mu, q, a):
        """optimize.py:46-48 (mu unused, as in the reference)."""
        return q ** 2 / (2 * (1 - a ** 2))

    def update_q(self, a, state_estimation):
        """optimize.py:50-53."""
        return np.std(state_estimation) * np.sqrt(1 - a ** 2)

    # ------------------------------------------------- generator-form control flow
    def _e_step(self, params):
        """optimize.py:28-32: yields the parameters to filter, receives (LL, states)."""
        key = (float(params[0]), float(params[1]), float(params[2]))
        if self._last is not None and self._last[0] == key:
            return self._last[1]
        ll, states = yield np.array(key)
        failed = ll == -1e10                                   # estimate.py:270-271
        res = _Pass(ll, None if failed else np.array(states))
        self._last = (key, res)
        return res

    def _random_perturbation(self, params, mu):
        """optimize.py:55-76 (writes a into `params`)."""
        tries = 0
        while True:
            a = np.clip(params[0] + self.rng.uniform(-self.perturb_scale, self.perturb_scale), 0.5, 0.999999)
            params[0] = a
            ukf = yield from self._e_step(params)
            if ukf.state_estimation is not None:
                break
            tries += 1
            if tries >= self.max_retries:
                raise RuntimeError(f"UKF failed for {tries} perturbations of a in a row")
        q = self.update_q(a, ukf.state_estimation)
        l = self.update_l(mu, q, a)
        return np.array([a, l, q])

    def _em(self, returns):
        """optimize.py:78-167."""
        params = np.array([self.a, self.l, self.q], dtype=np.float64)
        self.n_steps = len(returns)
        a, l, q = self.a, self.l, self.q
        with np.errstate(divide="ignore"):
            mu = np.mean(np.log(abs(returns)))
        for _ in range(self.max_iter):
            ukf = yield from self._e_step(params)
            if ukf.LL == -1e10:
                params = yield from self._random_perturbation(params, mu)
                continue
            LL_diff = np.abs(ukf.LL - self.best_LL)
            if LL_diff < self.tol:
                self.best_LL = ukf.LL
                self.best_params = params.copy()
                for _restart in range(self.restart_attempts):
                    params = yield from self._random_perturbation(self.best_params, mu)
                    ukf = yield from self._e_step(params)
                    if ukf.LL > self.best_LL:
                        self.best_LL = ukf.LL
                        self.best_params = params.copy()
                continue
            if ukf.LL > self.best_LL:
                self.best_LL = ukf.LL
                self.best_params = params.copy()
            ukf = yield from self._e_step(params)
            if ukf.state_estimation is None:
                params = yield from self._random_perturbation(params, mu)
                continue
            q_new = self.update_q(a, ukf.state_estimation)
            l_new = self.update_l(mu, q_new, a)
            a_new = np.clip(self.update_a_with_ols(ukf.state_estimation, a, l_new), 0.5, 0.99)
            if params[0] == a_new:
                params = yield from self._random_perturbation(self.best_params, mu)
            else:
                params[0] = a_new
                params[1] = l_new
                params[2] = q_new
        return self.best_params, self.best_LL

    def em_algorithm(self, returns):
        """optimize.py:78-167 for one series -> (best_params, best_LL)."""
        return em_lockstep([self], [returns])[0]


def em_lockstep(optimizers: Sequence[VolOptimizer], series: Sequence[np.ndarray],
                efilter: Optional[Callable] = None) -> List[tuple]:
    """Run one EM chain per (optimizer, series) in lockstep: every round, the pending
    E-step of each live chain goes into ONE filter launch (one series per lane).
    All series must have the same length."""
    series = [np.ascontiguousarray(s, dtype=np.float64) for s in series]
    if len({s.size for s in series}) > 1:
        raise ValueError("em_lockstep needs equal-length series")
    efilter = efilter or optimizers[0]._efilter
    gens = [o._em(s) for o, s in zip(optimizers, series)]
    out: List[Optional[tuple]] = [None] * len(gens)
    pending = {}
    for i, g in enumerate(gens):
        try:
            pending[i] = next(g)
        except StopIteration as e:
            out[i] = e.value
    while pending:
        idx = sorted(pending)
        ll, states = efilter(np.stack([series[i] for i in idx]), np.stack([pending[i] for i in idx]))
        for o in {id(optimizers[i]): optimizers[i] for i in idx}.values():
            o.launches += 1
        for j, i in enumerate(idx):
            optimizers[i].passes += 1
            try:
                pending[i] = gens[i].send((float(ll[j]), states[j]))
            except StopIteration as e:
                out[i] = e.value
                del pending[i]
    return out
