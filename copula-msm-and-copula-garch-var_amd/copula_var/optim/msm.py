"""MSM in-sample fit (markov_switching_multifractal/opti.py:8-139) with the
likelihoods on the device.

The reference runs one basin-hopping chain per fixed starting b
(b_values = linspace(1, 50, 10), opti.py:21) in a process pool (opti.py:121-129);
each chain makes basin_iter proposals, each one Hamilton-filter likelihood over
the in-sample returns (calc_prob.py:134-142, numba-jitted).  Here the chains run in
lockstep: the 10 proposals of one iteration go to the device as ONE batched
likelihood launch (cvq_msm_loglik: one lane-quad per parameter row, the transition
applied as k 2x2 butterflies), then each chain takes its accept / step-size /
reinitialise decision exactly as opti.py:82-98 does.

Randomness: the reference draws from numpy's global RandomState inside forked
workers (unseeded, scheduling-dependent).  Each chain here owns a
numpy RandomState(seed + chain) with the reference's draw sequence
(randn per parameter, opti.py:67; uniform on reinitialisation, :33), so a run
is reproducible and can be replayed on the CPU likelihood for parity.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from .. import engine


class Optimizer:
    """opti.py:Optimizer: same constructor arguments, likelihood, perturbation,
    basin hopping and b-sweep; the b chains evaluate their proposals in one launch.

    loglik(rows) -> log-likelihoods of rows (B, 4) = (m0, sigma, b, gamma); default
    the device kernel.  Tests pass the CPU oracle to replay the same chains.
    """

    def __init__(self, returns, k, max_iter=100, tol=1e-6, basin_iter=100, step_size=0.2, temperature=1.0,
                 gamma_weight=0, b_weight=0, seed: int = 0, device: int = 0, loglik: Optional[Callable] = None):
        self.returns = np.ascontiguousarray(returns, dtype=np.float64)
        self.k = k
        self.max_iter = max_iter
        self.tol = tol
        self.basin_iter = basin_iter
        self.step_size = step_size
        self.temperature = temperature
        self.sample_variance = np.var(self.returns)                     # opti.py:18
        self.gamma_weight = gamma_weight
        self.b_weight = b_weight
        self.b_values = np.linspace(1.0, 50.0, 10)                      # opti.py:21
        self.seed = seed
        self.device = device
        self._loglik = loglik or (lambda rows: engine.msm_loglik(self.returns, self.k, rows, self.device))
        self.launches = 0
        self.evaluations = 0

    def estimate_sigma(self, m_0=0.5):
        """opti.py:25-27."""
        factor = (m_0 ** 2 - 2 * m_0 + 2) ** (self.k / 2)
        return np.sqrt(self.sample_variance) / factor

    @staticmethod
    def reinitialize_near_bounds(params, bounds, rng):
        """opti.py:29-35."""
        for i, (param, (lower_bound, upper_bound)) in enumerate(zip(params, bounds)):
            if param <= lower_bound + 0.01 * (upper_bound - lower_bound) or param >= upper_bound - 0.01 * (
                    upper_bound - lower_bound):
                params[i] = rng.uniform(lower_bound + 0.1 * (upper_bound - lower_bound),
                                        upper_bound - 0.1 * (upper_bound - lower_bound))
        return params

    def _objective(self, params_list, caches):
        """likelihood (opti.py:37-56) of one parameter vector per chain, with the
        per-chain rounded-parameter caches; the misses go to the device in one launch."""
        keys = [tuple(np.round(p, decimals=6)) for p in params_list]
        out = [caches[c].get(keys[c]) for c in range(len(params_list))]
        miss = [c for c in range(len(params_list)) if out[c] is None]
        if miss:
            rows = np.array([[params_list[c][0], self.estimate_sigma(params_list[c][0]), params_list[c][1],
                              params_list[c][2]] for c in miss])
            ll = np.asarray(self._loglik(rows), dtype=np.float64)
            self.launches += 1
            self.evaluations += len(miss)
            for c, v in zip(miss, ll):
                m_0, b, gamma = params_list[c]
                val = -v
                val += self.gamma_weight * (len(self.returns) * (gamma - 0.5) ** 2) + \
                    self.b_weight * (len(self.returns) * (1.0 / b) ** 2)
                caches[c][keys[c]] = val
                out[c] = val
        return out

    @staticmethod
    def perturb_parameters(params, bounds, step_size, rng):
        """opti.py:58-73."""
        perturbed_params = np.copy(params)
        for i in range(len(params)):
            lower_bound, upper_bound = bounds[i]
            range_size = upper_bound - lower_bound
            perturbation = rng.randn() * step_size * range_size
            perturbed_params[i] += perturbation
            perturbed_params[i] = np.clip(perturbed_params[i], lower_bound, upper_bound)
        return perturbed_params

    def basin_hopping_batch(self, initial_params_list, bounds):
        """opti.py:75-105 for every chain in lockstep (one launch per iteration)."""
        C = len(initial_params_list)
        rngs = [np.random.RandomState(self.seed + c) for c in range(C)]
        caches = [{} for _ in range(C)]
        cur = [np.copy(p) for p in initial_params_list]
        cur_ll = self._objective(cur, caches)
        step = [self.step_size] * C
        patience = 10
        improvement_count = [0] * C
        for _ in range(self.basin_iter):
            new = [self.perturb_parameters(cur[c], bounds, step[c], rngs[c]) for c in range(C)]
            new_ll = self._objective(new, caches)
            for c in range(C):
                if new_ll[c] < cur_ll[c]:
                    cur[c], cur_ll[c] = new[c], new_ll[c]
                    step[c] *= 0.9
                    improvement_count[c] = 0
                else:
                    improvement_count[c] += 1
                    if improvement_count[c] >= patience:
                        step[c] *= 1.1
                        improvement_count[c] = 0
                        cur[c] = self.reinitialize_near_bounds(cur[c], bounds, rngs[c])
        sig = [self.estimate_sigma(p[0]) for p in cur]
        final = np.asarray(self._loglik(np.array([[p[0], s, p[1], p[2]] for p, s in zip(cur, sig)])))
        self.launches += 1
        return [(p[0], p[1], p[2], s, float(v)) for p, s, v in zip(cur, sig, final)]

    def optimize(self, initial_params=np.array([0.5, 10, 0.5])):
        """opti.py:112-139: one chain per b value.  Quirk kept: the chains report
        calc_likelihood() (a log-likelihood, opti.py:103) and the sweep keeps the
        SMALLEST one (opti.py:127), i.e. the worst-fitting chain."""
        bounds = [(0.2, 0.8), (1.0, 50.0), (0.05, 0.95)]
        starts = []
        for b in self.b_values:                                          # evaluate_b (opti.py:107-110)
            p = np.array(initial_params, dtype=np.float64)
            p[1] = b
            starts.append(p)
        best_likelihood, best_params = np.inf, None
        for m_0, b, gamma, sigma, global_likelihood in self.basin_hopping_batch(starts, bounds):
            if global_likelihood < best_likelihood:                      # opti.py:127-129
                best_likelihood = global_likelihood
                best_params = [m_0, b, gamma, sigma]
        return best_params
