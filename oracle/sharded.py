"""Oracle: the per-date / per-shard decomposition of calc_var -- TEST INFRASTRUCTURE ONLY.

The device solve (k_direct / k_solve_prefix + k_finalize) splits the
reference's batch-coupled bisection (utils/calc_var_class.py:95-177, 250-309)
into a per-date part that needs no communication and a tiny global part:

* every date runs a fixed budget of K bisection steps, recording the midpoint
  (lo+hi)/2 at the start of each step (snapshot k) and after the last (K);
* per shard, a header: the max over its dates of the step at which the date's
  own bracket first satisfied `hi - lo <= tol` (Q2's global while-condition is
  the max of these), an error flag if some date never did, and a bitmask of the
  steps at which some date had F != 0 (Q4's `np.all(F == 0)` break is the
  first step whose bit is clear in the OR over all shards);
* finalize: N = max over shards, kstop = min(N, first all-zero step), and
  VaR[t] = snapshot[t][kstop] + ptf_mean.

These functions restate that decomposition on the CPU over an
``oracle.quadrature.Problem`` so the sharding / collective logic
(copula_var/distributed.py) can be tested with gloo ranks without a GPU.
"""
from __future__ import annotations

import numpy as np


def local_solve(P, ptf_mean=0.0, K=24, obj_var=0.05, first_guess=-3.0, second_guess=(-3.5, -2.0),
                min_var=-7.5, max_var=0.0, lower=-100.0, tolerance=1e-6):
    """Per-date control flow of calc_var over P's dates (calc_var_class.py:114-160 + :250-309
    without the global coupling).  Returns (iters, error, nonzero_mask, snaps (T, K+1))."""
    T = P.T
    fg, sg0, sg1 = float(first_guess), float(second_guess[0]), float(second_guess[1])
    r0 = P.compute_integral(np.column_stack((np.full(T, float(lower)), np.full(T, fg))))
    nl = np.where(r0 >= obj_var, sg0, fg)
    nu = np.where(r0 < obj_var, sg1, fg)
    prev_upper = np.where(nl == sg0, sg0, fg)                                  # Q1
    nr = P.compute_integral(np.column_stack((nl, nu)))
    F = np.where(nl == fg, r0 + nr, r0 - nr)                                   # adjust_integral vs upper = fg
    lo, hi = np.full(T, np.nan), np.full(T, np.nan)                            # Q3
    m = F > obj_var
    lo[m], hi[m] = min_var, sg0
    m = (F < obj_var) & (nu == fg)
    lo[m], hi[m] = sg0, fg
    m = (F < obj_var) & (nu == sg1)
    lo[m], hi[m] = sg1, max_var
    m = (F > obj_var) & (nu == sg1)
    lo[m], hi[m] = fg, sg1
    ustack = ~((hi == sg0) | (hi == sg1))
    prev = F
    nt = np.full(T, -1)
    mask = 0
    snaps = np.empty((T, K + 1))
    for k in range(K):
        mid = (lo + hi) / 2
        snaps[:, k] = mid
        newly = (nt < 0) & ~(hi - lo > tolerance)
        nt[newly] = k
        b = np.where(ustack[:, None], np.column_stack((lo, mid)), np.column_stack((mid, hi)))
        val = P.compute_integral(b)
        Fn = np.where(b[:, 0] == prev_upper, prev + val, prev - val)
        if np.any(Fn != 0.0):
            mask |= 1 << k
        ustack = Fn < obj_var
        lo = np.where(ustack, mid, lo)
        hi = np.where(ustack, hi, mid)
        prev = Fn
        prev_upper = mid
    snaps[:, K] = (lo + hi) / 2
    newly = (nt < 0) & ~(hi - lo > tolerance)
    nt[newly] = K
    error = int(np.any(nt < 0))
    iters = int(nt.max()) if T else 0
    return iters, error, mask, snaps


def finalize(headers, snaps_all, T_total, K, ptf_mean=0.0):
    """k_finalize: headers = [(iters, error, nonzero)] per shard; snaps_all (>= T_total, K+1)."""
    N = max(h[0] for h in headers)
    err = any(h[1] for h in headers) or N > K
    nz = 0
    for h in headers:
        nz |= int(h[2])
    kstop = min(N, K)
    for k in range(kstop):
        if not (nz >> k) & 1:
            kstop = k
            break
    return np.asarray(snaps_all)[:T_total, kstop] + ptf_mean, kstop, bool(err)
