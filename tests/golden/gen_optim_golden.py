#!/usr/bin/env python3
"""Golden vectors for the in-sample optimiser layer.

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER.  Like gen_golden.py it imports the
read-only reference as a Python package with the identity ``numba`` shim on the
path (tests/golden/_shims), and writes inputs + the reference's outputs:

* optim_garch.npz -- GarchOptimizer(returns, p_max, q_max).optimize() on a
  synthetic GARCH(1,1) series (garch/opti.py:89-137): the selected (p, q), its
  parameters, -log-likelihood and BIC, the Newton-Raphson result of every (p, q)
  (garch/opti.py:139-172), and numba_garch_log_likelihood (garch/estimation.py:91-125)
  at a set of parameter rows per (p, q).
* optim_msm_ll.npz -- ProbEstimation(k, m0, sigma, b, gamma, returns).calc_likelihood()
  (markov_switching_multifractal/calc_prob.py) at a set of parameter rows.
* optim_msm_marg.npz -- calc_marginals / calc_densities
  (markov_switching_multifractal/calc_marginals.py:7-30, the in-sample MSM marginals
  and densities of msm_estimation.py:55-120) on the same returns and parameter rows.
* optim_ukf.npz -- KalmanFilterVolEstimation(a, l, q, l, q, n, returns)
  (kalman_mean_reverting/estimate.py:7-43 -> calculate_loglikelihood :230-281, called
  so by forecast.py:9 and optimize.py:31): LL, filtered state path and the forecast
  mean at a set of (a, l, q) rows on a synthetic OU-log-vol series.
* optim_garch_pq.npz -- garch/forecast.py:5-19 calc_forecast(omega, alpha, beta,
  window) for (p, q) in {(2,1), (1,2), (2,2), (3,2)} over rolling windows (the alpha /
  beta lag order of Q13: alpha_1 pairs with the oldest of the last p returns).

Usage:  python tests/golden/gen_optim_golden.py [all|msm_marginals|ukf_garch_pq]
"""
from __future__ import annotations

import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
SHIMS = os.path.join(HERE, "_shims")
PKG = os.path.join(REPO, "copula-msm-and-copula-garch-var_amd")
if not os.path.isdir(REF):
    sys.exit("gen_optim_golden.py: /root/reference is absent -- the committed .npz files are the vectors.")
sys.path[:0] = [SHIMS, REF, PKG]

from copula_var import synthetic  # noqa: E402  (our own generator, not reference code)

P_MAX = Q_MAX = 2


def garch_series(n=1135, seed=20241125):
    cfg = synthetic.baseline_configs()[1].with_(T=1, n_in=n - 1, seed=seed)
    r = synthetic.simulate_returns(cfg)[:, 0]
    return r - r.mean()


def main():
    import matplotlib
    matplotlib.use("Agg")
    from garch.opti import GarchOptimizer
    from garch.estimation import numba_garch_log_likelihood
    from markov_switching_multifractal.calc_prob import ProbEstimation

    r = garch_series()
    rng = np.random.default_rng(7)
    ll_rows, ll_vals, ll_pq = [], [], []
    for p in range(1, P_MAX + 1):
        for q in range(1, Q_MAX + 1):
            for _ in range(4):
                ab = rng.uniform(0.02, 0.9 / (p + q), size=p + q)
                row = np.concatenate(([rng.uniform(0.01, 0.2)], ab))
                ll_rows.append(np.pad(row, (0, 1 + P_MAX + Q_MAX - row.size)))
                ll_vals.append(numba_garch_log_likelihood(r, row[0], row[1:p + 1], row[p + 1:], 1e-7))
                ll_pq.append((p, q))
    opt = GarchOptimizer(r, p_max=P_MAX, q_max=Q_MAX)
    per_pq = {}
    orig = opt.newton_raphson

    def spy(initial, p, q):
        out = orig(initial, p, q)
        per_pq[(p, q)] = out
        return out
    opt.newton_raphson = spy
    with contextlib.redirect_stdout(io.StringIO()):
        best_pq, best_params, best_result, best_bic = opt.optimize()
    pq_keys = sorted(per_pq)
    nr_params = np.array([np.pad(np.asarray(per_pq[k][0], float), (0, 1 + P_MAX + Q_MAX - (1 + sum(k))))
                          for k in pq_keys])
    nr_nll = np.array([per_pq[k][1] for k in pq_keys])
    np.savez(os.path.join(HERE, "optim_garch.npz"), returns=r, p_max=P_MAX, q_max=Q_MAX,
             ll_rows=np.array(ll_rows), ll_pq=np.array(ll_pq), ll=np.array(ll_vals),
             best_pq=np.array(best_pq), best_params=np.asarray(best_params, float), best_nll=best_result,
             best_bic=best_bic, nr_pq=np.array(pq_keys), nr_params=nr_params, nr_nll=nr_nll)
    print("garch:", best_pq, best_params, best_result, best_bic)

    # MSM log-likelihood KATs (calc_prob.py: calc_likelihood)
    cfg = synthetic.baseline_configs()[2].with_(T=1, n_in=400)
    x = synthetic.simulate_returns(cfg)[:, 0]
    x = x - x.mean()
    rows, vals = [], []
    for m0, sig, b, g in [(0.45, 1.2, 3.0, 0.3), (0.6, 0.9, 10.0, 0.5), (0.3, 1.5, 1.5, 0.1), (0.5, 1.0, 40.0, 0.9)]:
        rows.append((m0, sig, b, g))
        vals.append(ProbEstimation(4, m0, sig, b, g, x).calc_likelihood())
    np.savez(os.path.join(HERE, "optim_msm_ll.npz"), returns=x, k=4, rows=np.array(rows), ll=np.array(vals))
    print("msm ll:", vals)


def msm_marginals():
    import matplotlib
    matplotlib.use("Agg")
    from markov_switching_multifractal.calc_marginals import calc_densities, calc_marginals
    z = np.load(os.path.join(HERE, "optim_msm_ll.npz"))
    x, k = z["returns"], int(z["k"])
    marg, eps, dens, vol = [], [], [], []
    for m0, sig, b, g in z["rows"]:
        m, e, v = calc_marginals(k, m0, sig, b, g, x)
        marg.append(m)
        eps.append(e)
        vol.append(v)
        dens.append(calc_densities(k, m0, sig, b, g, x))
    np.savez(os.path.join(HERE, "optim_msm_marg.npz"), returns=x, k=k, rows=z["rows"], marginals=np.array(marg),
             eps=np.array(eps), densities=np.array(dens), vol_states=np.array(vol))
    print("msm marginals:", np.array(marg).shape, np.array(dens).shape)


def ukf_garch_pq():
    import matplotlib
    matplotlib.use("Agg")
    from kalman_mean_reverting.estimate import KalmanFilterVolEstimation
    from garch.forecast import calc_forecast

    cfg = synthetic.baseline_configs()[5].with_(T=1, n_in=1134)
    r = synthetic.simulate_returns(cfg)[:, 0]
    r = r - r.mean()
    rows = [(0.97, 0.05, 0.15), (0.90, 0.0, 0.30), (0.99, -0.2, 0.10), (0.80, 0.30, 0.20), (0.5, 0.1, 0.5)]
    ll, states, fc = [], [], []
    for a, l, q in rows:
        k = KalmanFilterVolEstimation(a, l, q, l, q, r.size, r)
        ll.append(k.LL)
        states.append(np.asarray(k.state_estimation, dtype=np.float64))
        fc.append(k.forecasts)
    np.savez(os.path.join(HERE, "optim_ukf.npz"), returns=r, rows=np.array(rows), ll=np.array(ll, dtype=np.float64),
             states=np.array(states), forecast_mean=np.array(fc, dtype=np.float64))
    print("ukf ll:", ll)

    n_in, T = 400, 24
    s = garch_series(n=n_in + T - 1, seed=11)
    orders = [(2, 1), (1, 2), (2, 2), (3, 2)]
    prm = {(2, 1): [0.05, 0.05, 0.03, 0.85], (1, 2): [0.04, 0.07, 0.5, 0.38],
           (2, 2): [0.06, 0.04, 0.05, 0.45, 0.4], (3, 2): [0.05, 0.02, 0.03, 0.04, 0.5, 0.35]}
    out = np.zeros((len(orders), T))
    for i, (p, q) in enumerate(orders):
        w = np.asarray(prm[(p, q)], dtype=np.float64)
        for t in range(T):
            out[i, t] = calc_forecast(w[0], w[1:p + 1], w[p + 1:], s[t:t + n_in])
    np.savez(os.path.join(HERE, "optim_garch_pq.npz"), returns=s, n_in=n_in, orders=np.array(orders),
             params=np.array([np.pad(prm[o], (0, 6 - len(prm[o]))) for o in orders]), forecasts=out)
    print("garch pq forecasts:", out[:, :3])


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("all", "optim"):
        main()
    if what in ("all", "msm_marginals"):
        msm_marginals()
    if what in ("all", "ukf_garch_pq"):
        ukf_garch_pq()
