#!/usr/bin/env python3
"""Full-batch golden vectors: the pinned oracle's calc_var over a BASELINE workload's
WHOLE date batch.

The bisection couples every date of a batch (calc_var_class.py:275-293): the iteration
count is the maximum over all dates (Q2) and one all-zero iteration stops every date
(Q4).  The small goldens pin that coupling on 3-64 dates; these fixtures pin it at the
BASELINE batch sizes:

* fullbatch_cfg2.npz -- cfg 2 (MSM k = 4, Student, n = 256), T = 1000;
* fullbatch_cfg5.npz -- cfg 5 (UKF, Student, n = 256), T = 5000;
* fullbatch_cfg3.npz -- cfg 3 (GARCH(1, 1), Plackett, n = 512), T = 5000;
* fullbatch_cfg4.npz -- cfg 4 (3 assets, MSM k = 6, Gaussian, n = 128^3), the first 250 of its
  2000 dates (the oracle holds 16.8 MB of whole-box masses per date at 128^3, ~15 min here;
  250 dates = one eighth of the batch, the strong-scaling block of 8 GPUs).

Every fixture also holds the synthetic returns it was built from (`returns`, (n_in + T, dim))
and `n_in`, so the GPU box re-runs the device forecast stage from the same numbers
(tests/test_e2e_fullbatch_gpu.py) without depending on the RNG.

Inputs come from the oracle's own host forecast stage (oracle/forecast.py: rolling
windows, Hamilton filter / GARCH recursion / UKF, state collapse) on the synthetic
returns of copula_var.synthetic (numpy default_rng(20241125)); the expected output is
oracle.quadrature.calc_var (whole-box masses + boolean membership masks, no v*
tables) run over the full batch: the VaR vector, the global bisection count and the
Q4 break flag.  The oracle is pinned bit-exactly to reference-run goldens
(tests/test_oracle_golden.py).  Runs in the CPU container (minutes; cfg 3 holds
~10 GB of per-date masses); the GPU box only reads the .npz files.

Usage:  python tests/golden/gen_fullbatch.py [2] [5] [3] [4]
        python tests/golden/gen_fullbatch.py --add-returns [2] [5] [3]
          (adds `returns` / `n_in` to existing fixtures after checking that the oracle's
           forecast stage on them reproduces the stored tables bit for bit)
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "copula-msm-and-copula-garch-var_amd")]

from copula_var import synthetic                       # noqa: E402  (synthetic returns only)
from oracle import forecast as F                       # noqa: E402
from oracle.quadrature import Problem, calc_var        # noqa: E402


PREFIX_T = {4: 250}            # configs whose fixture holds the first dates of the batch only


def returns_for(cfg_no: int):
    """(config, returns) of the fixture: the BASELINE batch's synthetic returns, cut to the
    first PREFIX_T dates where the whole batch is too large for the oracle."""
    c = synthetic.baseline_configs()[cfg_no]
    rets = synthetic.simulate_returns(c)
    if cfg_no in PREFIX_T:
        c = c.with_(T=PREFIX_T[cfg_no])
        rets = rets[: c.n_in + c.T]
    return c, rets


def build(cfg_no: int):
    c, rets = returns_for(cfg_no)
    _, ptf_mean, windows = F.insample_split(rets, c.n_in, c.weights)
    out = dict(model=c.model, copula=c.copula, dim=c.dim, num_points=c.num_points, T=c.T,
               weights=c.weights, copula_params=np.asarray(c.copula_params(), dtype=np.float64),
               ptf_mean=ptf_mean, returns=rets, n_in=c.n_in)
    if c.model == "msm":
        m = F.msm_integration_params(windows, c.msm_params, c.k, c.num_points)
        out.update(forecasts_by_states=m["forecasts_by_states"], forecasts=m["forecasts"],
                   unique_vol_states=m["unique_vol_states"], densities=m["densities"], x_values=m["x_values"],
                   step=m["step"], combos=m["combos"])
        per = (m["forecasts_by_states"], m["forecasts"])
        uvs = m["unique_vol_states"]
    else:
        sig = F.sigma_forecasts(windows, c.model, c.model_params())
        x, step = F.x_grid(c.num_points, c.model)
        out.update(sigma_forecasts=sig, densities=np.ones((c.dim, 1, c.num_points)), x_values=x, step=step,
                   combos=np.zeros((1, c.dim)))
        per, uvs = sig, None
    P = Problem(c.model, c.copula, c.dim, out["x_values"], out["step"], out["densities"], out["combos"],
                c.weights, out["copula_params"], per, uvs)
    t0 = time.time()
    var, iters, broke = calc_var(P.compute_integral, P.T, ptf_mean)
    print(f"cfg {cfg_no}: T {c.T} iterations {iters} broke {broke} nan {int(np.isnan(var).sum())} "
          f"({time.time() - t0:.0f} s)", flush=True)
    out.update(var=var, iterations=iters, broke=broke)
    return out


def add_returns(cfg_no: int):
    path = os.path.join(HERE, f"fullbatch_cfg{cfg_no}.npz")
    z = dict(np.load(path, allow_pickle=False))
    c, rets = returns_for(cfg_no)
    assert int(z["T"]) == c.T
    _, ptf_mean, windows = F.insample_split(rets, c.n_in, c.weights)
    assert ptf_mean == float(z["ptf_mean"])
    if c.model == "msm":
        m = F.msm_integration_params(windows, c.msm_params, c.k, c.num_points)
        assert np.array_equal(m["forecasts_by_states"], z["forecasts_by_states"])
        assert np.array_equal(m["forecasts"], z["forecasts"])
    else:
        assert np.array_equal(F.sigma_forecasts(windows, c.model, c.model_params()), z["sigma_forecasts"])
    z.update(returns=rets, n_in=c.n_in)
    np.savez_compressed(path, **z)
    print(f"cfg {cfg_no}: returns {rets.shape} added", flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--add-returns":
        for cfg in [int(a) for a in args[1:]] or [2, 5, 3]:
            add_returns(cfg)
        return
    cfgs = [int(a) for a in args] or [2, 5, 3, 4]
    for cfg in cfgs:
        np.savez_compressed(os.path.join(HERE, f"fullbatch_cfg{cfg}.npz"), **build(cfg))


if __name__ == "__main__":
    main()
