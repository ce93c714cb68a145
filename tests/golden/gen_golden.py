#!/usr/bin/env python3
"""Generate the golden vectors that pin the oracle and the HIP path.

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER.  It imports the read-only
reference (/root/reference, Nassim-cha/copula-MSM-and-copula-Garch-VaR
@ 2024-11-25) as a Python package, with two identity stand-ins on the path
(tests/golden/_shims: ``numba`` -> decorators are identity, ``yfinance`` ->
raises; neither is installed and there is no network).  It is
never imported by the test-suite, the bench or the product; it refuses to run
when /root/reference is absent.  No reference source is copied: the reference
is driven exactly as main.py drives it, through its own injection seams:

* returns   -> data_loader.load_data.SharedCacheIndexReturns.returns_cache
               (load_data.py:21-24 short-circuits the download)
* in-sample -> SharedCacheCopula{MSM,Garch,MR}VaR.cache
               (msm_estimation.py:35-38, garch_estimation.py:36-39,
               mean_reverting_estimation.py:36-39)
* copula    -> ValueAtRiskCalcualtion.calc_copula_params replaced by a fixed
               value (calc_var_class.py:77-82; the IFM optimiser is out of scope)
* MSM k=6   -> "patched-k oracle" (SURVEY.md Q8): msm_estimation.py:125 computes
               k = int(sqrt(2**k)), which is wrong for k=6 and makes the
               reference raise IndexError; the patch makes that one sqrt return
               log2 so the rest of the reference (incl. Q5/Q6/Q7) runs unchanged.

Each case writes tests/golden/<case>.npz holding inputs (returns, params),
the reference's forecast/quadrature tables, every compute_integral call
(bounds, result) in order, and the final VaR vector.  Special-function
known-answer vectors (scipy, the reference's own dependency) go to kat_special.npz.

Usage:  python tests/golden/gen_golden.py [case ...]
"""
from __future__ import annotations

import contextlib
import io
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
SHIMS = os.path.join(HERE, "_shims")
PKG = os.path.join(REPO, "copula-msm-and-copula-garch-var_amd")

if not os.path.isdir(REF):
    sys.exit("gen_golden.py: /root/reference is absent -- fixtures can only be generated "
             "in the build container; the committed .npz files are the vectors.")

os.environ["PYTHONPATH"] = os.pathsep.join([SHIMS, REF, os.environ.get("PYTHONPATH", "")])
sys.path[:0] = [SHIMS, REF, PKG]

from copula_var import synthetic  # noqa: E402  (our own generator, not reference code)


def _import_reference():
    from data_loader import load_data
    from utils import calc_var_ABC, calc_var_class, factory
    from utils.model_estimation.model import msm_estimation
    return load_data, calc_var_ABC, calc_var_class, factory, msm_estimation


class _Log:
    def __init__(self):
        self.calls = []


def _inject(cfg, returns_df, load_data, calc_var_ABC, start_date):
    tickers = list(returns_df.columns)
    load_data.SharedCacheIndexReturns.returns_cache.clear()
    load_data.SharedCacheIndexReturns.insample_cache.clear()
    load_data.SharedCacheIndexReturns.returns_cache[(tuple(tickers), start_date, None)] = returns_df
    calc_var_ABC.SharedCacheCopulaMSMVaR.cache.clear()
    calc_var_ABC.SharedCacheCopulaGarchVaR.cache.clear()
    calc_var_ABC.SharedCacheCopulaMRVaR.cache.clear()
    for d, tk in enumerate(tickers):
        p = cfg.model_params()[d]
        if cfg.model == "msm":
            calc_var_ABC.SharedCacheCopulaMSMVaR.cache[(tk, cfg.k)] = {"optimal_params": dict(p)}
        elif cfg.model == "garch":
            calc_var_ABC.SharedCacheCopulaGarchVaR.cache[tk] = {"optimal_params": {
                "best_pq": (1, 1),
                "best_params": np.array([p["omega"], p["alpha"], p["beta"]]),
                "best_bic": 0.0}}
        else:
            calc_var_ABC.SharedCacheCopulaMRVaR.cache[tk] = {"optimal_params": dict(p)}
    return tickers


class _PatchedNp:
    """Proxy for msm_estimation's ``np`` whose sqrt(int 2**k) returns k (Q8 patch)."""

    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        return getattr(self._real, name)

    def sqrt(self, x, *a, **kw):
        if isinstance(x, (int, np.integer)) and x > 0 and (int(x) & (int(x) - 1)) == 0:
            return float(int(x).bit_length() - 1)
        return self._real.sqrt(x, *a, **kw)


def run_case(name, cfg, patched_k=False, calc_var_kwargs=None, quiet=True):
    load_data, calc_var_ABC, calc_var_class, factory, msm_estimation = _import_reference()
    returns = synthetic.simulate_returns(cfg)
    df = synthetic.returns_frame(returns)
    start_date = str(df.index[0].date())
    tickers = _inject(cfg, df, load_data, calc_var_ABC, start_date)

    V = calc_var_class.ValueAtRiskCalcualtion
    log = _Log()
    orig_compute = V.compute_integral
    orig_copula = V.calc_copula_params
    cp = cfg.copula_params()

    def compute_integral(self, bounds):
        res = orig_compute(self, bounds)
        log.calls.append((np.array(bounds, dtype=np.float64).copy(), np.array(res, dtype=np.float64).copy()))
        return res

    captured = {}
    M = msm_estimation.MSMEstimation
    orig_fa = M.__dict__["forecasts_array"]

    def forecasts_array(rolling_windows_dict, in_sample_params, k):
        out = orig_fa.__func__(rolling_windows_dict, in_sample_params, k)
        captured["filtered_probs"] = np.array(out, dtype=np.float64)
        return out

    V.compute_integral = compute_integral
    V.calc_copula_params = lambda self: cp
    M.forecasts_array = staticmethod(forecasts_array)
    real_np = msm_estimation.np
    if patched_k:
        msm_estimation.np = _PatchedNp(real_np)
    try:
        calc = factory.ValueAtRiskCalculationFactory.create_var_calculator(
            copula_type=cfg.copula, estimation_type=cfg.model)
        kw = {"k": cfg.k} if cfg.model == "msm" else {}
        sink = io.StringIO()
        t0 = time.time()
        with contextlib.redirect_stdout(sink if quiet else sys.stdout):
            obj = V(tickers, start_date, cfg.n_in, calc, None, num_points=cfg.num_points,
                    weights=cfg.weights, **kw)
            t_init = time.time() - t0
            t1 = time.time()
            var = obj.calc_var(**(calc_var_kwargs or {}))
            t_var = time.time() - t1
    finally:
        V.compute_integral = orig_compute
        V.calc_copula_params = orig_copula
        M.forecasts_array = orig_fa
        msm_estimation.np = real_np

    out = dict(
        case=name, model=cfg.model, copula=cfg.copula, dim=cfg.dim, num_points=cfg.num_points,
        T=obj.out_sample_N, n_in=cfg.n_in, k=cfg.k, weights=cfg.weights,
        returns=returns, ptf_mean=float(obj.ptf_mean),
        copula_params=np.atleast_1d(np.asarray(cp, dtype=np.float64)),
        var=np.asarray(var, dtype=np.float64), t_init=t_init, t_calc_var=t_var,
        n_calls=len(log.calls), patched_k=patched_k,
    )
    if calc_var_kwargs:
        for key, val in calc_var_kwargs.items():
            out[f"kw_{key}"] = np.asarray(val, dtype=np.float64)
    mp = cfg.model_params()
    keys = sorted(mp[0].keys())
    out["model_param_names"] = np.array(keys)
    out["model_params"] = np.array([[p[kk] for kk in keys] for p in mp], dtype=np.float64)
    for i, (b, r) in enumerate(log.calls):
        out[f"call{i:02d}_bounds"] = b
        out[f"call{i:02d}_result"] = r
    dens, xv, step, params = obj.grids_generations_params
    out["x_values"] = np.asarray(xv, dtype=np.float64)
    out["step"] = np.asarray(step, dtype=np.float64)
    out["densities"] = np.asarray(dens, dtype=np.float64)
    out["combos"] = np.asarray(params, dtype=np.int64)
    if cfg.model == "msm":
        fbs, fc = obj.integrations_params_t
        out["forecasts_by_states"] = np.asarray(fbs, dtype=np.float64)
        out["forecasts"] = np.asarray(fc, dtype=np.float64)
        out["unique_vol_states"] = np.asarray(obj.integrations_params_static, dtype=np.float64)
        out["vol_states_array"] = np.asarray(obj.vol_states_array, dtype=np.float64)
        out["filtered_probs"] = captured["filtered_probs"]
    else:
        out["sigma_forecasts"] = np.asarray(obj.integrations_params_t[0], dtype=np.float64)
    return out


def classes_of(out):
    """Bracket class per date, re-derived from the logged calls (calc_var_class.py:125-155)."""
    r0 = out["call00_result"]
    b1 = out["call01_bounds"]
    r1 = out["call01_result"]
    f = np.where(b1[:, 0] == -3.0, r0 + r1, r0 - r1)
    up = b1[:, 1]
    cls = np.full(len(r0), -1)
    cls[f > 0.05] = 0
    cls[(f < 0.05) & (up == -3.0)] = 1
    cls[(f < 0.05) & (up == -2.0)] = 2
    cls[(f > 0.05) & (up == -2.0)] = 3
    return cls


def kat_special():
    """Known-answer vectors for the special functions on the path (scipy 1.15.3):
    t.ppf (student.py:102), norm.ppf (gaussian.py:44), erf (utils.py:20)."""
    from scipy import special, stats
    rng = np.random.default_rng(7)
    u = np.concatenate([rng.random(3000), 10.0 ** rng.uniform(-300, -1, 1500),
                        1.0 - 10.0 ** rng.uniform(-16, -1, 1500), [0.5, 0.0, 1.0, 1e-300, 1 - 1e-16]])
    out = {"u": u}
    for nu in (1.0, 2.0, 3.0, 4.5, 5.364, 6.0, 10.0, 30.0, 150.0):
        out[f"tppf_nu{nu:g}"] = stats.t.ppf(u, nu)
    out["tppf_nus"] = np.array([1.0, 2.0, 3.0, 4.5, 5.364, 6.0, 10.0, 30.0, 150.0])
    out["ndtri"] = stats.norm.ppf(u)
    # mpmath ground truth (scipy's stdtrit is clamped/inaccurate below u ~ 1e-150)
    import mpmath as mp
    mp.mp.dps = 40
    ut = np.concatenate([10.0 ** -np.arange(1, 301, 7.0), [0.3, 0.45, 0.499, 0.7, 0.9, 1 - 1e-9]])
    out["truth_u"] = ut
    for nu in (1.0, 3.0, 6.0, 30.0):
        m_nu = mp.mpf(nu)

        def lower_cdf(s10):                       # F(-10**s10), decreasing in s10
            t = mp.power(10, s10)
            return 0.5 * mp.betainc(m_nu / 2, 0.5, 0, m_nu / (m_nu + t * t), regularized=True)

        vals = []
        for uu in ut:
            p = mp.mpf(uu) if uu < 0.5 else 1 - mp.mpf(uu)
            lo, hi = mp.mpf(-20), mp.mpf(330.0 / nu + 10)
            for _ in range(120):                  # bisection on log10|t|
                mid = (lo + hi) / 2
                if lower_cdf(mid) > p:
                    lo = mid
                else:
                    hi = mid
            tv = -mp.power(10, (lo + hi) / 2)
            vals.append(float(tv if uu < 0.5 else -tv))
        out[f"truth_tppf_nu{nu:g}"] = np.array(vals)
    x = np.concatenate([np.linspace(-8, 8, 4001), rng.uniform(-30, 30, 2000), [0.0, -0.0]])
    out["erf_x"] = x
    out["erf"] = special.erf(x)
    out["ncdf"] = 0.5 * (1 + special.erf(x / np.sqrt(2)))
    return out


def main(argv):
    base = synthetic.baseline_configs()
    cases = {
        # exact BASELINE config 1 (CPU plumbing case)
        "cfg1": (base[1], False, None),
        # headline model x copula at reduced size
        "cfg2_n64": (base[2].with_(num_points=64, T=24), False, None),
        "cfg2_n256": (base[2].with_(T=6), False, None),
        "cfg3_n128": (base[3].with_(num_points=128, T=16), False, None),
        "cfg5_n64": (base[5].with_(num_points=64, T=16), False, None),
        # 3-D (Q6/Q7): unpatched k=4 and patched-k k=6 (config 4 shape)
        "cfg4_k4_n16": (base[4].with_(k=4, num_points=16, T=4), False, None),
        "cfg4_k6_n16": (base[4].with_(num_points=16, T=3), True, None),
        # high vol -> brackets [-7.5,-3.5] and [-3.5,-3]
        "cfg1_hivol": (base[1].with_(T=24, vol_scale=1.7, seed=5), False, None),
        # low vol -> VaR in (-2,0], exercising Q1
        "q1_lowvol": (base[1].with_(T=12, vol_scale=0.55, seed=11), False, None),
        # other model x copula pairs
        "msm_gauss_n64": (base[2].with_(copula="gaussian", num_points=64, T=10, seed=3), False, None),
        "garch_student_n64": (base[1].with_(copula="student", nu=4.5, num_points=64, T=10,
                                             corr=np.array([[1.0, 0.3], [0.3, 1.0]])), False, None),
        "ukf_plackett_n64": (base[5].with_(copula="plackett", theta=2.5, num_points=64, T=10), False, None),
        "msm_plackett_n64": (base[2].with_(copula="plackett", theta=4.0, num_points=64, T=8, seed=5), False, None),
        "garch3d_student_n16": (base[1].with_(dim=3, copula="student", num_points=16, T=4, nu=5.0,
                                               corr=synthetic._R3, innov_corr=synthetic._R3,
                                               garch_params=[base[1].garch_params[0]] * 3), False, None),
        # non-default calc_var arguments
        "cfg1_kwargs": (base[1].with_(T=10, seed=21), False,
                        {"obj_var": 0.01, "first_guess": -4.0, "second_guess": (-4.5, -3.0)}),
    }
    names = argv or list(cases)
    for name in names:
        if name == "kat":
            np.savez_compressed(os.path.join(HERE, "kat_special.npz"), **kat_special())
            print("kat_special.npz written")
            continue
        cfg, patched, kw = cases[name]
        t0 = time.time()
        out = run_case(name, cfg, patched_k=patched, calc_var_kwargs=kw)
        cls = classes_of(out) if kw is None else np.array([])
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        v = out["var"]
        print(f"{name}: T={out['T']} calls={out['n_calls']} wall={time.time() - t0:.1f}s "
              f"nan={int(np.isnan(v).sum())} classes={np.bincount(cls[cls >= 0], minlength=4) if cls.size else '-'} "
              f"var[min,max]=[{np.nanmin(v):.4f},{np.nanmax(v):.4f}]", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
