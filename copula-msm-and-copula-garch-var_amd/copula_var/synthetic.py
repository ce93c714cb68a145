"""Synthetic inputs for the five BASELINE configurations.

The reference downloads index prices with yfinance (data_loader/load_data.py:59),
which is network-only.  Every run of this engine (tests, bench, golden
generation) instead uses returns simulated here, in percent log-return units
(load_data.py:65 multiplies by 100), from the same data-generating processes the
reference ships:

* MSM   : markov_switching_multifractal/generate_data.py:5-54
* GARCH : garch/generate_data.py:34-
* OU/UKF: kalman_mean_reverting/generate.py:18-38

Cross-asset dependence is injected through a Gaussian / Student-t copula on the
innovations.  All randomness comes from ``numpy.random.default_rng(seed)``.
In-sample model parameters and copula parameters are INJECTED (fixed), not
optimised -- the reference's optimisers use an unseeded RNG and are outside the
hot path.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Sequence

import numpy as np
from scipy import stats

N_IN_DEFAULT = 1135          # main.py:34
SEED_DEFAULT = 20241125


@dataclasses.dataclass
class Config:
    """One workload: model x copula x grid x dates (BASELINE.json ``configs``)."""
    name: str
    model: str                      # 'msm' | 'garch' | 'mean_reverting'
    copula: str                     # 'gaussian' | 'student' | 'plackett'
    dim: int
    num_points: int
    T: int
    n_in: int = N_IN_DEFAULT
    k: int = 4                      # MSM components
    msm_params: Optional[List[dict]] = None     # per asset {'m_0','sig','b','gamma'}
    garch_params: Optional[List[dict]] = None   # per asset {'omega','alpha','beta'}
    ukf_params: Optional[List[dict]] = None     # per asset {'a','l','q'}
    nu: float = 6.0
    corr: Optional[np.ndarray] = None
    theta: float = 3.0
    innov_copula: str = "student"   # dependence used to SIMULATE innovations
    innov_nu: float = 6.0
    innov_corr: Optional[np.ndarray] = None
    seed: int = SEED_DEFAULT
    vol_scale: float = 1.0          # multiplies simulated returns (bracket-mix tuning)

    @property
    def weights(self) -> np.ndarray:
        return np.full(self.dim, 1.0 / self.dim)

    def copula_params(self) -> np.ndarray:
        """Packed copula parameters exactly as the reference's adapters pack them
        (student_estimation.py:23-37, gaussian_estimation.py:36-44,
        plackett_estimation.py:29-37)."""
        if self.copula == "student":
            iu = np.triu_indices(self.dim, k=1)
            return np.concatenate(([float(self.nu)], np.asarray(self.corr)[iu]))
        if self.copula == "gaussian":
            iu = np.triu_indices(self.dim, k=1)
            return np.asarray(self.corr, dtype=np.float64)[iu].copy()
        if self.copula == "plackett":
            return float(self.theta)
        raise ValueError(f"unknown copula {self.copula}")

    def model_params(self) -> List[dict]:
        if self.model == "msm":
            return self.msm_params
        if self.model == "garch":
            return self.garch_params
        return self.ukf_params

    def with_(self, **kw) -> "Config":
        return dataclasses.replace(self, **kw)


def _corr2(rho: float) -> np.ndarray:
    return np.array([[1.0, rho], [rho, 1.0]])


_R3 = np.array([[1.0, 0.5, 0.4], [0.5, 1.0, 0.3], [0.4, 0.3, 1.0]])


def baseline_configs() -> Dict[int, Config]:
    """BASELINE.json configs[0..4] with the parameters of SURVEY.md §8d."""
    garch = [{"omega": 0.05, "alpha": 0.08, "beta": 0.90}] * 2
    msm2 = [{"m_0": 0.45, "sig": 1.2, "b": 3.0, "gamma": 0.3},
            {"m_0": 0.50, "sig": 1.2, "b": 3.0, "gamma": 0.3}]
    msm3 = [{"m_0": m, "sig": 1.2, "b": 3.0, "gamma": 0.3} for m in (0.45, 0.50, 0.55)]
    ukf = [{"a": 0.97, "l": 0.05, "q": 0.15}] * 2
    return {
        1: Config("cfg1_garch_gaussian_64", "garch", "gaussian", 2, 64, 50,
                  garch_params=garch, corr=_corr2(0.6), innov_copula="gaussian",
                  innov_corr=_corr2(0.6)),
        2: Config("cfg2_msm_student_256", "msm", "student", 2, 256, 1000, k=4,
                  msm_params=msm2, nu=6.0, corr=_corr2(0.5), innov_corr=_corr2(0.5)),
        3: Config("cfg3_garch_plackett_512", "garch", "plackett", 2, 512, 5000,
                  garch_params=garch, theta=3.0, innov_copula="gaussian",
                  innov_corr=_corr2(0.6)),
        4: Config("cfg4_msm_gaussian_3d_128", "msm", "gaussian", 3, 128, 2000, k=6,
                  msm_params=msm3, corr=_R3, innov_copula="gaussian", innov_corr=_R3),
        5: Config("cfg5_ukf_student_256", "mean_reverting", "student", 2, 256, 5000,
                  ukf_params=ukf, nu=6.0, corr=_corr2(0.5), innov_corr=_corr2(0.5)),
    }


def _innovations(cfg: Config, rng: np.random.Generator, n: int) -> np.ndarray:
    """Standard-normal marginals joined by a Gaussian or Student-t copula."""
    R = np.asarray(cfg.innov_corr if cfg.innov_corr is not None else np.eye(cfg.dim))
    Lc = np.linalg.cholesky(R)
    z = rng.standard_normal((n, cfg.dim)) @ Lc.T
    if cfg.innov_copula == "student":
        w = rng.chisquare(cfg.innov_nu, size=(n, 1))
        tdraw = z * np.sqrt(cfg.innov_nu / w)
        u = stats.t.cdf(tdraw, cfg.innov_nu)
        u = np.clip(u, 1e-15, 1 - 1e-15)
        return stats.norm.ppf(u)
    return z


def simulate_returns(cfg: Config) -> np.ndarray:
    """(n_in + T, dim) percent log-returns for ``cfg``."""
    rng = np.random.default_rng(cfg.seed)
    n = cfg.n_in + cfg.T
    eps = _innovations(cfg, rng, n)
    out = np.empty((n, cfg.dim))
    for d in range(cfg.dim):
        if cfg.model == "msm":
            p = cfg.msm_params[d]
            k = cfg.k
            gam = 1.0 - (1.0 - p["gamma"]) ** (p["b"] ** np.arange(k))
            m = rng.choice([p["m_0"], 2.0 - p["m_0"]], size=k)
            vol = np.empty(n)
            for t in range(n):
                flip = rng.random(k) >= 1.0 - gam / 2.0
                m = np.where(flip, 2.0 - m, m)
                vol[t] = np.sqrt(p["sig"] ** 2 * np.prod(m))
            out[:, d] = vol * eps[:, d]
        elif cfg.model == "garch":
            p = cfg.garch_params[d]
            s2 = p["omega"] / (1.0 - p["alpha"] - p["beta"])
            y_prev = 0.0
            for t in range(n):
                s2 = p["omega"] + p["alpha"] * y_prev ** 2 + p["beta"] * s2
                y_prev = np.sqrt(s2) * eps[t, d]
                out[t, d] = y_prev
        elif cfg.model == "mean_reverting":
            p = cfg.ukf_params[d]
            x = p["l"]
            for t in range(n):
                x = p["a"] * (x - p["l"]) + p["l"] + p["q"] * rng.standard_normal()
                out[t, d] = np.exp(x) * eps[t, d]
        else:
            raise ValueError(cfg.model)
    return out * cfg.vol_scale


def tickers_for(dim: int) -> List[str]:
    return [f"SYN{d}" for d in range(dim)]


def returns_frame(returns: np.ndarray, start: str = "2001-01-01"):
    """pandas DataFrame with a business-day index, as yfinance would return."""
    import pandas as pd
    idx = pd.bdate_range(start=start, periods=returns.shape[0])
    return pd.DataFrame(returns, index=idx, columns=tickers_for(returns.shape[1]))
