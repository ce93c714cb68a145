"""Offline returns loader with the reference's in-sample / rolling-window semantics.

Mirrors data_loader/load_data.py of the reference: ``SharedCacheIndexReturns``,
``IndexReturnsRetriever(tickers, start_date, N, weights, end_date)`` and
``get_insample_data()`` returning the same 8-tuple (load_data.py:69-159).

Differences, all about where the returns come from (there is no network):
* ``get_index_returns`` cannot download (the reference calls yfinance,
  load_data.py:59); it raises unless the returns are injected into
  ``SharedCacheIndexReturns.returns_cache[(tuple(tickers), start_date, end_date)]``
  -- the reference's own cache short-circuit (load_data.py:21-24) -- or built
  with ``returns_from_prices`` / ``load_returns_csv``.
* ``rolling_windows_dict`` is a lazy mapping with the reference's keys (window
  end dates) and values ({ticker: centred window}), backed by one centred
  matrix, so the device forecast stage can take the whole series at once
  instead of T copies of the window (load_data.py:130-137 materialises
  T x N x dim floats).
"""
from __future__ import annotations

from collections.abc import Mapping
from dataclasses import dataclass
from typing import Optional

import numpy as np
import pandas as pd


class SharedCacheIndexReturns:
    """load_data.py:7-9."""
    returns_cache = {}
    insample_cache = {}


def returns_from_prices(prices: pd.DataFrame) -> pd.DataFrame:
    """Daily log returns x 100 of adjusted closes (load_data.py:62-67)."""
    return np.log(prices / prices.shift(1)).dropna() * 100


def load_returns_csv(path: str, prices: bool = True) -> pd.DataFrame:
    """CSV with a date index and one column per ticker (adjusted closes, or returns)."""
    df = pd.read_csv(path, index_col=0, parse_dates=True)
    return returns_from_prices(df) if prices else df


class RollingWindows(Mapping):
    """{window end date: {ticker: centred window}} for windows i = 0..T-1 of length N
    (load_data.py:130-137), backed by the centred returns matrix."""

    def __init__(self, returns: pd.DataFrame, mean: pd.Series, N: int, T: int):
        self.N, self.T = int(N), int(T)
        self.tickers = list(returns.columns)
        self.index = returns.index
        self.centred = (returns - mean).to_numpy(dtype=np.float64)      # (N + T, dim), row-wise r - mean
        self._keys = [self.index[i + self.N - 1] for i in range(self.T)]
        self._pos = {k: i for i, k in enumerate(self._keys)}

    def __len__(self):
        return self.T

    def __iter__(self):
        return iter(self._keys)

    def __getitem__(self, key):
        i = self._pos[key]
        w = self.centred[i: i + self.N]
        return {tk: w[:, d].copy() for d, tk in enumerate(self.tickers)}


def centred_series(rolling_windows_dict, tickers=None) -> np.ndarray:
    """(N + T, dim) centred series behind a rolling-window dict (ours or a plain dict
    of consecutive windows, as the reference builds).  The last row is never used by
    the forecasts (window i ends at row i + N - 1)."""
    if isinstance(rolling_windows_dict, RollingWindows):
        return rolling_windows_dict.centred
    wins = list(rolling_windows_dict.values())
    if not wins:
        raise ValueError("rolling_windows_dict is empty")
    tickers = tickers or list(wins[0].keys())
    W = np.stack([np.column_stack([w[tk] for tk in tickers]) for w in wins])   # (T, N, dim)
    if W.shape[0] > 1 and not np.array_equal(W[1:, :-1], W[:-1, 1:]):
        raise ValueError("rolling windows are not consecutive shifts of one series")
    series = np.concatenate([W[0], W[1:, -1]], axis=0)
    return np.concatenate([series, np.zeros((1, series.shape[1]))], axis=0)


@dataclass
class IndexReturnsRetriever:
    """load_data.py:11-40 (offline)."""
    tickers: list
    start_date: str
    N: int
    weights: np.ndarray
    end_date: Optional[str] = None

    def __post_init__(self):
        cache_key = (tuple(self.tickers), self.start_date, self.end_date)
        if cache_key in SharedCacheIndexReturns.returns_cache:
            self.returns = SharedCacheIndexReturns.returns_cache[cache_key]
        else:
            self.returns = self.get_index_returns(self.tickers, self.start_date, self.end_date)
            SharedCacheIndexReturns.returns_cache[cache_key] = self.returns
        self.returns = self.returns.sort_index()
        self.start_date = pd.to_datetime(self.start_date)
        self.returns = self.returns[self.returns.index >= self.start_date]
        self.returns = self.returns.dropna()

    def get_index_returns(self, tickers, start_date, end_date=None):
        raise RuntimeError(
            "no network: the reference downloads prices with yfinance (load_data.py:59); inject a returns "
            "DataFrame (log returns x 100, one column per ticker) into "
            f"SharedCacheIndexReturns.returns_cache[{(tuple(tickers), start_date, end_date)!r}] "
            "or build one with returns_from_prices / load_returns_csv")

    def get_insample_data(self):
        """load_data.py:69-159: (in_sample_dict, rolling_windows_dict, mean_returns, end_date,
        out_sample_data, out_sample_N, dim, ptf_mean)."""
        cache_key = (tuple(self.tickers), self.start_date, self.N)
        if cache_key in SharedCacheIndexReturns.insample_cache:
            return SharedCacheIndexReturns.insample_cache[cache_key]
        if len(self.returns) < self.N:
            raise ValueError(
                f"Not enough returns after the start date for in-sample estimation. "
                f"Required: {self.N}, Available: {len(self.returns)}")
        in_sample_data = self.returns.iloc[:self.N]
        dim = self.returns.shape[1]
        mean_returns = in_sample_data.mean(axis=0)
        ptf_mean = np.sum(mean_returns.values * self.weights)
        in_sample_centered = in_sample_data - mean_returns
        in_sample_dict = {tk: in_sample_centered[tk].values for tk in self.returns.columns}
        end_date = in_sample_data.index[-1]
        out_sample_data = self.returns.iloc[self.N:]
        remaining = len(out_sample_data)
        rolling = RollingWindows(self.returns, mean_returns, self.N, remaining)
        out = (in_sample_dict, rolling, mean_returns.to_dict(), end_date, out_sample_data, remaining, dim,
               ptf_mean)
        SharedCacheIndexReturns.insample_cache[cache_key] = out
        return out
