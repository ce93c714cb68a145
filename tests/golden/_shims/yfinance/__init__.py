"""Offline stand-in for yfinance: never called (returns are injected through
the reference's own SharedCacheIndexReturns cache).  Raises if reached."""


def download(*args, **kwargs):
    raise RuntimeError("network access is not available; inject returns via the cache")
