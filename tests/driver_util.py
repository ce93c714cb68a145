"""Helpers that drive copula_var's reference-shaped driver on a golden case the
way tests/golden/gen_golden.py drove the reference: returns injected into the
loader cache, in-sample params into the model caches, copula params fixed."""
import numpy as np


def inject(z):
    """Populate the caches for golden case z; returns (tickers, start_date, kwargs)."""
    from copula_var import synthetic
    from copula_var.data_loader.load_data import SharedCacheIndexReturns
    from copula_var.utils import calc_var_ABC as A
    df = synthetic.returns_frame(z["returns"])
    tickers = list(df.columns)
    start = str(df.index[0].date())
    SharedCacheIndexReturns.returns_cache.clear()
    SharedCacheIndexReturns.insample_cache.clear()
    SharedCacheIndexReturns.returns_cache[(tuple(tickers), start, None)] = df
    for c in (A.SharedCacheCopulaMSMVaR, A.SharedCacheCopulaGarchVaR, A.SharedCacheCopulaMRVaR):
        c.cache.clear()
    names = [str(n) for n in z["model_param_names"]]
    model = str(z["model"])
    kw = {}
    for tk, row in zip(tickers, z["model_params"]):
        p = dict(zip(names, (float(v) for v in row)))
        if model == "msm":
            A.SharedCacheCopulaMSMVaR.cache[(tk, int(z["k"]))] = {"optimal_params": p}
            kw = {"k": int(z["k"])}
        elif model == "garch":
            A.SharedCacheCopulaGarchVaR.cache[tk] = {"optimal_params": {
                "best_pq": (1, 1), "best_params": np.array([p["omega"], p["alpha"], p["beta"]]), "best_bic": 0.0}}
        else:
            A.SharedCacheCopulaMRVaR.cache[tk] = {"optimal_params": p}
    return tickers, start, kw
