"""The main.py mirror (copula_var/main.py): CSV of adjusted closes -> loader cache ->
per estimation type the full pipeline (in-sample fit, marginals, copula fit, forecasts,
calc_var) -> CSV of VaR series + main.py's plot saved to a file."""
import numpy as np
import pandas as pd
import pytest

from conftest import load_golden


def _prices_csv(tmp_path, n=None):
    from copula_var import synthetic
    r = load_golden("cfg1")["returns"]
    r = r if n is None else r[:n]
    df = synthetic.returns_frame(r)
    prices = 100.0 * np.exp(np.vstack([np.zeros((1, r.shape[1])), np.cumsum(r / 100.0, axis=0)]))
    idx = pd.bdate_range(end=df.index[-1], periods=prices.shape[0])
    p = tmp_path / "prices.csv"
    pd.DataFrame(prices, index=idx, columns=df.columns).to_csv(p)
    return p, list(df.columns), str(idx[0].date())


def test_cli_loads_prices_and_fails_loudly_without_a_gpu(tmp_path):
    from copula_var import _native as N
    from copula_var.main import main
    from copula_var.data_loader.load_data import SharedCacheIndexReturns
    from copula_var.utils import calc_var_ABC as A
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: the end-to-end run is test_cli_end_to_end")
    except ImportError:
        pass
    for c in (A.SharedCacheCopulaMSMVaR, A.SharedCacheCopulaGarchVaR, A.SharedCacheCopulaMRVaR):
        c.cache.clear()
    SharedCacheIndexReturns.returns_cache.clear()
    SharedCacheIndexReturns.insample_cache.clear()
    p, tickers, start = _prices_csv(tmp_path, n=300)
    with pytest.raises(N.NativeError):
        main(["--prices", str(p), "--tickers", *tickers, "--start", start, "--n-in", "250",
              "--estimation", "garch", "--num-points", "32"])
    key = (tuple(tickers), start, None)
    r = SharedCacheIndexReturns.returns_cache[key]                     # log returns x 100 of the closes
    np.testing.assert_allclose(r.to_numpy(), load_golden("cfg1")["returns"][:300], rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_cli_end_to_end(tmp_path):
    from copula_var.main import main
    from copula_var.data_loader.load_data import SharedCacheIndexReturns
    from copula_var.utils import calc_var_ABC as A
    for c in (A.SharedCacheCopulaMSMVaR, A.SharedCacheCopulaGarchVaR, A.SharedCacheCopulaMRVaR):
        c.cache.clear()
    SharedCacheIndexReturns.returns_cache.clear()
    SharedCacheIndexReturns.insample_cache.clear()
    p, tickers, start = _prices_csv(tmp_path)
    out, png = tmp_path / "var.csv", tmp_path / "var.png"
    assert main(["--prices", str(p), "--tickers", *tickers, "--start", start, "--n-in", "1135",
                 "--copula", "gaussian", "--estimation", "garch", "msm", "--num-points", "64",
                 "--out", str(out), "--plot", str(png)]) == 0
    f = pd.read_csv(out, index_col=0)
    assert list(f.columns) == ["var_garch", "var_msm", "portfolio_return"] and len(f) > 10
    assert np.all(np.isfinite(f[["var_garch", "var_msm"]].to_numpy())) and np.all(f[["var_garch", "var_msm"]] < 0)
    assert png.exists() and png.stat().st_size > 0
