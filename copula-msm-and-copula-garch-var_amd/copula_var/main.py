"""Command-line driver mirroring the reference's main.py (main.py:25-75), offline.

    python -m copula_var.main --prices prices.csv --tickers ^GSPC ^IXIC \\
        --start 2009-04-15 --end 2015-10-12 --n-in 1135 --copula student \\
        --estimation garch msm --num-points 100 --k 4 --out var.csv --plot var.png

The reference downloads adjusted closes with yfinance; here they come from a CSV
(date index, one column per ticker), converted to the reference's log returns x 100
and put into the loader's cache under the reference's key (load_data.py:21-24).
Then, per estimation type, the pipeline main.py runs: factory -> ValueAtRiskCalcualtion
(in-sample fit, marginals, copula fit, forecasts) -> calc_var, all on the device.
The VaR series (one column per estimation type) and the equal-weight portfolio
returns go to --out; --plot saves main.py's plot_var_and_returns figure to a file.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np
import pandas as pd

from .data_loader.load_data import SharedCacheIndexReturns, load_returns_csv
from .utils.calc_var_class import ValueAtRiskCalcualtion
from .utils.factory import ValueAtRiskCalculationFactory


def plot_var_and_returns(series: dict, portfolio_returns, path: str) -> None:
    """main.py:6-21, saved to `path` instead of shown."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure(figsize=(10, 6))
    for (name, var), style in zip(series.items(), ["-", "--", "-."]):
        plt.plot(range(len(var)), var, label=f"{name.upper()} VaR", linestyle=style, alpha=0.8)
    plt.plot(range(len(portfolio_returns)), portfolio_returns, label="Portfolio Returns", linestyle=":", alpha=0.8)
    plt.title("VaR and Portfolio Returns Over Time")
    plt.xlabel("Time")
    plt.ylabel("Value")
    plt.legend()
    plt.grid(True)
    plt.savefig(path)
    plt.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--prices", required=True, help="CSV of adjusted closes (date index, one column per ticker)")
    ap.add_argument("--returns", action="store_true", help="the CSV already holds log returns x 100")
    ap.add_argument("--tickers", nargs="+", required=True)
    ap.add_argument("--start", required=True)
    ap.add_argument("--end", default=None)
    ap.add_argument("--n-in", type=int, default=1135, help="in-sample days (main.py:34)")
    ap.add_argument("--copula", default="student", choices=["student", "gaussian", "plackett"])
    ap.add_argument("--estimation", nargs="+", default=["garch", "msm"], choices=["garch", "msm", "mean_reverting"])
    ap.add_argument("--num-points", type=int, default=100)
    ap.add_argument("--k", type=int, default=4, help="MSM components")
    ap.add_argument("--weights", type=float, nargs="+", default=None)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", default=None, help="CSV of the VaR series")
    ap.add_argument("--plot", default=None, help="PNG of main.py's VaR / returns plot")
    a = ap.parse_args(argv)

    df = load_returns_csv(a.prices, prices=not a.returns)[a.tickers]
    SharedCacheIndexReturns.returns_cache[(tuple(a.tickers), a.start, a.end)] = df
    weights = np.array(a.weights if a.weights else [1.0 / len(a.tickers)] * len(a.tickers))
    out, runs = {}, {}
    for est in a.estimation:
        calc = ValueAtRiskCalculationFactory.create_var_calculator(copula_type=a.copula, estimation_type=est)
        kw = {"k": a.k} if est == "msm" else {}
        runs[est] = ValueAtRiskCalcualtion(a.tickers, a.start, a.n_in, calc, a.end, num_points=a.num_points,
                                           weights=weights, device=a.device, **kw)
        out[est] = runs[est].calc_var()
        print(f"{est}/{a.copula}: {out[est].size} dates, mean VaR {np.nanmean(out[est]):.4f}", file=sys.stderr)
    first = runs[a.estimation[0]]
    portfolio = first.out_sample_data.mean(axis=1).to_numpy()                    # main.py:73
    if a.out:
        idx = first.out_sample_data.index[:len(out[a.estimation[0]])]
        frame = pd.DataFrame({f"var_{k}": v for k, v in out.items()}, index=idx)
        frame["portfolio_return"] = portfolio[:len(frame)]
        frame.to_csv(a.out)
    if a.plot:
        plot_var_and_returns(out, portfolio, a.plot)
    return 0


if __name__ == "__main__":
    sys.exit(main())
