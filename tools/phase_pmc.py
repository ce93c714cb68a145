"""Phase cost of the COMPACT solve from ablation builds (GPU box, under rocprofv3 --pmc).
Run mode: one cfg-2 plan (1000 dates), 5 solves (errors ignored: an ablation build stops each
date early, so its VaR is meaningless).  Report mode: per-variant per-date counters of the
k_compact dispatches and the differences between consecutive variants.
usage: python3 tools/phase_pmc.py --run [--config 2]
       python3 tools/phase_pmc.py --report <dir> base abl3 abl2 abl1"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "copula-msm-and-copula-garch-var_amd")]


def run(cfg_no):
    from copula_var import synthetic, tables
    from copula_var.engine import QuadraturePlan
    c = synthetic.baseline_configs()[cfg_no]
    rets = synthetic.simulate_returns(c)
    _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    dens, x, step, combos = ggp
    p = QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                       vol_states=uvs, strategy="compact")
    p.set_dates(ipt)
    for _ in range(5):
        try:
            p.calc_var(ptf)
        except Exception as e:                       # noqa: BLE001 -- ablation builds
            print("solve:", type(e).__name__, str(e)[:80])


def report(d, variants, dates=1000):
    prev = None
    for v in variants:
        rows = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(d, v, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_compact" in r.get("Kernel_Name", "") and "true, false>" in r.get("Kernel_Name", ""):
                    rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if not rows:
            print(v, "no k_compact dispatches")
            continue
        avg = {c: sum(rows[i][c] for i in rows) / len(rows) / dates for c in next(iter(rows.values()))}
        line = " ".join(f"{c.replace('SQ_INSTS_', '')}={avg[c]:.0f}" for c in sorted(avg))
        print(f"{v:6s} per date: {line}")
        if prev is not None:
            print(f"       {prev[0]} - {v}: " + " ".join(f"{c.replace('SQ_INSTS_', '')}={prev[1][c] - avg[c]:.0f}"
                                                   for c in sorted(avg)))
        prev = (v, avg)


if __name__ == "__main__":
    if "--report" in sys.argv:
        i = sys.argv.index("--report")
        report(sys.argv[i + 1], sys.argv[i + 2:])
    else:
        run(int(sys.argv[sys.argv.index("--config") + 1]) if "--config" in sys.argv else 2)
