"""Where a solve's instructions go (GPU box, under rocprofv3 --pmc; tools/valu_split.sh).

For one BASELINE workload at full size the plan runs, in this order, 3 x each of:
  A  compute_integral over an empty slab   -> tables + launch overhead (mode 1, zero nodes)
  B  compute_integral over (-100, 0]       -> A + every reachable node once (mode 1)
  C  calc_var                              -> the solve
and prints the nodes the solve evaluates per date (device count).  `--report <dir>` then
splits the solve's per-wave instruction counts into tables (A), node loops (nodes x the
per-node cost from B - A) and the rest (levels, reductions, tails).
usage: python3 tools/valu_split.py --config 5 [--strategy sorted]   (the run; mode-1 slabs need SORTED)
       python3 tools/valu_split.py --report <dir> --config 5 --nodes N --reach G --dates T
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "copula-msm-and-copula-garch-var_amd")]


def run(cfg_no, T, strategy):
    import numpy as np
    from copula_var import synthetic, tables
    from copula_var.engine import QuadraturePlan
    c = synthetic.baseline_configs()[cfg_no]
    if T:
        c = c.with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, ptf_mean, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    dens, x, step, combos = ggp
    p = QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                       vol_states=uvs, strategy=strategy)
    p.set_dates(ipt)
    T = c.T
    empty = np.tile([-100.0, -100.0], (T, 1))
    full = np.tile([-100.0, 0.0], (T, 1))
    for _ in range(3):
        p.compute_integral(empty)
    for _ in range(3):
        p.compute_integral(full)
    for _ in range(3):
        p.calc_var(ptf_mean)
    p.count_nodes(True)
    p.calc_var(ptf_mean)
    nodes = p.nodes_evaluated()
    print(json.dumps({"config": cfg_no, "dates": T, "nodes_per_date": nodes / T}), flush=True)


def report(d, nodes, reach, dates):
    rows = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if "k_sorted" not in k and "k_compact" not in k:
                continue
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(rows)
    if len(ids) < 10:
        sys.exit(f"expected >= 10 solve-kernel dispatches, got {len(ids)}")
    groups = {"A": ids[0:3], "B": ids[3:6], "C": ids[6:9]}
    avg = {g: {c: sum(rows[i][c] for i in v) / len(v) for c in rows[v[0]]} for g, v in groups.items()}
    waves = avg["C"]["SQ_WAVES"]
    wpd = waves / dates
    keys = [c for c in avg["C"] if c != "SQ_WAVES"]
    print(f"waves per date {wpd:.0f}; nodes per date: solve {nodes:.0f}, reachable {reach}")
    print(f"{'counter':26s} {'A tables':>10s} {'per node':>10s} {'C solve':>10s} {'nodes':>10s} {'rest':>10s}   (per date)")
    for c in sorted(keys):
        a = avg["A"][c] / dates
        per = (avg["B"][c] - avg["A"][c]) / dates / reach
        s = avg["C"][c] / dates
        nd = per * nodes
        print(f"{c:26s} {a:10.0f} {per * 64:10.2f} {s:10.0f} {nd:10.0f} {s - a - nd:10.0f}")
    print("per node = instructions per 64 nodes (one wave instruction per lane-node)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--dates", type=int, default=0)
    ap.add_argument("--report")
    ap.add_argument("--strategy", default="sorted")
    ap.add_argument("--nodes", type=float)
    ap.add_argument("--reach", type=float)
    a = ap.parse_args()
    if a.report:
        report(a.report, a.nodes, a.reach, a.dates)
    else:
        run(a.config, a.dates, a.strategy)
