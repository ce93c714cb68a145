"""Diagnostic (GPU box): SORTED compute_integral vs PREFIX near the v_cap edge."""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "copula-msm-and-copula-garch-var_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
from copula_var.engine import QuadraturePlan
G = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
z = dict(np.load(os.path.join(G, "cfg1.npz")))
per = z["sigma_forecasts"][:4]
plans = {}
for s, cap in (("sorted", 0.0), ("sorted", 1.0), ("prefix", 1.0), ("compact", 0.0)):
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), 2, z["x_values"], z["step"], z["densities"], z["combos"],
                       z["weights"], z["copula_params"], strategy=s, v_cap=cap)
    p.set_dates([per])
    plans[(s, cap)] = p
for b in ([-0.1, -0.05], [-0.05, -0.01], [-0.01, -1e-6], [-1e-6, -1e-15], [-1e-15, 0.0], [-0.1, 0.0], [-0.1, 1e-9],
          [-0.1, 0.5], [-0.5, -0.1], [-3.0, -0.1], [-3.0, 0.0], [-100.0, 0.0]):
    bounds = np.tile(b, (per.shape[0], 1))
    row = {f"{s}{cap:g}": p.compute_integral(bounds)[0] if b[1] <= cap else None for (s, cap), p in plans.items()}
    print(b, {k: (f"{v:.12e}" if v is not None else None) for k, v in row.items()}, flush=True)
print("reach", {k: p.reach_nodes for k, p in plans.items()})
