"""Phase breakdown of the DIRECT kernel from s_memtime stamps (diagnostic build aid).
Run on the GPU box:  CVQ_STAMPS=1 python tools/stamps.py [--config 2]"""
import os, sys, json
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "copula-msm-and-copula-garch-var_amd"), os.path.join(os.path.dirname(__file__), "..")]
os.environ["CVQ_STAMPS"] = "1"
import torch
from copula_var import engine, synthetic, tables
from copula_var import _native as N
cfg = synthetic.baseline_configs()[int(sys.argv[sys.argv.index("--config") + 1]) if "--config" in sys.argv else 2]
rets = synthetic.simulate_returns(cfg)
mean, ptf, centred, T = tables.insample_split(rets, cfg.n_in, cfg.weights)
ipt, uvs, ggp = (tables.msm_integration_params(centred, cfg.n_in, cfg.msm_params, cfg.k, cfg.num_points)
                 if cfg.model == "msm" else tables.sigma_integration_params(centred, cfg.n_in, cfg.model, cfg.model_params(), cfg.num_points))
dens, x, step, combos = ggp
p = engine.QuadraturePlan(cfg.model, cfg.copula, cfg.dim, x, step, dens, combos, cfg.weights, cfg.copula_params(),
                          vol_states=uvs, strategy="direct")
p.set_dates(ipt)
for _ in range(3):
    var, it = p.calc_var(ptf)
buf = np.zeros(T * 32, dtype=np.uint64)
N.check(N.lib().cvq_plan_debug_stamps(p._h, N.ptr(buf), buf.size), "stamps")
st = buf.reshape(T, 32).astype(np.int64)
names = ["tables", "rowsetup", "slab1", "slab2", "bracket"] + [f"it{i}" for i in range(it)]
d = np.diff(st[:, :5 + it + 1], axis=1)
print("iterations", it, "dates", T)
tot = st[:, 5 + it] - st[:, 0]
print(f"per-WG total cycles: mean {tot.mean():.0f}  max {tot.max():.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:9s} mean {d[:, i].mean():9.0f}  max {d[:, i].max():9.0f}")
start = st[:, 0] - st[:, 0].min()
print("WG start spread (cycles): max", start.max())
