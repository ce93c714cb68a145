"""Time the device MSM forecast stage (cvq_msm_tables) alone for a BASELINE config: one
stream, HIP events around K runs.  GPU box.  usage: python tools/time_msm_tables.py [--config 4]"""
import os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "copula-msm-and-copula-garch-var_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
import numpy as np
import torch
from copula_var import engine, synthetic, tables

cfg_no = int(sys.argv[sys.argv.index("--config") + 1]) if "--config" in sys.argv else 4
K = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
c = synthetic.baseline_configs()[cfg_no]
rets = synthetic.simulate_returns(c)
_, _, centred, T = tables.insample_split(rets, c.n_in, c.weights)
vsa = np.array([tables.msm_vol_states(c.k, p["m_0"], p["sig"]) for p in c.msm_params])
smap, uvs = tables.unique_vol_map(vsa)
prm = [[p["m_0"], p["sig"], p["b"], p["gamma"]] for p in c.msm_params]
mt = engine.MsmTables(prm, c.k, smap, uvs.shape[1], c.n_in, T, 0)
r_dev = torch.tensor(np.ascontiguousarray(centred[:-1].T), dtype=torch.float64, device="cuda")
for _ in range(3):
    mt.run(r_dev)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    mt.run(r_dev)
e1.record()
torch.cuda.synchronize()
mt.status()
print(f"cfg {cfg_no} k {c.k} dim {c.dim} T {T} n_in {c.n_in}: cvq_msm_tables {e0.elapsed_time(e1) / K * 1e3:.1f} us per run")
