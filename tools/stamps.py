"""Phase breakdown of the DIRECT / COMPACT solve kernels from s_memtime stamps
(diagnostic build aid).  Run on the GPU box:
    python tools/stamps.py [--config 2] [--strategy direct|compact|sorted]"""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "copula-msm-and-copula-garch-var_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
os.environ["CVQ_STAMPS"] = "1"
from copula_var import engine, synthetic, tables
from copula_var import _native as N

STRAT = sys.argv[sys.argv.index("--strategy") + 1] if "--strategy" in sys.argv else "direct"
cfg = synthetic.baseline_configs()[int(sys.argv[sys.argv.index("--config") + 1]) if "--config" in sys.argv else 2]
if "--dates" in sys.argv:                      # the first N dates only (e.g. 1: one date alone on the GPU)
    cfg = cfg.with_(T=int(sys.argv[sys.argv.index("--dates") + 1]))
rets = synthetic.simulate_returns(cfg)
mean, ptf, centred, T = tables.insample_split(rets, cfg.n_in, cfg.weights)
ipt, uvs, ggp = (tables.msm_integration_params(centred, cfg.n_in, cfg.msm_params, cfg.k, cfg.num_points)
                 if cfg.model == "msm" else
                 tables.sigma_integration_params(centred, cfg.n_in, cfg.model, cfg.model_params(), cfg.num_points))
dens, x, step, combos = ggp
p = engine.QuadraturePlan(cfg.model, cfg.copula, cfg.dim, x, step, dens, combos, cfg.weights, cfg.copula_params(),
                          vol_states=uvs, strategy=STRAT)
p.set_dates(ipt)
for _ in range(3):
    var, it = p.calc_var(ptf)
buf = np.zeros(T * 32, dtype=np.uint64)
N.check(N.lib().cvq_plan_debug_stamps(p._h, N.ptr(buf), buf.size), "stamps")
st = buf.reshape(T, 32).astype(np.int64)
if "--dump" in sys.argv:                       # raw per-date stamps + VaR for offline analysis
    np.savez_compressed(sys.argv[sys.argv.index("--dump") + 1], st=st, var=var, ptf=ptf)
if STRAT in ("compact", "sorted") and (st[:, 27] != 0).any():
    # placement: HW_ID bits cu 11:8, sh 12, se 15:13; XCC_ID low bits in the high word
    hw = st[:, 27] & 0xFFFFFFFF
    xcc = (st[:, 27] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    dur = (st[:, 26] - st[:, 25]).astype(np.float64)
    print(f"placement: {uk.size} distinct CUs for {T} workgroups; per-CU count histogram "
          f"{dict(zip(*np.unique(cnt, return_counts=True)))}; XCDs {np.unique(xcc).size}")
    if (st[:, 20] != 0).any():
        # SIMD of each wave (HW_ID bits 5:4): are the waves that carry a date's long rows on
        # the same SIMD for every date of a CU?
        simd = (st[:, 20:24] >> 4) & 3
        for w in range(4):
            print(f"  wave {w}: SIMD histogram {np.bincount(simd[:, w], minlength=4).tolist()}")
        same = [np.unique(simd[inv == k, 0]).size == 1 for k in range(uk.size) if (inv == k).sum() > 1]
        print(f"  CUs whose dates' wave 0 all share one SIMD: {sum(same)} of {len(same)}")
        print(f"  wave SIMD = (wave + c) mod 4 for every date: "
              f"{bool(((simd - simd[:, :1]) % 4 == np.arange(4)).all())}")
    per_wg = cnt[inv]
    for c in np.unique(per_wg):
        m = per_wg == c
        print(f"  WGs on a CU with {c} dates: {m.sum():5d}  duration mean {dur[m].mean():7.0f}  max {dur[m].max():7.0f}"
              f" (10 ns ticks)")
    # arrival order of each workgroup on its CU (0 = first started) vs duration: the SIMD
    # arbitration favours older waves
    t0 = st[:, 25].astype(np.float64)
    order = np.zeros(T, dtype=int)
    for k in range(uk.size):
        idx = np.nonzero(inv == k)[0]
        order[idx[np.argsort(t0[idx], kind="stable")]] = np.arange(idx.size)
    print("  duration by arrival order on the CU:",
          " ".join(f"#{o}: {dur[order == o].mean():.0f}" for o in np.unique(order)))
    # by bracket class of the solved VaR (calc_var_class.py:137-149): (<-3.5], (-3.5,-3], (-3,-2], (-2,0]
    v = var - ptf
    cls = np.digitize(v, [-3.5, -3.0, -2.0])
    print("  duration by VaR bracket (<-3.5, -3.5..-3, -3..-2, -2..0):",
          " ".join(f"{dur[cls == c].mean():.0f} (n={int((cls == c).sum())})" for c in range(4) if (cls == c).any()))
if STRAT == "direct":
    names = ["tables", "rowsetup", "slab1", "slab2", "bracket"] + [f"it{i}" for i in range(it)]
    cols = list(range(6 + it))
else:   # COMPACT / SORTED: 0 start, 1 tables, 2 slab1, 3 slab2, 4 bracket, 5+it block levels, 29 tail build, 31 end
    rt = st[:, 25:27].copy()
    lev = [i for i in range(5, 20) if (st[:, i] != 0).any()]
    cols = [0, 1, 2, 3, 4] + lev + [29, 31]
    names = ["tables", "slab1", "slab2", "bracket"] + [f"lev{i - 5}" for i in lev] + ["tailbuild", "tail"]
if STRAT in ("sorted", "sweep"):
    nodes = st[:, 28]
    print(f"nodes evaluated per date: mean {nodes.mean():.0f} p50 {np.median(nodes):.0f} max {nodes.max()} "
          f"(reachable {p.reach_nodes})")
st = st[:, cols]
for c in range(1, st.shape[1]):                 # dates that skipped a phase: zero length
    st[:, c] = np.where(st[:, c] == 0, st[:, c - 1], st[:, c])
d = np.diff(st, axis=1)
print("strategy", STRAT, "iterations", it, "dates", T)
tot = st[:, -1] - st[:, 0]
print(f"per-WG total cycles: mean {tot.mean():.0f}  max {tot.max():.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:9s} mean {d[:, i].mean():9.0f}  max {d[:, i].max():9.0f}")
slow = np.argsort(tot)[-max(1, T // 20):]        # slowest 5% of the workgroups
print("slowest 5%: mean cycles by phase:", " ".join(f"{nm}={d[slow, i].mean():.0f}" for i, nm in enumerate(names)))
if STRAT in ("sorted", "sweep") and T <= 16:      # dates alone on the GPU: per-date phases
    for i in range(T):
        print(f"  date {i}: nodes {int(nodes[i])} us {(rt[i, 1] - rt[i, 0]) / 100:.1f} phases "
              + " ".join(f"{nm}={d[i, k]}" for k, nm in enumerate(names)))
if STRAT != "direct":
    r0 = rt[:, 0] - rt[:, 0].min()
    r1 = rt[:, 1] - rt[:, 0].min()
    print("realtime (10 ns ticks): start spread max %d; end max %d p50 %d; WG duration mean %.0f max %d"
          % (r0.max(), r1.max(), np.median(r1), (r1 - r0).mean(), (r1 - r0).max()))
