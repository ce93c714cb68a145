"""LDS bank-conflict model of k_sorted's 2-D node loop (range_sum), from the plan's own node
words.  GPU box (the plan is built by the library; no kernel is timed).  For every wave-instruction
of a strided range sum over sorted positions [ps, pe) -- thread t of the 256 reads position
p0 + t + u NT, u < kSortIlp -- the two ds_read_b128 record reads (rec0 = 16 i0, rec2 = 16 (ns + j))
are split into the MI355X_MICROARCH.md lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...);
a group costs one LDS cycle per distinct 16-B address on its busiest bank slot ((a / 16) mod 16),
so a conflict-free b128 read costs 4 cycles.
usage: python tools/lds_sim.py [--config 3] [--dates 8] [--unaligned]
(--unaligned: lanes start at each range's first position, the round-3 kernel)"""
import ctypes as C
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "copula-msm-and-copula-garch-var_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
from copula_var import _native as N, engine, synthetic, tables   # noqa: E402

ALIGNED = "--unaligned" not in sys.argv
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def cycles(addr, valid):
    """LDS cycles of one ds_read_b128 wave-instruction (64 byte addresses, invalid lanes masked)."""
    tot = 0
    for g in GROUPS:
        a = {int(addr[l]) for l in g if valid[l]}
        if not a:
            continue
        slots = {}
        for x in a:
            slots.setdefault((x // 16) % 16, set()).add(x)
        tot += max(len(v) for v in slots.values())
    return tot


def simulate(words, ps, pe, nt=256, ilp=4, aligned=True):
    """aligned: the rounds start at ps rounded down to 64 (lane = position mod 64, the current
    kernel); otherwise at ps (the round-3 kernel)."""
    off0 = (words & 0xFFFF).astype(np.int64)
    off2 = (words >> 16).astype(np.int64)
    c0 = c2 = n0 = 0
    start = (ps & ~63) if aligned else ps
    for p0 in range(start, pe, ilp * nt):
        for u in range(ilp):
            for w in range(nt // 64):
                p = p0 + u * nt + w * 64 + np.arange(64)
                v = (p < pe) & (p >= ps)
                if not v.any():
                    continue
                pp = np.minimum(p, pe - 1)
                c0 += cycles(off0[pp], v)
                c2 += cycles(off2[pp], v)
                n0 += 1
    return c0, c2, n0


def main():
    cfg_no = int(sys.argv[sys.argv.index("--config") + 1]) if "--config" in sys.argv else 3
    T = int(sys.argv[sys.argv.index("--dates") + 1]) if "--dates" in sys.argv else 8
    c = synthetic.baseline_configs()[cfg_no].with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    dens, x, step, combos = ggp
    p = engine.QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                              vol_states=uvs, strategy="sorted")
    p.set_dates(ipt)
    p.calc_var(ptf)
    G = p.reach_nodes
    words = np.empty(G, dtype=np.uint32)
    fix = np.zeros(6, dtype=np.int32)
    N.check(N.lib().cvq_plan_debug_nodes(p._h, words.ctypes.data_as(C.c_void_p), G, fix.ctypes.data_as(C.c_void_p)),
            "cvq_plan_debug_nodes")
    if "--save" in sys.argv:                         # solve-order words + segment ends, for offline study
        cnt = C.c_int32(0)
        N.check(N.lib().cvq_plan_debug_cuts(p._h, None, 0, C.byref(cnt)), "cvq_plan_debug_cuts")
        cuts = np.empty(cnt.value, dtype=np.int32)
        N.check(N.lib().cvq_plan_debug_cuts(p._h, cuts.ctypes.data_as(C.c_void_p), cnt.value, C.byref(cnt)),
                "cvq_plan_debug_cuts")
        np.savez(sys.argv[sys.argv.index("--save") + 1], words=words, cuts=cuts, fix=fix, n=c.num_points)
    p.close()
    print(f"cfg {cfg_no}: n {c.num_points}, reachable nodes {G}, fixed-level positions {fix.tolist()}")
    names = ["lower", "sg0", "fg", "sg1", "vmin", "vmax"]
    order = np.argsort(fix)
    for a, b in zip(order[:-1], order[1:]):
        ps, pe = int(fix[a]), int(fix[b])
        if pe - ps < 64:
            continue
        c0, c2, n0 = simulate(words, ps, pe, aligned=ALIGNED)
        print(f"  ({names[a]}, {names[b]}]: {pe - ps:7d} nodes, {n0:6d} wave reads each: rec0 {c0 / n0:5.2f} "
              f"rec2 {c2 / n0:5.2f} LDS cycles per b128 read (4 = conflict-free)")
    # deep levels: 256-node windows spread over the bracket range (the solve's late levels)
    lo, hi = int(fix.min()), int(fix.max())
    tot0 = tot2 = tn = 0
    for s in np.linspace(lo, max(lo, hi - 256), 64).astype(int):
        c0, c2, n0 = simulate(words, s, s + 256, aligned=ALIGNED)
        tot0, tot2, tn = tot0 + c0, tot2 + c2, tn + n0
    print(f"  256-node cells (64 samples): rec0 {tot0 / tn:5.2f} rec2 {tot2 / tn:5.2f} LDS cycles per b128 read")




def dump(cfg_no=2, T=4, at=0.6, count=64):
    """The (i0, j) of `count` consecutive solve-order nodes at fraction `at` of the reachable list."""
    c = synthetic.baseline_configs()[cfg_no].with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    dens, x, step, combos = ggp
    p = engine.QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                              vol_states=uvs, strategy="sorted")
    p.set_dates(ipt)
    p.calc_var(ptf)
    G = p.reach_nodes
    words = np.empty(G, dtype=np.uint32)
    N.check(N.lib().cvq_plan_debug_nodes(p._h, words.ctypes.data_as(C.c_void_p), G, None), "nodes")
    p.close()
    ns = (c.num_points + 1) & ~1
    s0 = int(at * G)
    w = words[s0:s0 + count]
    i0 = (w & 0xFFFF) // 16
    j = (w >> 16) // 16 - ns
    print("i0:", i0.tolist())
    print("j :", j.tolist())


if __name__ == "__main__":
    if "--dump" in sys.argv:
        dump(at=float(sys.argv[sys.argv.index("--dump") + 1]))
    else:
        main()
