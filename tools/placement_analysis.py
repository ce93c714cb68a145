"""Offline analysis of tools/placement_runs.sh dumps: which dispatch positions share a CU, and
how each CU's finish time follows its dates' node counts.
usage: python3 tools/placement_analysis.py gpurun_out/<tag>/pl_c2_d1000_o0.npz [...]"""
import sys

import numpy as np

for path in sys.argv[1:]:
    z = np.load(path)
    st, var, ptf = z["st"], z["var"], float(z["ptf"])
    T = st.shape[0]
    hw = st[:, 27] & 0xFFFFFFFF
    xcc = (st[:, 27] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    b = st[:, 30]
    t0, t1 = st[:, 25].astype(np.float64), st[:, 26].astype(np.float64)
    g0 = t0.min()
    nodes = st[:, 28].astype(np.float64)
    cls = np.digitize(var - ptf, [-3.5, -3.0, -2.0])
    print(f"== {path}: T {T}, kernel span {(t1.max() - g0) / 100:.1f} us, distinct CUs {np.unique(key).size}")
    pos = np.argsort(b)                                 # dates in dispatch order
    print("  xcc of dispatch positions 0..15:", xcc[pos[:16]].tolist())
    ck = key[pos]
    uk = {k: i for i, k in enumerate(dict.fromkeys(ck.tolist()))}
    print("  CU (first-seen index) of positions 0..63:", [uk[k] for k in ck[:64].tolist()])
    print("  CU of positions 256..287:", [uk[k] for k in ck[256:288].tolist()] if T > 288 else "-")
    same = np.array([uk[k] for k in ck.tolist()])
    # per CU: dates, node sum, first start, last end
    rows = []
    for k in np.unique(key):
        m = key == k
        rows.append((m.sum(), nodes[m].sum(), (t0[m].min() - g0) / 100, (t1[m].max() - g0) / 100,
                     int((cls[m] == 3).sum())))
    rows = np.array(rows)
    print(f"  per CU: dates {np.bincount(rows[:, 0].astype(int)).tolist()} (histogram), node sum mean "
          f"{rows[:, 1].mean():.0f} max {rows[:, 1].max():.0f} min {rows[:, 1].min():.0f}")
    print(f"  per CU finish (us): mean {rows[:, 3].mean():.1f} p90 {np.percentile(rows[:, 3], 90):.1f} "
          f"max {rows[:, 3].max():.1f}; corr(finish, node sum) {np.corrcoef(rows[:, 3], rows[:, 1])[0, 1]:.2f}")
    for h in range(int(rows[:, 4].max()) + 1):
        m = rows[:, 4] == h
        if m.any():
            print(f"    CUs with {h} heavy dates: {m.sum():4d}  finish mean {rows[m, 3].mean():6.1f} max {rows[m, 3].max():6.1f}"
                  f"  node sum mean {rows[m, 1].mean():.0f}")
    # start-time profile: how many dates start within each 5-us window
    hist = np.histogram((t0 - g0) / 100, bins=np.arange(0, (t1.max() - g0) / 100 + 5, 5))[0]
    print("  dates starting per 5-us window:", hist.tolist()[:30])
    d = (t1 - t0) / 100
    print(f"  date duration: heavy {d[cls == 3].mean() if (cls == 3).any() else 0:.1f} us, "
          f"light {d[cls < 3].mean():.1f} us; heavy share {(cls == 3).mean():.2f}")
