"""Lane slots of COMPACT's bisection-level slabs (VERDICT r05 #3's lane-balanced level sum).

For each bracket of k_compact's tree (the solve's default first / second guesses), every cell
the levels can sum (both children of each cell above the block-tail cap) is a date-independent
node set: row r holds columns (cut_r(lo), cut_r(hi)].  Row-per-thread (the kernel) costs each
wave its longest row; a host schedule like the fixed slabs' (half-rows sorted, longest paired
with shortest, two loops) costs each wave its longest half-row pair.  Prints nodes and lane
slots (64 x the wave's loop trips, summed over waves and cells) for both."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import forecast as F  # noqa: E402


def main(cfg=2, NT=256, blk=12):
    z = np.load(f"tests/golden/fullbatch_cfg{cfg}.npz", allow_pickle=False)
    w0, w1 = (float(v) for v in z["weights"])
    n = int(z["x_values"].shape[0])
    x, _ = F.x_grid(n, str(z["model"]))

    def cut(v):
        return np.array([np.searchsorted(x * w0 + x[r] * w1, v, side="right") for r in range(n)])

    def rowper(lens):
        L = np.zeros(((len(lens) + 63) // 64) * 64, int)
        L[:len(lens)] = lens
        return int((L.reshape(-1, 64).max(1) * 64).sum())

    def sched(lens):
        M = NT * ((n + NT - 1) // NT)
        h = []
        for l in lens:
            m = (l + 1) // 2
            h += [m, l - m]
        h = sorted(h + [0] * (2 * M - len(h)), reverse=True)
        return sum((max(h[e] for e in range(k * 64, k * 64 + 64)) +
                    max(h[2 * M - 1 - e] for e in range(k * 64, k * 64 + 64))) * 64 for k in range(M // 64))

    cap = NT * blk
    for b, (lo, hi) in enumerate([(-7.5, -3.5), (-3.5, -3.0), (-2.0, 0.0), (-3.0, -2.0)]):
        cells, nodes, s_row, s_sch = [(lo, hi)], 0, 0, 0
        for _ in range(24):
            nxt = []
            for a, c in cells:
                mid = (a + c) / 2
                for p, q in ((a, mid), (mid, c)):
                    lens = np.maximum(cut(q) - cut(p), 0)
                    nn = int(lens.sum())
                    if nn == 0:
                        continue
                    nodes += nn
                    s_row += rowper(lens)
                    s_sch += sched(lens)
                    if nn > cap:
                        nxt.append((p, q))
            cells = nxt
            if not cells:
                break
        print(f"cfg {cfg} bracket {b} ({lo}, {hi}]: nodes {nodes}, row-per-thread slots {s_row} "
              f"({s_row / max(nodes, 1):.2f}x), scheduled half-row pairs {s_sch} ({s_sch / max(nodes, 1):.2f}x)")


if __name__ == "__main__":
    for cfg in (2, 5):
        main(cfg)
