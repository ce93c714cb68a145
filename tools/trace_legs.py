"""Split a rocprofv3 kernel trace of one bench.py run into its legs (GPU-box tool).

bench.py runs, in order: the in-flight leg (warmup + steps launches of the dominant
kernel), the single-solve leg (warmup + steps, one batch at a time; two HIP events
bracket its timed launches, and bracket / steps is bench.py's "roofline" launch time),
one node-counting solve (1 launch), then the e2e leg (warmup + steps).  The dominant
kernel's dispatches, in start-time order, are cut accordingly and each leg's average
kernel duration and launch-to-launch gap are printed.

usage: python tools/trace_legs.py <dir with *kernel_trace.csv> [--steps 100 --warmup 5 --kernel k_compact
       --legs inflight,single_solve,count=1,e2e]      (name=N: a leg of N launches, all timed)
"""
import csv
import glob
import os
import sys


def arg(name, default):
    return type(default)(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    root = sys.argv[1]
    steps, warmup = arg("--steps", 100), arg("--warmup", 5)
    kern = arg("--kernel", "k_compact")
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {root}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if kern in name and "true>(" not in name:                     # k_compact: the fast instance (GEN = false)
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    per = warmup + steps
    legs, off = [], 0
    for ent in arg("--legs", "inflight,single_solve,count=1,e2e").split(","):
        nm, _, cnt = ent.partition("=")
        n_l, w_l = (int(cnt), 0) if cnt else (per, warmup)
        legs.append((nm, off + w_l, off + n_l))
        off += n_l
    print(f"{len(rows)} dispatches of {kern} (fast instance); legs of {per} = {warmup} warmup + {steps} timed")
    for nm, lo, hi in legs:
        seg = rows[lo: hi]
        if not seg:
            continue
        d = [(e - s) / 1e3 for s, e, _ in seg]
        span = (seg[-1][1] - seg[0][0]) / 1e3
        gaps = [(seg[i + 1][0] - seg[i][1]) / 1e3 for i in range(len(seg) - 1)]
        gap = f"  mean end->next start {sum(gaps) / len(gaps):7.2f} us" if gaps else ""
        print(f"  {nm:13s} launches {len(d):4d}  avg {sum(d) / len(d):8.2f} us  min {min(d):8.2f}  max {max(d):8.2f}"
              f"  first-start..last-end {span:9.1f} us{gap}")
    if rows:
        print(f"  kernel: {rows[0][2][:160]}")


if __name__ == "__main__":
    main()
