"""One-line summary of a bench.py JSON line read from stdin."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
k = {n: round(v["avg_us"], 1) for n, v in d["kernels"].items()}
ss = d.get("single_solve") or {}
rf = d.get("roofline") or {}
e2e = d.get("e2e") or {}
print(round(d["value"]), round(d["ms_per_step"] * 1e3, 1), "us/step", "single", round(ss.get("value", 0)),
      "fp64", round(rf.get("frac", 0), 4), "launch_us", round(rf.get("avg_launch_us", 0), 1), d["var_checksum"],
      d["var_nan"], k, *(["e2e", round(e2e.get("value", 0)), e2e.get("var_matches_resident_tables")] if e2e else []))
