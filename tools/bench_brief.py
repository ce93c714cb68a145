"""One-line summary of a bench.py JSON line read from stdin."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
k = {n: round(v["avg_us"], 1) for n, v in d["kernels"].items()}
print(round(d["value"]), round(d["ms_per_step"] * 1e3, 1), "us/step", d["var_checksum"], d["var_nan"], k)
