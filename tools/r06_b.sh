#!/bin/bash
# Round 6 COMPACT A/B: default (host half-row schedule + speculative second slab) vs CVQ_SPEC=0
# vs CVQ_FPAIR=0 (the r05 pairing, no speculation), cfg 2 and cfg 5, plus 625 / 1250-date blocks.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r06b}
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fullbatch_gpu.py \
    tests/test_e2e_fullbatch_gpu.py > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
b() {   # label, env, args
  env $2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>/dev/null || return 1
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,2), round(d['single_solve']['value']/1e6,2), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/bench_scan.txt
}
for i in 1 2; do
  b new "CVQ_FPAIR=1" "--steps 100 --warmup 5" || exit 1
  b nospec "CVQ_SPEC=0" "--steps 100 --warmup 5" || exit 1
  b old "CVQ_FPAIR=0" "--steps 100 --warmup 5" || exit 1
  b new5 "CVQ_FPAIR=1" "--config 5 --steps 50 --warmup 5" || exit 1
  b nospec5 "CVQ_SPEC=0" "--config 5 --steps 50 --warmup 5" || exit 1
  b old5 "CVQ_FPAIR=0" "--config 5 --steps 50 --warmup 5" || exit 1
done
for d in 625 1250; do
  b new5d$d "CVQ_FPAIR=1" "--config 5 --steps 50 --warmup 5 --dates-per-gpu $d --inflight 1" || exit 1
  b nospec5d$d "CVQ_SPEC=0" "--config 5 --steps 50 --warmup 5 --dates-per-gpu $d --inflight 1" || exit 1
  b old5d$d "CVQ_FPAIR=0" "--config 5 --steps 50 --warmup 5 --dates-per-gpu $d --inflight 1" || exit 1
done
b s20 "CVQ_FPAIR=1" "--steps 20 --warmup 5" || exit 1
b s20 "CVQ_FPAIR=1" "--steps 20 --warmup 5" || exit 1
