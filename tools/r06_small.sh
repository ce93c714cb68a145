#!/bin/bash
# small date blocks (strong scaling, 1/8 of the BASELINE batch): COMPACT vs SORTED for cfg 5 / cfg 2,
# SORTED widths for cfg 3 / 4 (one batch at a time)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06i
mkdir -p $out
run() {
  env $2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 --inflight 1 > $out/b.json 2>$out/b.err \
    || { echo "$1 failed"; tail -3 $out/b.err; return 1; }
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,3), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/small.txt
}
for rep in 1 2; do
  run c5_compact "X=1" "--config 5 --steps 50 --warmup 5 --dates-per-gpu 625 --strategy compact" || exit 1
  run c5_sorted "X=1" "--config 5 --steps 50 --warmup 5 --dates-per-gpu 625 --strategy sorted" || exit 1
  run c2_compact "X=1" "--config 2 --steps 50 --warmup 5 --dates-per-gpu 125 --strategy compact" || exit 1
  run c2_sorted "X=1" "--config 2 --steps 50 --warmup 5 --dates-per-gpu 125 --strategy sorted" || exit 1
  run c5_full_compact "X=1" "--config 5 --steps 30 --warmup 5 --strategy compact" || exit 1
  run c3_625 "X=1" "--config 3 --steps 50 --warmup 5 --dates-per-gpu 625" || exit 1
  run c3_full "X=1" "--config 3 --steps 20 --warmup 3" || exit 1
  run c4_250 "X=1" "--config 4 --steps 50 --warmup 5 --dates-per-gpu 250" || exit 1
  run c4_full "X=1" "--config 4 --steps 20 --warmup 3" || exit 1
done
