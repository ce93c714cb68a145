#!/bin/bash
# auto-rule check: COMPACT vs SORTED for every 2-D copula on the MSM (cfg 2) and UKF (cfg 5) full batches
# (bench --copula overrides the config's copula), in flight and one batch at a time
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1
out=gpurun_out/$tag
mkdir -p $out
for cfgc in "2 gaussian" "2 plackett" "5 gaussian" "5 plackett" "2 student" "5 student"; do
  set -- $cfgc
  for st in compact sorted; do
    args="--config $1 --copula $2 --strategy $st --steps 20 --warmup 3"
    timeout -k 10 300 python3 bench.py $args --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>$out/b.err \
      || { echo "$args failed"; tail -3 $out/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/b.json')); print('$args', round(d['value']/1e6,3), round(d['single_solve']['value']/1e6,3), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/scan.txt
  done
done
