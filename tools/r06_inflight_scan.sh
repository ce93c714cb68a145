#!/bin/bash
# batches in flight (independent 1000-date plans on their own streams): 2 / 3 / 4 / 6 on cfg 2, 3 / 4 on cfg 5
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
for rep in 1 2; do
  for args in "--inflight 3" "--inflight 4" "--inflight 6" "--inflight 2" "--config 5 --steps 30 --inflight 3" "--config 5 --steps 30 --inflight 4"; do
    timeout -k 10 300 python3 bench.py $args --other-configs none --cpu-baseline 0 --e2e 0 --single 0 > $out/b.json 2>$out/b.err \
      || { echo "$args failed"; tail -3 $out/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/b.json')); print('$args', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,2), d['var_checksum'])" | tee -a $out/inflight.txt
  done
done
