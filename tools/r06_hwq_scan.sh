#!/bin/bash
# batches in flight with 8 hardware queues per process (GPU_MAX_HW_QUEUES=8) against the default 4
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
for rep in 1 2; do
  for q in 4 8; do
    for n in 3 4 6; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --inflight $n --other-configs none --cpu-baseline 0 --e2e 0 --single 0 \
          > $out/b.json 2>$out/b.err || { echo "q $q n $n failed"; tail -3 $out/b.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$out/b.json')); print('hwq $q inflight $n', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,2), d['var_checksum'])" | tee -a $out/hwq.txt
    done
  done
done
