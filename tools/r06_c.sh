#!/bin/bash
# speculation A/B after moving the policy word off the ticket's cache line; stamps of cfg 5 both ways
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r06c}
mkdir -p $out
b() {
  env $2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>/dev/null || return 1
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,2), round(d['single_solve']['value']/1e6,2), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/bench_scan.txt
}
b new5 "CVQ_SPEC=1" "--config 5 --steps 50 --warmup 5" || exit 1
b nospec5 "CVQ_SPEC=0" "--config 5 --steps 50 --warmup 5" || exit 1
b new "CVQ_SPEC=1" "--steps 100 --warmup 5" || exit 1
b nospec "CVQ_SPEC=0" "--steps 100 --warmup 5" || exit 1
CVQ_SPEC=1 timeout -k 10 200 python3 tools/stamps.py --config 5 --strategy compact > $out/stamps_spec.txt 2>&1 || exit 1
CVQ_SPEC=0 timeout -k 10 200 python3 tools/stamps.py --config 5 --strategy compact > $out/stamps_nospec.txt 2>&1 || exit 1
head -40 $out/stamps_spec.txt; head -40 $out/stamps_nospec.txt
