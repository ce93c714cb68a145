#!/bin/bash
# rocprofv3 kernel-trace summaries of the SORTED configs' bench (final build).  GPU box.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for c in 3 5 4; do
  bash tools/profile.sh r05fin_c$c --config $c --e2e 0 --steps 20 > /dev/null 2>&1 || { echo "profile cfg $c failed"; exit 1; }
  python3 -c "
import csv, json
rows = list(csv.DictReader(open('gpurun_out/prof_r05fin_c$c/kernel_stats.csv')))
top = max(rows, key=lambda r: float(r['TotalDurationNs']))
b = json.load(open('gpurun_out/prof_r05fin_c$c/bench.json'))
print('cfg $c:', top['Name'][:60], 'calls', top['Calls'], 'avg', round(float(top['AverageNs'])/1e3, 1), 'us; bench events avg_launch_us', round(b['roofline']['avg_launch_us'], 1))
"
done
