#!/bin/bash
# GPU box: per-date stamps (placement HW_ID / XCC_ID, dispatch position, start / end realtime, nodes)
# of full solves, dumped for offline analysis (tools/placement_analysis.py).
# usage: tools/placement_runs.sh <tag>
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for spec in "2 compact 1000" "5 sorted 625" "5 sorted 5000"; do
  set -- $spec
  for o in 0; do
    timeout -k 10 120 python3 tools/stamps.py --config $1 --strategy $2 --dates $3 \
        --dump $out/pl_c$1_d$3_o$o.npz > $out/pl_c$1_d$3_o$o.txt 2>&1 \
      || { echo "stamps $spec order $o failed"; tail -5 $out/pl_c$1_d$3_o$o.txt; exit 1; }
    head -3 $out/pl_c$1_d$3_o$o.txt
  done
done
