#!/bin/bash
# Solve-order node words and segment ends of the SORTED plans (cfg 3, 5, 2), row-major order
# (CVQ_SORT_BANK=0), for offline study of the node order.  GPU box.  usage: tools/dump_sorted.sh <tag>
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
for c in 3 5 2; do
  CVQ_SORT_BANK=0 timeout -k 10 120 python3 tools/lds_sim.py --config $c --save $out/nodes_c$c.npz > $out/c$c.txt 2>&1 \
    || { echo "cfg $c failed"; tail -5 $out/c$c.txt; exit 1; }
done
ls -la $out
