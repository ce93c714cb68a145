#!/bin/bash
# SORTED phase stamps + workgroup placement at small date blocks (GPU box).  usage: tools/stamps_scan.sh <tag>
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
for c in 5 3; do
  for nt in 256 512; do
    CVQ_SORT_NT=$nt timeout -k 10 120 python3 tools/stamps.py --config $c --strategy sorted --dates 625 \
        > $out/st_c${c}_d625_w$nt.txt 2>&1 || { echo "stamps $c $nt failed"; tail -5 $out/st_c${c}_d625_w$nt.txt; exit 1; }
  done
done
head -20 $out/*.txt
