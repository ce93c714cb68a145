#!/bin/bash
# single-solve strategy x dates-per-launch scan (GPU box).  usage: tools/strat_scan.sh <tag> <cfgs> <strategies> <dates>
#   e.g. tools/strat_scan.sh r04j "3 5" "sorted sweep" "5000 625"
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for c in $2; do
  for st in $3; do
    for d in $4; do
      f=$out/c${c}_${st}_d$d
      timeout -k 10 240 python3 bench.py --config $c --strategy $st --dates-per-gpu $d --inflight 1 --steps 20 --warmup 3 \
          --e2e 0 --cpu-baseline 0 > $f.json 2> $f.err || { echo "cfg $c $st $d failed"; tail -5 $f.err; exit 1; }
      echo "cfg $c $st dates $d: $(python3 tools/bench_brief.py < $f.json)" | tee -a $out/scan.txt
    done
  done
done
