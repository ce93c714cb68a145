#!/bin/bash
# GPU box: dispatch-order A/B (CVQ_DATE_ORDER=0/1) on the single solve of every SORTED / COMPACT
# workload and the 1/8 blocks, interleaved, 2 reps.  usage: tools/order_ab.sh <tag>
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for rep in 1 2; do
  for cd in "2 1000" "5 5000" "5 625" "3 5000" "3 625" "4 2000" "4 250"; do
    set -- $cd
    for v in 0 1; do
      CVQ_DATE_ORDER=$v timeout -k 10 240 python3 bench.py --config $1 --dates-per-gpu $2 --inflight 1 --steps 20 \
          --warmup 3 --e2e 0 --cpu-baseline 0 > $out/c$1_d$2_o${v}_$rep.json 2> $out/c$1_d$2_o${v}_$rep.err \
        || { echo "cfg $1 dates $2 order $v failed rc=$?"; tail -5 $out/c$1_d$2_o${v}_$rep.err; exit 1; }
      echo "cfg $1 dates $2 order $v rep $rep: $(python3 tools/bench_brief.py < $out/c$1_d$2_o${v}_$rep.json)" | tee -a $out/order_ab.txt
    done
  done
done
