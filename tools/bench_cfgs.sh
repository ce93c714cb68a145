#!/bin/bash
# GPU box: the default bench line (cfg 2) and the SORTED configs' bench lines (in flight, single
# solve, end to end).  usage: tools/bench_cfgs.sh <tag> [cfgs]
set -uo pipefail
tag=$1; cfgs=${2:-"2 3 4 5"}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for c in $cfgs; do
  cb=0; [ $c -eq 2 ] && cb=1
  timeout -k 10 400 python3 bench.py --config $c --steps 50 --warmup 5 --cpu-baseline $cb > $out/bench_c$c.json 2> $out/bench_c$c.err \
    || { echo "bench cfg $c failed"; tail -5 $out/bench_c$c.err; exit 1; }
  echo "cfg $c: $(python3 tools/bench_brief.py < $out/bench_c$c.json)" | tee -a $out/bench.txt
done
