#!/bin/bash
# r04s: SORTED register fixes (range-sum ILP by instance, wide 2-D at 6 waves): parity, fitted-nu and
# small-block benches, then the round-end validation (tools/round_end.sh).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/sorted_check.sh r04s 3 5 || exit 1
out=gpurun_out/r04s
for c in 2 5; do
  timeout -k 10 240 python3 bench.py --config $c --nu 5.364 --strategy sorted --steps 20 --warmup 3 --e2e 0 --cpu-baseline 0 \
      > $out/nu_c$c.json 2> $out/nu_c$c.err || { echo "nu bench $c failed"; exit 1; }
  echo "cfg $c nu 5.364 sorted: $(python3 tools/bench_brief.py < $out/nu_c$c.json)" | tee -a $out/bench.txt
done
timeout -k 10 240 python3 bench.py --config 4 --dates-per-gpu 250 --inflight 1 --steps 20 --warmup 3 --e2e 0 --cpu-baseline 0 \
    > $out/c4_d250.json 2> $out/c4_d250.err || { echo "cfg 4 bench failed"; exit 1; }
echo "cfg 4 dates 250: $(python3 tools/bench_brief.py < $out/c4_d250.json)" | tee -a $out/bench.txt
bash tools/round_end.sh r04final2
