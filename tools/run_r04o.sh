#!/bin/bash
# r04o: parity after the SORTED loop / width changes, benches, width A/B at small blocks, 2-rank bench test.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/sorted_check.sh r04o 3 5 || exit 1
out=gpurun_out/r04o
for c in 3 5; do
  for w in 256 384 512; do
    CVQ_SORT_NT=$w timeout -k 10 240 python3 bench.py --config $c --dates-per-gpu 625 --inflight 1 --steps 20 --warmup 3 \
        --e2e 0 --cpu-baseline 0 > $out/w_c${c}_$w.json 2> $out/w_c${c}_$w.err || { echo "width $c $w failed"; exit 1; }
    echo "cfg $c 625 dates width $w: $(python3 tools/bench_brief.py < $out/w_c${c}_$w.json)" | tee -a $out/widths.txt
  done
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_bench_ranks_gpu.py \
    > $out/ranks.txt 2>&1 || { echo "ranks test failed"; tail -20 $out/ranks.txt; exit 1; }
tail -1 $out/ranks.txt
