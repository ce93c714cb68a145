#!/bin/bash
# GPU box: full GPU suite, then the cfg 5 (auto = COMPACT) and cfg 2 bench lines with e2e.
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.txt 2>&1 \
    || { echo "pytest failed"; tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for cd in "5 5000" "5 625" "2 1000"; do
  set -- $cd
  timeout -k 10 240 python3 bench.py --config $1 --dates-per-gpu $2 --steps 50 --warmup 5 --cpu-baseline 0 \
      > $out/c$1_d$2.json 2> $out/c$1_d$2.err || { echo "bench $cd failed"; tail -5 $out/c$1_d$2.err; exit 1; }
  echo "cfg $1 dates $2: $(python3 tools/bench_brief.py < $out/c$1_d$2.json)" | tee -a $out/bench.txt
done
