#!/bin/bash
# GPU box: parity suites touched by the dead-entry fast records, then single-solve benches.
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_fullbatch_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_gpu_parity.py \
    tests/test_sorted_gpu.py tests/test_sorted_width_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $out/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for cd in "5 5000" "5 625" "3 5000" "2 1000"; do
  set -- $cd
  timeout -k 10 240 python3 bench.py --config $1 --dates-per-gpu $2 --steps 50 --warmup 5 --e2e 1 --cpu-baseline 0 \
      > $out/c$1_d$2.json 2> $out/c$1_d$2.err || { echo "bench $cd failed"; tail -5 $out/c$1_d$2.err; exit 1; }
  echo "cfg $1 dates $2: $(python3 tools/bench_brief.py < $out/c$1_d$2.json)" | tee -a $out/bench.txt
done
timeout -k 10 240 python3 bench.py --config 5 --strategy compact --steps 50 --warmup 5 --e2e 0 --cpu-baseline 0 \
    > $out/c5_compact.json 2> $out/c5_compact.err && echo "cfg 5 compact: $(python3 tools/bench_brief.py < $out/c5_compact.json)" | tee -a $out/bench.txt
