#!/bin/bash
# SORTED change check: parity tests, then single-solve benches of the SORTED configs (GPU box).
# usage: tools/sorted_check.sh <tag> [configs...]
set -uo pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_sorted_gpu.py tests/test_sorted_width_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_gpu_parity.py \
    > $out/pytest.txt 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for c in "${@:-3 5}"; do
  for d in 0 625; do
    extra=(); [ $d != 0 ] && extra=(--dates-per-gpu $d --inflight 1)
    timeout -k 10 240 python3 bench.py --config $c --steps 20 --warmup 3 --e2e 0 --cpu-baseline 0 "${extra[@]}" \
        > $out/c${c}_d$d.json 2> $out/c${c}_d$d.err || { echo "bench $c failed"; tail -5 $out/c${c}_d$d.err; exit 1; }
    echo "cfg $c dates $d: $(python3 tools/bench_brief.py < $out/c${c}_d$d.json)" | tee -a $out/bench.txt
  done
done
