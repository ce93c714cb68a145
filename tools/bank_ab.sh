#!/bin/bash
# SORTED bank-aware node order: parity tests, LDS model and bench A/B (CVQ_SORT_BANK=1 vs 0).
# GPU box.  usage: tools/bank_ab.sh <tag>
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_sorted_gpu.py tests/test_sorted_width_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_gpu_parity.py \
    > $out/pytest.txt 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for c in 3 5 2; do
  timeout -k 10 120 python3 tools/lds_sim.py --config $c >> $out/lds_model.txt 2>&1 || { echo "lds_sim $c failed"; exit 1; }
  CVQ_SORT_BANK=0 timeout -k 10 120 python3 tools/lds_sim.py --config $c --unaligned >> $out/lds_model_r03.txt 2>&1 || exit 1
done
for c in 3 5; do
  for b in 1 0 1 0; do
    CVQ_SORT_BANK=$b timeout -k 10 240 python3 bench.py --config $c --steps 20 --warmup 3 --e2e 0 --cpu-baseline 0 \
        > $out/c${c}_b${b}.json 2> $out/c${c}_b${b}.err || { echo "bench $c $b failed"; tail -5 $out/c${c}_b${b}.err; exit 1; }
    echo "cfg $c bank $b: $(python3 tools/bench_brief.py < $out/c${c}_b${b}.json)" | tee -a $out/ab.txt
  done
  for d in 625 1250; do
    for b in 1 0; do
      CVQ_SORT_BANK=$b timeout -k 10 240 python3 bench.py --config $c --dates-per-gpu $d --inflight 1 --steps 20 --warmup 3 \
          --e2e 0 --cpu-baseline 0 > $out/c${c}_d${d}_b${b}.json 2> $out/c${c}_d${d}_b${b}.err || exit 1
      echo "cfg $c dates $d bank $b: $(python3 tools/bench_brief.py < $out/c${c}_d${d}_b${b}.json)" | tee -a $out/ab.txt
    done
  done
done
cat $out/lds_model.txt
