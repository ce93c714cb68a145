#!/bin/bash
# r04y: FP64-MFMA superblock scan for k = 6: forecast tests, tables timing, cfg 4 e2e.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04y
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_forecast_device_gpu.py \
    > gpurun_out/r04y/pytest.txt 2>&1 || { echo "forecast tests failed"; tail -30 gpurun_out/r04y/pytest.txt; exit 1; }
tail -1 gpurun_out/r04y/pytest.txt
for i in 1 2; do timeout -k 10 120 python3 tools/time_msm_tables.py --config 4 --steps 20 2>&1 | tail -1; done
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --config 4 --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/r04y/c4_$i.json 2> gpurun_out/r04y/c4_$i.err \
    || { echo "bench failed"; tail -5 gpurun_out/r04y/c4_$i.err; exit 1; }
  echo "cfg 4 e2e run $i: $(python3 tools/bench_brief.py < gpurun_out/r04y/c4_$i.json)"
done
