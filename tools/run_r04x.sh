#!/bin/bash
# r04x: scan-filter step normalisation (every 1 / 4 / 8 steps): forecast tests, tables timing, cfg 4 e2e.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04x
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_forecast_device_gpu.py \
    > gpurun_out/r04x/pytest.txt 2>&1 || { echo "forecast tests failed"; tail -20 gpurun_out/r04x/pytest.txt; exit 1; }
tail -1 gpurun_out/r04x/pytest.txt
bash tools/run_scanwin_abl.sh sn4 sn1 sn8 sn4 sn1 || exit 1
echo "== cfg 4 e2e"; AB_OUT=gpurun_out/r04x/e2e bash tools/ab.sh "--config 4 --steps 20 --warmup 3" sn4 sn1 || exit 1
