#!/bin/bash
# Round 6, first GPU pass: the new parity tests (UKF variance regime, e2e full batches, RCCL
# world 1, integrated_function, n > 512, device scope) + the full-batch suite, smoke, a
# steps/warmup scan of the default bench line (the 20-step driver gap) and the
# fixed-slab schedule A/B (CVQ_FPAIR=0: the (r, n-1-r) pairing, CVQ_SPEC=0: no speculative
# second slab).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06a
mkdir -p $out
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_ukf_variance_gpu.py tests/test_device_scope_gpu.py tests/test_rccl_gpu.py \
    tests/test_integrated_function_gpu.py tests/test_large_grid_gpu.py tests/test_e2e_fullbatch_gpu.py \
    tests/test_fullbatch_gpu.py tests/test_forecast_device_gpu.py tests/test_gpu_parity.py \
    > $out/pytest_new.txt 2>&1; rc=$?
tail -25 $out/pytest_new.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { echo smoke failed; exit 1; }
tail -1 $out/smoke.txt
b() {   # label, env, args
  env $2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>/dev/null || return 1
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,2), round(d['single_solve']['value']/1e6,2), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/bench_scan.txt
}
for i in 1 2; do
  b new "CVQ_FPAIR=1" "--steps 100 --warmup 5" || exit 1
  b nospec "CVQ_SPEC=0" "--steps 100 --warmup 5" || exit 1
  b old "CVQ_FPAIR=0" "--steps 100 --warmup 5" || exit 1
  b new5 "CVQ_FPAIR=1" "--config 5 --steps 50 --warmup 5" || exit 1
  b nospec5 "CVQ_SPEC=0" "--config 5 --steps 50 --warmup 5" || exit 1
  b old5 "CVQ_FPAIR=0" "--config 5 --steps 50 --warmup 5" || exit 1
done
b s20 "CVQ_FPAIR=1" "--steps 20 --warmup 5" || exit 1
b s20 "CVQ_FPAIR=1" "--steps 20 --warmup 5" || exit 1
b s20w50 "CVQ_FPAIR=1" "--steps 20 --warmup 50" || exit 1
for d in 625 1250; do
  b new5d$d "CVQ_FPAIR=1" "--config 5 --steps 50 --warmup 5 --dates-per-gpu $d --inflight 1" || exit 1
  b old5d$d "CVQ_FPAIR=0" "--config 5 --steps 50 --warmup 5 --dates-per-gpu $d --inflight 1" || exit 1
done
