#!/bin/bash
# GPU box: UKF forecast-pass variant (build_variants/ukf2) -- its parity tests, then cfg 5 end to end
# against the base library, interleaved.  usage: tools/ukf_ab.sh <tag>
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/ukf2/libcvq.so timeout -k 10 300 python3 -u -m pytest tests/test_insample_gpu.py \
    tests/test_gpu_parity.py tests/test_forecast_device_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for r in 1 2; do for v in base ukf2; do
  CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 240 python3 bench.py --config 5 --steps 20 \
      --warmup 3 --cpu-baseline 0 --other-configs none > $out/c5_${v}_$r.json 2> $out/c5_${v}_$r.err \
    || { echo "bench $v failed"; tail -5 $out/c5_${v}_$r.err; exit 1; }
  echo "cfg 5 $v rep $r: $(python3 tools/bench_brief.py < $out/c5_${v}_$r.json)" | tee -a $out/ab.txt
done; done
