#!/bin/bash
# forecast-stage A/B (end-to-end leg): in-tree library vs build_variants/<v> on cfg 5 (UKF) and cfg 3 (GARCH),
# after the forecast parity tests
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; v=$2
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_e2e_fullbatch_gpu.py \
    tests/test_ukf_variance_gpu.py tests/test_forecast_device_gpu.py tests/test_gpu_parity.py > $out/pytest.txt 2>&1 \
    || { tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
run() {
  CVQ_LIB=$2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 > $out/b.json 2>$out/b.err \
    || { echo "$1 failed"; tail -3 $out/b.err; return 1; }
  python3 -c "
import json; d=json.load(open('$out/b.json')); e=d.get('e2e') or {}; print('$1', '$3', round(d['value']/1e6,3), round(d['single_solve']['value']/1e6,3), round((e.get('value') or 0)/1e6,3), e.get('var_matches_resident_tables'), d['var_checksum'])" | tee -a $out/ab.txt
}
main=$GRAFT_REPO_ROOT/copula-msm-and-copula-garch-var_amd/copula_var/libcvq.so
for rep in 1 2; do
  for args in "--config 5 --steps 20 --warmup 3" "--config 3 --steps 20 --warmup 3"; do
    run main $main "$args" || exit 1
    run $v $GRAFT_REPO_ROOT/build_variants/$v/libcvq.so "$args" || exit 1
  done
done
