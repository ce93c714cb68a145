#!/bin/bash
# SORTED A/B (in-tree library vs build_variants/<v>): cfg 3 full + 625, cfg 1, cfg 5 SORTED 625, cfg 4 250
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; v=$2
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fullbatch_gpu.py tests/test_large_grid_gpu.py \
    tests/test_sorted_gpu.py tests/test_sorted_width_gpu.py > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
run() {
  CVQ_LIB=$2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 --inflight 1 > $out/b.json 2>$out/b.err \
    || { echo "$1 failed"; tail -3 $out/b.err; return 1; }
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,3), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/ab.txt
}
main=$GRAFT_REPO_ROOT/copula-msm-and-copula-garch-var_amd/copula_var/libcvq.so
for rep in 1 2; do
  for args in "--config 3 --steps 20 --warmup 3" "--config 3 --steps 50 --warmup 5 --dates-per-gpu 625" \
              "--config 1 --steps 100 --warmup 5" "--config 5 --steps 50 --warmup 5 --dates-per-gpu 625 --strategy sorted"; do
    run main $main "$args" || exit 1
    run $v $GRAFT_REPO_ROOT/build_variants/$v/libcvq.so "$args" || exit 1
  done
done
