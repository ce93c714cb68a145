#!/bin/bash
# COMPACT Gaussian A/B: in-tree library vs build_variants/<v>, full GPU suite first, then cfg 1 (GARCH Gaussian)
# at 1000 dates with --strategy compact, SORTED (in-tree) beside it
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; v=$2
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $out/pytest.txt 2>&1 \
    || { tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
run() {
  CVQ_LIB=$2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>$out/b.err \
    || { echo "$1 failed"; tail -3 $out/b.err; return 1; }
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,3), round(d['single_solve']['value']/1e6,3), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/ab.txt
}
main=$GRAFT_REPO_ROOT/copula-msm-and-copula-garch-var_amd/copula_var/libcvq.so
for rep in 1 2; do
  c="--config 1 --dates-per-gpu 1000 --steps 30 --warmup 3"
  run main $main "$c --strategy compact" || exit 1
  run $v $GRAFT_REPO_ROOT/build_variants/$v/libcvq.so "$c --strategy compact" || exit 1
  run main $main "$c --strategy sorted" || exit 1
done
