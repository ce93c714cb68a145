#!/bin/bash
# Interleaved A/B: the in-tree libcvq.so ("main") against build_variants/<v>/libcvq.so, cfg 2 (100 steps)
# and cfg 5 (50 steps), two reps.  usage: tools/r06_ab.sh <tag> <variant> [<variant> ...]
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
run() {  # label lib args
  CVQ_LIB=$2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>$out/b.err \
    || { echo "$1 failed"; tail -3 $out/b.err; return 1; }
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,2), round(d['single_solve']['value']/1e6,2), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/ab.txt
}
main=$GRAFT_REPO_ROOT/copula-msm-and-copula-garch-var_amd/copula_var/libcvq.so
for rep in 1 2; do
  for cfg in "--steps 100 --warmup 5" "--config 5 --steps 50 --warmup 5"; do
    run main $main "$cfg" || exit 1
    for v in "$@"; do run $v $GRAFT_REPO_ROOT/build_variants/$v/libcvq.so "$cfg" || exit 1; done
  done
done
