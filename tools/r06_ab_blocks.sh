#!/bin/bash
# A/B over full batches and small per-GPU blocks: in-tree library vs build_variants/<v>[,<v2>...] (each
# variant's full-batch parity tests first, through CVQ_LIB)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; v=$2
out=gpurun_out/$tag
mkdir -p $out
for vv in ${v//,/ }; do
  CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$vv/libcvq.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 \
      --timeout-method thread tests/test_fullbatch_gpu.py tests/test_e2e_fullbatch_gpu.py tests/test_q4_zero_gpu.py \
      tests/test_gpu_parity.py > $out/pytest_$vv.txt 2>&1 || { tail -30 $out/pytest_$vv.txt; exit 1; }
  echo "$vv: $(tail -1 $out/pytest_$vv.txt)"
done
run() {
  CVQ_LIB=$2 timeout -k 10 300 python3 bench.py $3 --other-configs none --cpu-baseline 0 --e2e 0 > $out/b.json 2>$out/b.err \
    || { echo "$1 failed"; tail -3 $out/b.err; return 1; }
  python3 -c "
import json; d=json.load(open('$out/b.json')); print('$1', '$3', round(d['value']/1e6,3), round(d['single_solve']['value']/1e6,3), round(d['roofline']['avg_launch_us'],2), d['var_checksum'])" | tee -a $out/ab.txt
}
main=$GRAFT_REPO_ROOT/copula-msm-and-copula-garch-var_amd/copula_var/libcvq.so
for rep in 1 2; do
  for args in "--steps 50 --warmup 5" "--steps 50 --warmup 5 --dates-per-gpu 125 --inflight 1" \
              "--config 5 --steps 30 --warmup 5" "--config 5 --steps 50 --warmup 5 --dates-per-gpu 625 --inflight 1"; do
    run main $main "$args" || exit 1
    for vv in ${v//,/ }; do run $vv $GRAFT_REPO_ROOT/build_variants/$vv/libcvq.so "$args" || exit 1; done
  done
done
