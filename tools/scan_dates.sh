#!/bin/bash
# single_solve scan over dates per launch (one batch at a time): the 8-GPU strong-scaling
# ceiling measured on one GPU.  GPU box.  usage: tools/scan_dates.sh <tag> [extra bench args]
set -uo pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
scan() {   # config, dates...
  local c=$1; shift
  for d in "$@"; do
    timeout -k 10 240 python3 bench.py --config $c --dates-per-gpu $d --inflight 1 --steps 20 --warmup 3 \
        --e2e 0 --cpu-baseline 0 "${EXTRA[@]}" > $out/c${c}_d${d}.json 2> $out/c${c}_d${d}.err \
      || { echo "cfg $c dates $d failed rc=$?"; tail -5 $out/c${c}_d${d}.err; exit 1; }
    echo "cfg $c dates $d: $(python3 tools/bench_brief.py < $out/c${c}_d${d}.json)" | tee -a $out/dates_scan.txt
  done
}
EXTRA=("$@")
for c in ${SCAN_CFGS:-3 5 4 2}; do
  case $c in
    3|5) scan $c 5000 2500 1250 625 ;;
    4) scan 4 2000 1000 500 250 ;;
    2) scan 2 1000 500 250 125 ;;
  esac
done
