#!/bin/bash
# GPU box: single-solve A/B of library variants (build_variants/<v>/libcvq.so) over configs,
# strategies and dates per launch.  usage: tools/ab_scan.sh <tag> "<cfgs>" "<strategies>" "<dates>" v1 v2 ...
set -uo pipefail
tag=$1; cfgs=$2; strats=$3; dates=$4; shift 4
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for c in $cfgs; do for st in $strats; do for d in $dates; do for v in "$@"; do
  f=$out/c${c}_${st}_d${d}_$v
  CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 240 python3 bench.py --config $c --strategy $st \
      --dates-per-gpu $d --inflight 1 --steps 20 --warmup 3 --e2e 0 --cpu-baseline 0 > $f.json 2> $f.err \
    || { echo "cfg $c $st $d $v failed"; tail -5 $f.err; exit 1; }
  echo "cfg $c $st dates $d $v: $(python3 tools/bench_brief.py < $f.json)" | tee -a $out/scan.txt
done; done; done; done
