#!/bin/bash
# GPU box: default-mode bench lines (batches in flight + single solve) of library variants,
# interleaved.  usage: tools/ab_lib.sh <tag> "<cfgs>" <reps> v1 v2 ...
set -uo pipefail
tag=$1; cfgs=$2; reps=$3; shift 3
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $reps); do for c in $cfgs; do for v in "$@"; do
  f=$out/c${c}_${v}_$r
  CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 240 python3 bench.py --config $c --steps 50 \
      --warmup 5 --e2e 0 --cpu-baseline 0 > $f.json 2> $f.err || { echo "cfg $c $v failed"; tail -5 $f.err; exit 1; }
  echo "cfg $c $v rep $r: $(python3 tools/bench_brief.py < $f.json)" | tee -a $out/ab.txt
done; done; done
