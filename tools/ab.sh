#!/bin/bash
# Interleaved A/B of library variants on the bench (run on the GPU box).
# usage: tools/ab.sh "<bench args>" variantA variantB ...
args=$1; shift
for rep in 1 2 3; do
  for v in "$@"; do
    CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 120 python bench.py --cpu-baseline 0 $args 2>/dev/null | \
      python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', 'rep $rep', round(d['value']), 'solve_us', round(d['kernels']['solve']['avg_us'],1), 'mass_us', round(d['kernels']['mass']['avg_us'],1), 'tables_us', round(d['kernels']['tables']['avg_us'],1))"
  done
done
