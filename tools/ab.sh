#!/bin/bash
# Interleaved A/B of library variants on the bench (run on the GPU box).
# usage: tools/ab.sh "<bench args>" variantA variantB ...   (build_variants/<v>/libcvq.so)
args=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    echo -n "$v rep $rep: "
    CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 120 python bench.py --cpu-baseline 0 $args 2>/dev/null | python3 tools/bench_brief.py
  done
done
