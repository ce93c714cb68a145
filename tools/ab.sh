#!/bin/bash
# Interleaved A/B of library variants on the bench (run on the GPU box).
# usage: tools/ab.sh "<bench args>" variantA variantB ...   (build_variants/<v>/libcvq.so)
# Each run's stdout (JSON) and stderr are kept under gpurun_out/ab/<variant>_<rep>.{json,err};
# a run that prints no JSON is reported with its exit code and the tail of its stderr.
args=$1; shift
out=${AB_OUT:-gpurun_out/ab}
mkdir -p $out
for rep in 1 2; do
  for v in "$@"; do
    echo -n "$v rep $rep: "
    CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 120 python bench.py --cpu-baseline 0 $args \
        > $out/${v}_$rep.json 2> $out/${v}_$rep.err
    rc=$?
    if [ -s $out/${v}_$rep.json ]; then
      python3 tools/bench_brief.py < $out/${v}_$rep.json
    else
      echo "NO JSON (exit $rc): $(tail -n 3 $out/${v}_$rep.err | tr '\n' ' ')"
    fi
  done
done
