#!/bin/bash
# Interleaved A/B of runtime variants selected by environment settings (GPU box).
# usage: tools/ab_env.sh "<bench args>" "ENV=a" "ENV=b" ...
# Each run's stdout / stderr are kept under gpurun_out/ab_env/; a run without JSON is
# reported with its exit code and the tail of its stderr.
args=$1; shift
out=${AB_OUT:-gpurun_out/ab_env}
mkdir -p $out
for rep in 1 2 3; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 120 python bench.py --cpu-baseline 0 $args > $out/v${i}_$rep.json 2> $out/v${i}_$rep.err
    rc=$?
    if [ -s $out/v${i}_$rep.json ]; then
      echo -n "$v rep $rep: "; python3 tools/bench_brief.py < $out/v${i}_$rep.json
    else
      echo "$v rep $rep: NO JSON (exit $rc): $(tail -n 3 $out/v${i}_$rep.err | tr '\n' ' ')"
    fi
  done
done
