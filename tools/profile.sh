#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (run on the GPU box).
# usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 bench.py --cpu-baseline 0 --other-configs none "$@" > $out/bench.json 2> $out/stderr.log
find $out -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
ls -R $out | head -30
