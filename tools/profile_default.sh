#!/bin/bash
# rocprofv3 kernel trace + stats of EXACTLY the default bench command (`python3 bench.py`),
# then the dominant kernel's durations split by bench leg (tools/trace_legs.py).  GPU box.
# usage: tools/profile_default.sh <tag>      -> gpurun_out/prof_<tag>/
set -uo pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 bench.py > $out/bench.json 2> $out/stderr.log || { echo "rocprofv3 run failed rc=$?"; tail -5 $out/stderr.log; exit 1; }
find $out -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
python3 tools/trace_legs.py $out --steps 100 --warmup 5 > $out/kernel_legs.txt
cat $out/kernel_legs.txt
