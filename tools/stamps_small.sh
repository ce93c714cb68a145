#!/bin/bash
# GPU box: SORTED phase stamps of a few dates alone on the GPU (the latency chain without
# contention).  usage: tools/stamps_small.sh <tag> "<cfgs>" "<dates>" [strategy]
set -uo pipefail
tag=$1; cfgs=$2; dates=$3; st=${4:-sorted}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for c in $cfgs; do for d in $dates; do
  timeout -k 10 120 python3 tools/stamps.py --config $c --strategy $st --dates $d > $out/st_c${c}_d${d}_$st.txt 2>&1 \
    || { echo "stamps $c $d failed"; tail -5 $out/st_c${c}_d${d}_$st.txt; exit 1; }
  grep -v amdgpu.ids $out/st_c${c}_d${d}_$st.txt
done; done
