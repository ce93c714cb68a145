#!/bin/bash
# phase stamps of COMPACT at small / full blocks (cfg 5 625 and 5000 dates, cfg 2 1000 dates)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06h
mkdir -p $out
for a in "--config 5 --dates 625" "--config 2" "--config 5 --dates 1" "--config 2 --dates 1"; do
  tag=$(echo $a | tr -d ' -')
  timeout -k 10 200 python3 tools/stamps.py $a --strategy compact > $out/st_$tag.txt 2>&1 || exit 1
  echo "== $a"; grep -A14 "per-WG total cycles" $out/st_$tag.txt
done
