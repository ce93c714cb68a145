#!/bin/bash
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06k
mkdir -p $out
for a in "--config 3 --dates 625" "--config 3 --dates 1" "--config 4 --dates 250" "--config 4 --dates 1"; do
  tag=$(echo $a | tr -d ' -')
  timeout -k 10 200 python3 tools/stamps.py $a --strategy sorted > $out/st_$tag.txt 2>&1 || exit 1
  echo "== $a"; grep -A16 "per-WG total cycles" $out/st_$tag.txt
done
