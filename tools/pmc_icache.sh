#!/bin/bash
# GPU box: instruction-cache counters of the solve kernel (SQC ICACHE hits / misses, SQ
# instruction fetches and issue waits), one pass each.  usage: tools/pmc_icache.sh <tag> [bench args...]
set -uo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmci_$tag
mkdir -p $out
passes=(
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES"
  "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"
  "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $out/p$i -o run -- \
      python3 bench.py --cpu-baseline 0 --other-configs none --steps 5 --warmup 1 --e2e 0 --inflight 1 "$@" > $out/p$i.log 2>&1 \
      || { echo "pass $i failed rc=$?"; tail -3 $out/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $out "$@" > $out/summary.txt
grep -A12 "k_sorted\|k_compact" $out/summary.txt | head -40 || true
