#!/bin/bash
# LDS counters of the solve kernel, CVQ_SORT_BANK=1 vs 0 (GPU box).  usage: tools/pmc_lds.sh <tag> <config>...
set -uo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
P="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"
for c in "$@"; do
  for b in 1 0; do
    d=$out/c${c}_b$b
    CVQ_SORT_BANK=$b timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $d/p0 -o run -- \
        python3 bench.py --cpu-baseline 0 --steps 5 --warmup 1 --e2e 0 --config $c > $d.log 2>&1 || { echo "pmc $c $b failed rc=$?"; exit 1; }
    python3 tools/pmc_summary.py $d --config $c > $d.summary.txt 2>&1 || true
    echo "== cfg $c bank $b"; grep -A12 "k_sorted" $d.summary.txt | head -14 || true
  done
done
