#!/bin/bash
# Instruction-mix / LDS / wait counters of the solve kernel for one strategy (GPU box).
# usage: tools/pmc_quick.sh <tag> [bench args...]
set -uo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmcq_$tag
mkdir -p $out
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $out/p$i -o run -- \
      python3 bench.py --cpu-baseline 0 --other-configs none --steps 5 --warmup 1 "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $out "$@" > $out/summary.txt
grep -A20 "k_direct\|k_compact\|k_sorted" $out/summary.txt | head -44 || true
