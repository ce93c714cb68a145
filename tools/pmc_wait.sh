#!/bin/bash
# Stall breakdown of the solve kernel (GPU box): two counter passes per case.
# usage: tools/pmc_wait.sh <tag> "<bench args>" ["<bench args>" ...]
set -uo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
P0="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
P1="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
k=0
for args in "$@"; do
  d=$out/case$k
  i=0
  for P in "$P0" "$P1"; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $d/p$i -o run -- \
        python3 bench.py --cpu-baseline 0 --other-configs none --steps 5 --warmup 1 --e2e 0 $args > $d.p$i.log 2>&1 \
      || { echo "pmc case $k pass $i failed rc=$?"; tail -5 $d.p$i.log; exit 1; }
    i=$((i+1))
  done
  echo "== case $k: $args" | tee -a $out/summary.txt
  python3 tools/pmc_summary.py $d $args 2>&1 | grep -B1 -A20 "^void cvq::k_" | grep -v "^{" | tee -a $out/summary.txt
  k=$((k+1))
done
rm -f gpurun_out/pmc_traffic_cfg*.json
