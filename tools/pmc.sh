#!/bin/bash
# PMC counter passes for the bench kernels (run on the GPU box).  One pass per
# counter group, --kernel-trace only (no sys/runtime tracing with --pmc).
# usage: tools/pmc.sh <tag> [bench args...]
set -uo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p $out
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $out/p$i -o run -- \
      python3 bench.py --cpu-baseline 0 --other-configs none "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $out "$@" > $out/summary.txt
cat $out/summary.txt
