#!/bin/bash
# GPU box: SQ instruction counters of the cfg-2 COMPACT solve for the base library and the
# ablation builds under build_variants/abl{3,2,1} (stop before the block tail / before the
# levels / after the tables).  usage: tools/phase_pmc.sh <tag>
set -uo pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM"
for v in base abl3 abl2 abl1; do
  lib=copula-msm-and-copula-garch-var_amd/copula_var/libcvq.so
  [ $v != base ] && lib=build_variants/$v/libcvq.so
  CVQ_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $out/$v -o run -- \
      python3 tools/phase_pmc.py --run > $out/$v.log 2>&1 || { echo "variant $v failed rc=$?"; tail -5 $out/$v.log; exit 1; }
done
python3 tools/phase_pmc.py --report $out base abl3 abl2 abl1 | tee $out/phase.txt
