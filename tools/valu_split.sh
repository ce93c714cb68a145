#!/bin/bash
# GPU box: instruction split of the SORTED solve (tools/valu_split.py) for configs 5 and 3, one
# --pmc pass each.  usage: tools/valu_split.sh <tag>
set -uo pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/vsplit_$tag
mkdir -p $out
ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VMEM_RD"
for c in 5 3; do
  reach=$([ $c = 5 ] && echo 32779 || echo 131095)
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $out/c$c -o run -- \
      python3 tools/valu_split.py --config $c > $out/c$c.log 2>&1 || { echo "cfg $c failed rc=$?"; tail -5 $out/c$c.log; exit 1; }
  nodes=$(python3 -c "import json,sys; print([json.loads(l) for l in open('$out/c$c.log') if l.startswith('{')][-1]['nodes_per_date'])")
  python3 tools/valu_split.py --report $out/c$c --config $c --nodes $nodes --reach $reach --dates 5000 | tee $out/c$c.txt
done
