#!/bin/bash
# GPU box: the full GPU suite, then a single-solve strategy scan and phase stamps of the SORTED
# configs.  usage: tools/gpu_check.sh <tag> [cfgs] [strategies] [dates]
set -uo pipefail
tag=$1
cfgs=${2:-"5 3"}; strats=${3:-"sorted sweep"}; dates=${4:-"5000 625"}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.txt 2>&1
rc=$?; tail -3 $out/pytest.txt; [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; grep -E "FAILED|Error" $out/pytest.txt | head -20; exit 1; }
bash tools/strat_scan.sh $tag "$cfgs" "$strats" "$dates" || exit 1
for c in $cfgs; do for st in $strats; do for d in $dates; do
  [ $d -le 1250 ] || continue
  timeout -k 10 120 python3 tools/stamps.py --config $c --strategy $st --dates $d > $out/st_c${c}_d${d}_$st.txt 2>&1 \
    || { echo "stamps $c $st $d failed"; exit 1; }
done; done; done
echo done
