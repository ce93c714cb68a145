#!/bin/bash
# k_msm_scanwin_w phase ablation (GPU box): cvq_msm_tables time for cfg 4 (k = 6) with each library variant.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  CVQ_LIB=$GRAFT_REPO_ROOT/build_variants/$v/libcvq.so timeout -k 10 120 python3 tools/time_msm_tables.py --config 4 --steps 20 \
      2>&1 | tail -1 | sed "s/^/$v: /" || exit 1
done
