#!/bin/bash
# PMC traffic passes (FETCH_SIZE / WRITE_SIZE and the SQ groups) of k_sorted for BASELINE configs 3 / 5 / 4,
# keyed to the library build (tools/pmc_summary.py writes gpurun_out/pmc_traffic_cfg<N>.json).  GPU box.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for c in 3 5 4; do
  bash tools/pmc.sh r05fin_c$c --config $c --e2e 0 --steps 20 > gpurun_out/pmc_sorted_c$c.txt 2>&1 \
    || { echo "pmc cfg $c failed"; tail -20 gpurun_out/pmc_sorted_c$c.txt; exit 1; }
  tail -1 gpurun_out/pmc_sorted_c$c.txt | cut -c1-400
done
