#!/bin/bash
# fitted-nu (nu = 5.364) SORTED range-sum ILP A/B (GPU box): 1 / 2 / 4 nodes in flight for the general-power nodes,
# plus the wide 2-D min-waves change at 625 dates (head = ilp2 library).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for c in 2 5; do
  echo "== cfg $c nu 5.364"; AB_OUT=gpurun_out/r04r/c${c}_nu bash tools/ab.sh "--config $c --nu 5.364 --strategy sorted --steps 20 --warmup 3 --e2e 0" ilp2 ilp1 ilp4 || exit 1
done
for c in 5 3; do
  echo "== cfg $c 625 (head)"; AB_OUT=gpurun_out/r04r/c${c}_625 bash tools/ab.sh "--config $c --dates-per-gpu 625 --inflight 1 --steps 20 --warmup 3 --e2e 0" ilp2 || exit 1
done
