#!/bin/bash
# cfg 4 (3-D SORTED) A/B of the range-sum word prefetch (GPU box): full batch with e2e, 500 and 250 dates.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
echo "== cfg 4 full + e2e"; AB_OUT=gpurun_out/r04u/full bash tools/ab.sh "--config 4 --steps 20 --warmup 3" head nopf || exit 1
echo "== cfg 4 500"; AB_OUT=gpurun_out/r04u/d500 bash tools/ab.sh "--config 4 --dates-per-gpu 500 --inflight 1 --steps 20 --warmup 3 --e2e 0" head nopf || exit 1
echo "== cfg 4 250"; AB_OUT=gpurun_out/r04u/d250 bash tools/ab.sh "--config 4 --dates-per-gpu 250 --inflight 1 --steps 20 --warmup 3 --e2e 0" head nopf || exit 1
