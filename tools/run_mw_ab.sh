#!/bin/bash
# min-waves A/B for the 2-D SORTED kernel (GPU box): head vs mw6 at cfg 5 / cfg 3, full batch and 625 dates.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for c in 5 3; do
  echo "== cfg $c 5000"; AB_OUT=gpurun_out/r04q/c${c}_full bash tools/ab.sh "--config $c --steps 20 --warmup 3 --e2e 0" head mw6 || exit 1
  echo "== cfg $c 625"; AB_OUT=gpurun_out/r04q/c${c}_625 bash tools/ab.sh "--config $c --dates-per-gpu 625 --inflight 1 --steps 20 --warmup 3 --e2e 0" head mw6 || exit 1
done
