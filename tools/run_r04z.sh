#!/bin/bash
# r04z (final build): single-solve dates-per-launch scans (the 8-GPU strong-scaling ceiling on one GPU)
# and an 8-rank gloo rehearsal of the strong-scaling bench with the local-solve / all-gather split.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
SCAN_CFGS="3 5 4" bash tools/scan_dates.sh r04z || exit 1
mkdir -p gpurun_out/r04z
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 8 --backend gloo --config 3 --global-dates 5000 --steps 10 --warmup 2 --e2e 0 --cpu-baseline 0 \
    > gpurun_out/r04z/rehearsal_c3_8ranks.json 2> gpurun_out/r04z/rehearsal_c3_8ranks.err || { echo "rehearsal failed"; tail -20 gpurun_out/r04z/rehearsal_c3_8ranks.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04z/rehearsal_c3_8ranks.json').read().strip().splitlines()[-1])
print('8 gloo ranks on one GPU, cfg 3 strong 5000:', round(d['value']), 'VaR-dates/s; single_solve', {k: d['single_solve'][k] for k in ('ms_per_step', 'local_solve_ms', 'allgather_finalize_ms')})
"
