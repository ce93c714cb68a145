#!/bin/bash
# Round-end validation on the GPU box: the full GPU suite, smoke(), the PMC traffic passes of the
# default bench (written into profiles/ on the box so the following bench attaches them), the
# default bench, and the rocprofv3 kernel trace of the default command.  usage: tools/round_end.sh <tag>
set -uo pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/pytest_gpu.txt 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest_gpu.txt; exit 1; }
tail -1 $out/pytest_gpu.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 $out/smoke.txt; exit 1; }
echo "smoke ok"
bash tools/pmc.sh $tag > $out/pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $out/pmc.txt; exit 1; }
cp gpurun_out/pmc_traffic_cfg2.json profiles/pmc_traffic_cfg2.json
tail -2 $out/pmc.txt
timeout -k 10 600 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err \
    || { echo "bench failed rc=$?"; tail -20 $out/bench_default.err; exit 1; }
python3 tools/bench_brief.py < $out/bench_default.json
bash tools/profile_default.sh $tag > $out/profile.txt 2>&1 || { echo "profile failed"; tail -20 $out/profile.txt; exit 1; }
tail -8 $out/profile.txt
