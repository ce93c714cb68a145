# usage: bash tools/gpu_ab.sh <tag> "<cfg list>" "<strategy list>" [pytest -k expr]
set -o pipefail
tag=$1; cfgs=$2; strats=$3; kexpr=$4
mkdir -p gpurun_out/$tag
if [ -n "$kexpr" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sorted_gpu.py -x -q -k "$kexpr" --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/$tag/pytest.txt; exit 1; }
  tail -1 gpurun_out/$tag/pytest.txt
fi
for c in $cfgs; do for s in $strats; do
  timeout -k 10 120 python bench.py --config $c --strategy $s --cpu-baseline 0 --steps 20 ${BENCH_EXTRA} > gpurun_out/$tag/b_${c}_$s.json 2> gpurun_out/$tag/b_${c}_$s.err || { echo BENCH_FAIL; tail gpurun_out/$tag/b_${c}_$s.err; exit 1; }
  echo "cfg $c $s: $(python tools/bench_brief.py < gpurun_out/$tag/b_${c}_$s.json)"
done; done
