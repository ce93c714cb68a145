set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04l
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_sorted_gpu.py tests/test_sorted_width_gpu.py tests/test_fullsize_oracle_gpu.py tests/test_gpu_parity.py \
    > gpurun_out/r04l/pytest.txt 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/r04l/pytest.txt; exit 1; }
tail -1 gpurun_out/r04l/pytest.txt
for c in 3 5; do
  echo "== cfg $c 5000"; AB_OUT=gpurun_out/r04l/c${c}_d5000 bash tools/ab.sh "--config $c --steps 20 --warmup 3 --e2e 0" pf nopf || exit 1
  echo "== cfg $c 625"; AB_OUT=gpurun_out/r04l/c${c}_d625 bash tools/ab.sh "--config $c --dates-per-gpu 625 --inflight 1 --steps 20 --warmup 3 --e2e 0" pf nopf || exit 1
done
