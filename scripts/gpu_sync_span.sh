# Sync-span cost at a TP8 rank (default vs DL_SYNC_MEASURE=0) and the tests that read Sync.
set -o pipefail
mkdir -p gpurun_out/span
for m in 1 0; do
  DL_SYNC_MEASURE=$m timeout -k 10 120 python -u scripts/tp_rank_compute.py --tp 8 2>&1 | grep -v "^ℹ\|amdgpu" >> gpurun_out/span/runs.log || exit 1
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_xgmi.py -k "sync or bytes or q80_tp or engine_tp" > gpurun_out/span/tests.log 2>&1
