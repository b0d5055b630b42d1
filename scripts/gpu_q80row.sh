# Wave-local Q80 exchange tail: TP numerics tests (verbose, durations), then the 7-worker CLI case.
set -o pipefail
mkdir -p gpurun_out/q80row
timeout -k 10 500 python -u -m pytest -x -v --durations=0 --timeout 170 --timeout-method thread tests/test_gpu_xgmi.py tests/test_gpu_engine.py -k "(tp or xgmi or compute_only or fused) and not cli_root and not api" > gpurun_out/q80row/tests2.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --durations=0 --timeout 170 --timeout-method thread tests/test_gpu_xgmi.py -k "cli_root" > gpurun_out/q80row/cli.log 2>&1
