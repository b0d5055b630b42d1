#!/bin/bash
# GPU parity pass: greedy equality vs CPU, Q80 TP vs CPU Q80 TP, then the headline bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_xgmi.py -x -q --timeout 120 --timeout-method thread -k "greedy_64 or q80_tp_matches_cpu" > gpurun_out/parity_tests.log 2>&1 || { tail -40 gpurun_out/parity_tests.log; exit 1; }
tail -2 gpurun_out/parity_tests.log
timeout -k 10 300 python -u bench.py --steps 32 --warmup 4 > gpurun_out/parity_bench.log 2>&1 || { tail -30 gpurun_out/parity_bench.log; exit 1; }
tail -1 gpurun_out/parity_bench.log
