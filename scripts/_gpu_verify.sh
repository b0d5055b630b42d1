#!/bin/bash
# GPU verification pass: op/engine/xGMI tests, then the headline bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py tests/test_gpu_xgmi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { tail -30 gpurun_out/verify_tests.log; exit 1; }
tail -3 gpurun_out/verify_tests.log
timeout -k 10 300 python -u bench.py --steps 32 --warmup 4 > gpurun_out/verify_bench.log 2>&1 || { tail -30 gpurun_out/verify_bench.log; exit 1; }
tail -3 gpurun_out/verify_bench.log
