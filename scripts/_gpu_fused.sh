#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_xgmi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 || { tail -40 gpurun_out/fused_tests.log; exit 1; }
tail -2 gpurun_out/fused_tests.log
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 > gpurun_out/fused_bench.log 2>&1 || { tail -30 gpurun_out/fused_bench.log; exit 1; }
tail -1 gpurun_out/fused_bench.log
DL_ATTN_FUSED=0 timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --no-cli --no-f32kv > gpurun_out/unfused_bench.log 2>&1 || { tail -30 gpurun_out/unfused_bench.log; exit 1; }
tail -1 gpurun_out/unfused_bench.log
