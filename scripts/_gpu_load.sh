#!/bin/bash
# GPU check of the file load pipeline: engine tests (file-loaded models, TP slices), then the
# full-size 8B load benchmark.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_xgmi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/load_tests.log 2>&1 || { tail -30 gpurun_out/load_tests.log; exit 1; }
tail -2 gpurun_out/load_tests.log
timeout -k 10 400 python -u scripts/bench_load.py --keep > gpurun_out/load_bench.log 2>&1 || { tail -30 gpurun_out/load_bench.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_load.py >> gpurun_out/load_bench.log 2>&1 || { tail -30 gpurun_out/load_bench.log; exit 1; }
cat gpurun_out/load_bench.log
