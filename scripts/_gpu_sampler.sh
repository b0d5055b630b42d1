#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof_sample2
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "sampl" > gpurun_out/sampler_tests.log 2>&1 || { tail -40 gpurun_out/sampler_tests.log; exit 1; }
tail -2 gpurun_out/sampler_tests.log
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sample2 -o run -- python3 $R/scripts/bench_sample.py 64 20 > $R/gpurun_out/prof_sample2/log.txt 2>&1 ) || { tail -20 gpurun_out/prof_sample2/log.txt; exit 1; }
timeout -k 10 500 python -u scripts/bench_api.py > gpurun_out/api_bench2.log 2>&1 || { tail -30 gpurun_out/api_bench2.log; exit 1; }
grep sampled_vs_greedy gpurun_out/api_bench2.log
