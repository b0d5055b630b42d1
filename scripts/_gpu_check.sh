#!/bin/bash
# GPU health check of the current tree: GPU tests, then the headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed: $?"; tail -30 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
