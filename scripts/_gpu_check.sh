#!/bin/bash
# GPU health check of the current tree: GPU tests, the headline bench, batched decode points.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed: $?"; tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
grep '"metric"' gpurun_out/bench.log
for b in 8 64; do timeout -k 10 200 python -u bench.py --batch $b --steps 16 --warmup 4 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k > gpurun_out/bench_b$b.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_b$b.log; done
