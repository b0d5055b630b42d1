#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for b in 2 3 4; do for g in 5 2; do
  DL_GEMM_MIN=$g timeout -k 10 200 python -u bench.py --batch $b --steps 32 --warmup 8 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k > gpurun_out/gmin.log 2>&1 || { echo fail; exit 1; }
  echo "batch $b DL_GEMM_MIN=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gmin.log)"
done; done
