#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for f in 1 0; do
  echo "== DL_GEMM_FUSE_NORM=$f"
  DL_GEMM_FUSE_NORM=$f timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --long-ctx 0 --no-cli --no-f32kv > gpurun_out/bench_fuse$f.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_fuse$f.log; exit 1; }
  grep -o '"eval_ms_per_token": [0-9.]*\|"pred_ms_per_token": [0-9.]*\|"prompt_4k_eval_ms_per_token": [0-9.]*\|"value": [0-9.]*' gpurun_out/bench_fuse$f.log
  for b in 8 64; do DL_GEMM_FUSE_NORM=$f timeout -k 10 200 python -u bench.py --batch $b --steps 16 --warmup 4 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k > gpurun_out/bench_fuse${f}_b$b.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_fuse${f}_b$b.log; done
done
