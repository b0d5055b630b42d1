#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 --no-cli > gpurun_out/bench_ff.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_ff.log; exit 1; }
grep -o '"eval_ms_per_token": [0-9.]*\|"pred_ms_per_token": [0-9.]*\|"prompt_4k_eval_ms_per_token": [0-9.]*\|"value": [0-9.]*\|"long_ctx_pred_ms_per_token": [0-9.]*' gpurun_out/bench_ff.log
for cfg in "DL_GEMM_STG1=3" "DL_GEMM_STG1=4" "DL_GEMM_STG2=3" "DL_GEMM_WG=512 DL_GEMM_STG1=3 DL_GEMM_STG2=3" "DL_GEMM_STG4=2"; do
  echo "== $cfg"; env $cfg timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 64 > gpurun_out/sweep.log 2>&1 || { echo "bench failed"; exit 1; }
  head -6 gpurun_out/sweep.log | tail -5
done
