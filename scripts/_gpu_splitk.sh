#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q -k "gemm or batched or prefill" --timeout 120 --timeout-method thread > gpurun_out/splitk_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/splitk_tests.log; exit 1; }
tail -1 gpurun_out/splitk_tests.log
for wg in 256 512 1024; do
  echo "== DL_GEMM_WG=$wg"; DL_GEMM_WG=$wg timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 > gpurun_out/bench_gemm_nf_wg$wg.log 2>&1 || { echo "bench failed"; exit 1; }
  head -6 gpurun_out/bench_gemm_nf_wg$wg.log | tail -5
done
timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --long-ctx 0 --no-cli --no-f32kv > gpurun_out/bench_nf.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_nf.log; exit 1; }
grep -o '"eval_ms_per_token": [0-9.]*\|"pred_ms_per_token": [0-9.]*\|"prompt_4k_eval_ms_per_token": [0-9.]*\|"value": [0-9.]*' gpurun_out/bench_nf.log
for b in 8 64; do timeout -k 10 200 python -u bench.py --batch $b --steps 16 --warmup 4 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k > gpurun_out/bench_nf_b$b.log 2>&1 || exit 1; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_nf_b$b.log; done
