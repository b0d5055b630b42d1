#!/bin/bash
# Full GPU check: GPU tests, TP2/TP4 same-GPU rehearsals of bench.py, GEMM split-K sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for w in 2 4; do
  DL_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2951$w bench.py --gpus $w --steps 32 --warmup 8 --no-prefill4k --long-ctx 0 > gpurun_out/r2_tp${w}_samegpu.log 2>&1 || { echo "tp$w failed"; tail -20 gpurun_out/r2_tp${w}_samegpu.log; exit 1; }
  grep '"metric"' gpurun_out/r2_tp${w}_samegpu.log | cut -c1-400
done
for wg in 256 512 1024; do
  echo "== DL_GEMM_WG=$wg"; DL_GEMM_WG=$wg timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 > gpurun_out/bench_gemm_wg$wg.log 2>&1 || { echo "bench failed"; exit 1; }
  head -5 gpurun_out/bench_gemm_wg$wg.log
done
