#!/bin/bash
# 8-rank tensor-parallel rehearsal of bench.py on one GPU (fused xGMI exchange, RCCL fallback path)
set -o pipefail
mkdir -p gpurun_out
DL_BENCH_SAME_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 16 --warmup 4 --no-prefill4k --long-ctx 0 > gpurun_out/r2_tp8_samegpu.log 2>&1 || { echo "tp8 failed"; tail -30 gpurun_out/r2_tp8_samegpu.log; exit 1; }
grep '"metric"' gpurun_out/r2_tp8_samegpu.log | cut -c1-900
