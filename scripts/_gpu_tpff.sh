#!/bin/bash
# fence-free pull all-reduce: xGMI tests + same-GPU TP2/TP4 rehearsals
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xgmi_tests.log 2>&1 || { echo "xgmi tests failed"; tail -30 gpurun_out/xgmi_tests.log; exit 1; }
tail -1 gpurun_out/xgmi_tests.log
for w in 2 4; do
  DL_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2952$w bench.py --gpus $w --steps 32 --warmup 8 --no-prefill4k --long-ctx 0 --no-f32kv > gpurun_out/r2_tp${w}_ff.log 2>&1 || { echo "tp$w failed"; tail -20 gpurun_out/r2_tp${w}_ff.log; exit 1; }
  grep -o '"value": [0-9.]*\|"eval_ms_per_token": [0-9.]*\|"pred_ms_per_token": [0-9.]*\|"tp_comm": "[a-z]*"' gpurun_out/r2_tp${w}_ff.log | tr '\n' ' '; echo
done
