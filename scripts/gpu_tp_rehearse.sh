# Same-GPU rehearsal of the multi-rank bench path (torch.distributed.run, all ranks on GPU 0,
# DL_BENCH_SAME_GPU=1: labelled as a rehearsal, not a scaling point). TP2 at 8B, TP4 at 1B shape.
set -o pipefail
mkdir -p gpurun_out/tp_rehearse
export DL_BENCH_SAME_GPU=1 HSA_ENABLE_IPC_MODE_LEGACY=0 GPU_MAX_HW_QUEUES=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 32 --warmup 8 --no-prefill4k > gpurun_out/tp_rehearse/tp2.log 2>&1 || exit 1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 4 --steps 32 --warmup 8 --shape llama3_2_1b --no-prefill4k > gpurun_out/tp_rehearse/tp4.log 2>&1
