# Same-GPU rehearsal of the multi-rank bench path (torch.distributed.run, all ranks on GPU 0,
# DL_BENCH_SAME_GPU=1: labelled as a rehearsal, not a scaling point). TP2 at 8B (HIP's default
# hardware queues, then one per process), TP4 at the 1B shape.
set -o pipefail
mkdir -p gpurun_out/tp_rehearse
export DL_BENCH_SAME_GPU=1 HSA_ENABLE_IPC_MODE_LEGACY=0
F="--steps 32 --warmup 8 --no-prefill4k --no-cap128k --no-f32kv --long-ctx 0"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 $F > gpurun_out/tp_rehearse/tp2.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 $F > gpurun_out/tp_rehearse/tp2_q1.log 2>&1 || exit 1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 4 --shape llama3_2_1b $F > gpurun_out/tp_rehearse/tp4.log 2>&1
