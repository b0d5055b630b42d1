# Closing measurements: 70B-shaped decode and batched decode steps on the current tree.
set -o pipefail
mkdir -p gpurun_out/close
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0 --tp-rank-compute= --steps 32 --warmup 8"
timeout -k 10 400 python -u bench.py --shape llama3_3_70b $F > gpurun_out/close/b70.log 2>&1 || exit 1
NO_TESTS=1 BATCHES="4 8 64" bash scripts/gpu_batch_bench.sh
