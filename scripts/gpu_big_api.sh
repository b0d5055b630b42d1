# 70B-shaped decode on one GPU and dllama-api serving throughput (64 / 16 concurrent requests).
set -o pipefail
mkdir -p gpurun_out/big
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0 --tp-rank-compute= --steps 32 --warmup 8"
timeout -k 10 400 python -u bench.py --shape llama3_3_70b $F > gpurun_out/big/b70.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/bench_api.py --n 64 > gpurun_out/big/api64.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_api.py --n 16 > gpurun_out/big/api16.log 2>&1
