# dequant without per-lane shifts: numerics + microbench + decode/eval bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/deq
E="timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm or split_det" > gpurun_out/deq/test.txt 2>&1 &&
timeout -k 10 300 python -u scripts/bench_gemm.py 8 32 64 128 > gpurun_out/deq/gemm.txt 2>&1 &&
$E --batch 8 > gpurun_out/deq/b8.txt 2>&1 &&
$E --batch 64 > gpurun_out/deq/b64.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 64 --warmup 8 > gpurun_out/deq/b1_full.txt 2>&1
