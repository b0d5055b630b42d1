# software-pipelined narrow GEMM block loop: numerics, microbench, decode batches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/swp
B="timeout -k 10 300 python -u scripts/bench_gemm.py 8 32 64"
E="timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm_q40 or split_det" > gpurun_out/swp/test.txt 2>&1 &&
DL_GEMM_L16=0 $B > gpurun_out/swp/nol16.txt 2>&1 &&
$B > gpurun_out/swp/l16.txt 2>&1 &&
DL_GEMM_L16=0 $E --batch 8 > gpurun_out/swp/b8.txt 2>&1 &&
$E --batch 8 > gpurun_out/swp/b8_l16.txt 2>&1 &&
$E --batch 32 > gpurun_out/swp/b32.txt 2>&1 &&
$E --batch 64 > gpurun_out/swp/b64.txt 2>&1
