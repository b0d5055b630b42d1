# narrow vs wide (128-row tiles) MFMA GEMM at 16-64 tokens
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wm
timeout -k 10 300 python -u scripts/bench_gemm.py 16 32 48 64 > gpurun_out/wm/narrow.txt 2>&1 &&
DL_GEMM_WIDE_MIN=16 timeout -k 10 300 python -u scripts/bench_gemm.py 16 32 48 64 > gpurun_out/wm/wide.txt 2>&1 &&
DL_GEMM_WIDE_MIN=17 timeout -k 10 300 python -u bench.py --batch 32 --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k > gpurun_out/wm/b32_wide.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --batch 32 --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k > gpurun_out/wm/b32_narrow.txt 2>&1 &&
DL_GEMM_WIDE_MIN=17 timeout -k 10 300 python -u bench.py --batch 64 --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k > gpurun_out/wm/b64_wide.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --batch 64 --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k > gpurun_out/wm/b64_narrow.txt 2>&1
