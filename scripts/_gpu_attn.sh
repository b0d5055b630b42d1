set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DL_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_engine.py > gpurun_out/r2_attn_tests.log 2>&1 && \
timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/r2_bench_attn.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 32 --warmup 4 --no-cli > gpurun_out/r2_bench_n1_attn.log 2>&1 && \
timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 64 > gpurun_out/r2_bench_gemm_v1.log 2>&1
