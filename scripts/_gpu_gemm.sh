set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DL_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_engine.py > gpurun_out/r2_gemm_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gemm.py 8 16 32 > gpurun_out/r2_bench_gemm.log 2>&1 && \
for b in 8 32; do timeout -k 10 300 python -u bench.py --steps 32 --warmup 4 --batch $b --no-cli --long-ctx 0 > gpurun_out/r2_bench_b$b.log 2>&1 || exit 1; done
