set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DL_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "sampler or sample" > gpurun_out/r2_sample_tests.log 2>&1 && \
PROBE=1 timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 > gpurun_out/r2_bench_gemm_probe.log 2>&1 && \
timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/r2_bench_attn.log 2>&1
