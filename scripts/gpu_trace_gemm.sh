# per-workgroup timeline of the narrow GEMMs (old LDS-staged and register-ring kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tg
timeout -k 10 300 python -u scripts/trace_gemm.py 8 32 64 > gpurun_out/tg/old.txt 2>&1 &&
DL_GEMM_REG=64 timeout -k 10 300 python -u scripts/trace_gemm.py 8 32 64 > gpurun_out/tg/reg.txt 2>&1 &&
DL_GEMM_REG=64 timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/tg/rccl.txt 2>&1
