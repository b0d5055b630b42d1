# narrow GEMM: 1 vs 2 row tiles (64 / 128 rows) per workgroup, numerics with RT=2 forced
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rt
B="timeout -k 10 300 python -u scripts/bench_gemm.py 8 32 64"
E="timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --no-cli --no-cap128k --long-ctx 0 --no-f32kv --no-prefill4k"
DL_GEMM_RT1=2 DL_GEMM_RT2=2 DL_GEMM_RT4=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm_q40 or split_det" > gpurun_out/rt/test.txt 2>&1 &&
DL_GEMM_RT1=2 DL_GEMM_RT2=2 DL_GEMM_RT4=2 $B > gpurun_out/rt/rt2.txt 2>&1 &&
DL_GEMM_RT1=2 DL_GEMM_RT2=2 DL_GEMM_RT4=2 $E --batch 64 > gpurun_out/rt/b64_rt2.txt 2>&1 &&
DL_GEMM_RT1=2 DL_GEMM_RT2=2 DL_GEMM_RT4=2 $E --batch 32 > gpurun_out/rt/b32_rt2.txt 2>&1 &&
DL_GEMM_RT1=2 DL_GEMM_RT2=2 DL_GEMM_RT4=2 $E --batch 8 > gpurun_out/rt/b8_rt2.txt 2>&1
