# narrow GEMM pipeline depth sweep (stage buffers per token width, 16-block-chunk kernel on/off)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stg
B="timeout -k 10 300 python -u scripts/bench_gemm.py"
$B 8 32 64 > gpurun_out/stg/base.txt 2>&1 &&
DL_GEMM_L16=0 $B 8 > gpurun_out/stg/l16off_s2.txt 2>&1 &&
DL_GEMM_L16=0 DL_GEMM_STG1=3 $B 8 > gpurun_out/stg/l16off_s3.txt 2>&1 &&
DL_GEMM_L16=0 DL_GEMM_STG1=4 $B 8 > gpurun_out/stg/l16off_s4.txt 2>&1 &&
DL_GEMM_STG2=3 $B 32 > gpurun_out/stg/m32_s3.txt 2>&1 &&
DL_GEMM_STG2=4 $B 32 > gpurun_out/stg/m32_s4.txt 2>&1 &&
DL_GEMM_STG4=2 $B 64 > gpurun_out/stg/m64_s2.txt 2>&1 &&
DL_GEMM_STG4=3 $B 64 > gpurun_out/stg/m64_s3.txt 2>&1
