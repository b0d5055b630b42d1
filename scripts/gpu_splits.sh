# narrow GEMM split-K workgroup target sweep (grid fill vs combine cost)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sp
B="timeout -k 10 300 python -u scripts/bench_gemm.py 8 32 64"
for t in 512 1024; do
  DL_GEMM_WG_TARGET=$t DL_GEMM_MAX_SPLITS=16 $B > gpurun_out/sp/t$t.txt 2>&1 || exit 1
  DL_GEMM_WG_TARGET=$t DL_GEMM_MAX_SPLITS=16 DL_GEMM_L16=0 $B > gpurun_out/sp/t${t}_nol16.txt 2>&1 || exit 1
done
exit 0
