#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "DL_GEMM_WG=256 DL_GEMM_MAXS=8" "DL_GEMM_WG=512 DL_GEMM_MAXS=16" "DL_GEMM_WG=1024 DL_GEMM_MAXS=32"; do
  echo "== $cfg"; env $cfg timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 > gpurun_out/sweep2.log 2>&1 || { echo "bench failed"; exit 1; }
  grep -v amdgpu.ids gpurun_out/sweep2.log
done
