#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for hg in "" 1 2 4; do
  DL_ATTN_HG=$hg timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/attn_hg$hg.log 2>&1 || { echo "attn bench failed"; tail gpurun_out/attn_hg$hg.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/attn_hg$hg.log | head -14
done
