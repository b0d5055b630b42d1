#!/bin/bash
# PMC passes on the batched GEMM (w13 28672x4096, M=32) and the batch-1 GEMV on the same matrix
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
export M=32
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc2/list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/pmc2/a -o run --output-format csv -- python3 $R/scripts/prof_gemm_one.py > $R/gpurun_out/pmc2/a.log 2>&1 && echo "pass a ok" && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -d $R/gpurun_out/pmc2/b -o run --output-format csv -- python3 $R/scripts/prof_gemm_one.py > $R/gpurun_out/pmc2/b.log 2>&1 && echo "pass b ok" && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace -d $R/gpurun_out/pmc2/c -o run --output-format csv -- python3 $R/scripts/prof_gemm_one.py > $R/gpurun_out/pmc2/c.log 2>&1 && echo "pass c ok"
ls -R $R/gpurun_out/pmc2 | head -30
