#!/bin/bash
# PMC passes (counters only, one set per run) over narrow GEMM launches at 8 tokens.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmcg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/p1 -- python3 $R/scripts/prof_gemm_m8.py > $O/p1.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/p1 > $O/p1.md 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/p2 -- python3 $R/scripts/prof_gemm_m8.py > $O/p2.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/p2 > $O/p2.md 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -- python3 $R/scripts/prof_gemm_m8.py > $O/p3.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/p3 > $O/p3.md 2>&1
exit 0
