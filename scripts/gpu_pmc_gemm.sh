#!/bin/bash
# PMC passes (counters only, one set per run) over narrow GEMM launches (w13 8B shape) at each
# token count in $M_LIST (default "8 64"); summaries per pass under gpurun_out/$1.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmcg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
C3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES"
for M in ${M_LIST:-8 64}; do
  for p in 1 2 3; do
    eval C=\$C$p
    M=$M timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/m${M}_p$p -- python3 $R/scripts/prof_gemm_one.py > $O/m${M}_p$p.log 2>&1 || exit $?
    python3 $R/scripts/pmc_summary.py $O/m${M}_p$p > $O/m${M}_p$p.md 2>&1
  done
done
exit 0
