#!/bin/bash
# PMC passes (counters only, one set per run) over 1024-row prefill forwards of the 8B shapes:
# LDS bank conflicts / waits of the prefill attention and the wide GEMM.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmcp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
P="$R/scripts/profile_prefill.py --tokens 1024 --reps 2"
timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/p1 -- python3 $P > $O/p1.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/p1 > $O/p1.md 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/p2 -- python3 $P > $O/p2.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/p2 > $O/p2.md 2>&1
exit 0
