set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export DL_SKIP_BUILD=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $R/gpurun_out/pmc/a -o run --output-format csv -- python3 $R/scripts/prof_gemm_one.py > $R/gpurun_out/pmc/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace -d $R/gpurun_out/pmc/b -o run --output-format csv -- python3 $R/scripts/prof_gemm_one.py > $R/gpurun_out/pmc/b.log 2>&1
