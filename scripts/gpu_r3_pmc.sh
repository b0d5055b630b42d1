#!/bin/bash
# Round-3 PMC pass (one counter set per run, counters only) + kernel trace of 1024-row prefill
# forwards (wide GEMM, LDS-DMA prefill attention); wide-GEMM numerics first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "gemm or wide or prefill_mfma or attention or long_context" > $O/tests.log 2>&1 || exit $?
timeout -k 10 60 $R/build/probe_attn 150 > $O/probe_attn.log 2>&1 || exit $?
CN="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 180 rocprofv3 --pmc $CN --output-format csv -d $O/pf -- python3 $R/scripts/profile_prefill.py --tokens 1024 --reps 2 > $O/pf.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/pf > $O/pf.md 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/pf_trace -- python3 $R/scripts/profile_prefill.py --tokens 1024 --reps 2 > $O/pf_trace.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/pf_trace > $O/pf_trace.md 2>&1
timeout -k 10 300 python -u $R/bench.py --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv > $O/bench.log 2>&1 || exit $?
exit 0
