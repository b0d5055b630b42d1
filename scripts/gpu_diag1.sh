#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-diag1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python -u $R/scripts/trace_decode_engine.py 100 5 > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 python -u $R/scripts/diag_pde_positions.py > $O/positions.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k --no-cap128k > $O/prof_b1.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b1 > $O/prof_b1.md 2>&1
exit 0
