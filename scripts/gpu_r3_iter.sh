#!/bin/bash
# Fused-attention-block iteration: diagnostics, correctness tests, timeline trace, A/B decode bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3g}
mkdir -p $O
timeout -k 10 200 python -u $R/scripts/diag_attn_block.py > $O/diag.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "attn_block or greedy or decode_greedy" > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python $R/scripts/trace_attn_block.py 100 > $O/trace.log 2>&1 || exit $?
for v in 1 0; do
  DL_ATTN_BLOCK=$v timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench$v.log 2>&1 || exit $?
done
