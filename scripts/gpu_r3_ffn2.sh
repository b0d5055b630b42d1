#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3ffn2}
mkdir -p $O
DL_FFN_BLOCK=1 timeout -k 10 200 python -u $R/scripts/trace_ffn_block.py > $O/trace.log 2>&1 || exit $?
DL_FFN_BLOCK=1 DL_FFN_RING_EARLY=1 timeout -k 10 200 python -u $R/scripts/trace_ffn_block.py > $O/trace_early.log 2>&1 || exit $?
DL_FFN_BLOCK=1 DL_FFN_MARGIN=0 timeout -k 10 200 python -u $R/scripts/trace_ffn_block.py > $O/trace_m0.log 2>&1 || exit $?
DL_FFN_BLOCK=1 DL_FFN_MARGIN=0 timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_m0.log 2>&1 || exit $?
DL_FFN_BLOCK=1 DL_FFN_MARGIN=0 DL_FFN_RING_EARLY=1 timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_m0e.log 2>&1 || exit $?
