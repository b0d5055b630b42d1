#!/bin/bash
# Fused-FFN-block + 128-token GEMM tile iteration: correctness tests, GEMM sweep, A/B decode bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3ffn}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "ffn_block or attn_block or greedy or prefill" > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "gemm" > $O/ops.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_xgmi.py -x -v --timeout 150 --timeout-method thread -k "fused_blocks or tp_matches_single or batched" > $O/xgmi.log 2>&1 || exit $?
timeout -k 10 200 python -u $R/scripts/bench_gemm.py 64 128 > $O/gemm.log 2>&1 || exit $?
DL_FFN_BLOCK=0 timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_off.log 2>&1 || exit $?
timeout -k 10 300 python $R/bench.py --steps 64 --warmup 8 > $O/bench_on.log 2>&1 || exit $?
DL_FFN_RING_EARLY=1 timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_early.log 2>&1 || exit $?
DL_FFN_BLOCK=0 timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_off2.log 2>&1 || exit $?
