#!/bin/bash
# Round-3 iteration: LDS-DMA prefill attention tests and prefill points.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3dbg5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "attention or prefill or wide or long_context or paged" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u $R/bench.py --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk 1024 > $O/bench_c1024.log 2>&1 || exit $?
DL_PF_ATTN_DMA=0 timeout -k 10 300 python -u $R/bench.py --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk 1024 > $O/bench_c1024_old.log 2>&1 || exit $?
exit 0
