#!/bin/bash
# Round-3 iteration: GEMV geometry sweep, serving throughput (contiguous and paged KV).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3dbg6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/bench_gemv.py auto 16x2 32x4 32x7 64x2 > $O/gemv_sweep.log 2>&1 || exit $?
timeout -k 10 300 python3 -u $R/scripts/bench_api.py --n 64 --max-tokens 64 > $O/api.log 2>&1 || exit $?
timeout -k 10 300 python3 -u $R/scripts/bench_api.py --n 64 --max-tokens 64 --kv-pages 160 --kv-page-size 64 > $O/api_paged.log 2>&1 || exit $?
exit 0
