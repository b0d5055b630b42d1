#!/bin/bash
# Round-3 iteration: wide GEMM (2 blocks per stage) tests and prefill points.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3dbg4}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "gemm or batched or prefill or wide or outlier or slots or paged" > $O/tests.log 2>&1 || exit $?
for c in 256 1024; do
  timeout -k 10 200 python -u $R/bench.py --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk $c > $O/bench_c$c.log 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_pf -- python3 $R/bench.py --steps 4 --warmup 1 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk 1024 > $O/prof_pf.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_pf > $O/prof_pf.md 2>&1
exit 0
