#!/bin/bash
# Round-3 GEMV geometry sweep + per-kernel decode profile (run through gpurun).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r3c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/bench_gemv.py auto 16x1 16x2 16x4 32x1 32x2 32x4 32x7 64x1 64x2 64x3 > $R/gpurun_out/r3c/gemv_sweep.log 2>&1 || exit $?
timeout -k 10 240 python3 -m pytest $R/tests/test_bench_harness.py -m gpu -x -q > $R/gpurun_out/r3c/harness.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3c/prof -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $R/gpurun_out/r3c/prof_bench.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $R/gpurun_out/r3c/prof > $R/gpurun_out/r3c/prof_summary.md 2>&1
