#!/bin/bash
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k > gpurun_out/bench_small.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_small.log; exit 1; }
grep -o '"eval_ms_per_token": [0-9.]*\|"pred_ms_per_token": [0-9.]*\|"value": [0-9.]*' gpurun_out/bench_small.log
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_r2_b1b; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 $R/scripts/profile_decode.py --steps 64 --batch 1 > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
python3 $R/scripts/rocpd_summary.py $OUT/run_results.db > $OUT/summary.md 2>&1 || true
grep -E "argmax|embedding|attnKernel" $OUT/summary.md
