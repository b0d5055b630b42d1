#!/bin/bash
# rocprofv3 kernel traces: batch-1 decode, batch-8 decode, 32-token prefill chunks
set -o pipefail
R=$PWD
cd /tmp && export TMPDIR=/tmp
for b in 1 8; do
  OUT=$R/gpurun_out/prof_r2_b$b; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 $R/scripts/profile_decode.py --steps 64 --batch $b > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
  tail -1 $OUT/log.txt
  python3 $R/scripts/rocpd_summary.py $OUT/run_results.db > $OUT/summary.md 2>&1 || true
  head -16 $OUT/summary.md
done
OUT=$R/gpurun_out/prof_r2_prefill; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cli --no-f32kv --long-ctx 0 --no-prefill4k > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
python3 $R/scripts/rocpd_summary.py $OUT/run_results.db > $OUT/summary.md 2>&1 || true
head -20 $OUT/summary.md
