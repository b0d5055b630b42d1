#!/bin/bash
# rocprofv3 kernel trace of the headline decode (optionally with an env override as $1)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof_decode${2:-}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ -n "$1" ]; then export $1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --no-f32kv > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
python3 $R/scripts/rocpd_summary.py $OUT/run_results.db | head -25
