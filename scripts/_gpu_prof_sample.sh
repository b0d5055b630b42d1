#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof_sample
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sample -o run -- python3 $R/scripts/bench_sample.py 64 20 > $R/gpurun_out/prof_sample/log.txt 2>&1 || { tail -20 $R/gpurun_out/prof_sample/log.txt; exit 1; }
find $R/gpurun_out/prof_sample -name "*kernel_stats.csv" | head -1 | xargs cat | head -12
