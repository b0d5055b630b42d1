#!/bin/bash
# TEMP: 16-token GEMM tile stage-count sweep (bench_gemm M=8/16, bench.py batch 8).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-stg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
for s in 2 3 4; do
  DL_GEMM_STG1=$s timeout -k 10 300 python -u $R/scripts/bench_gemm.py 8 16 > $O/gemm_s$s.log 2>&1 || exit $?
  DL_GEMM_STG1=$s timeout -k 10 240 python3 $R/bench.py --batch 8 --steps 16 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k --no-cap128k > $O/b8_s$s.log 2>&1 || exit $?
done
exit 0
