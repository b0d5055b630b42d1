#!/bin/bash
# A/B of the fused attention block on one box: per-kernel tables with and without it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  DL_ATTN_BLOCK=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof$v -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench$v.log 2>&1 || exit $?
  python3 $R/scripts/prof_summary.py $O/prof$v > $O/sum$v.md 2>&1
done
