#!/bin/bash
# Round-3 iteration: residual + RMS norm split between producer / consumer GEMVs (decode, TP1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3un}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for u in 0 1; do
  DL_UNORM=$u timeout -k 10 300 python -u $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_un$u.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -- python3 $R/bench.py --steps 16 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/prof.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof > $O/prof.md 2>&1
exit 0
