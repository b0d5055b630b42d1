#!/bin/bash
# Round-3 checkpoint: GPU tests, headline bench, batched / prefill points, per-kernel profiles.
# usage (through gpurun): bash scripts/gpu_r3_baseline.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3base}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 240 python -u $R/bench.py --steps 64 --warmup 8 > $O/bench.log 2>&1 || exit $?
for b in 8 64; do
  timeout -k 10 200 python -u $R/bench.py --batch $b --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_b$b.log 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/prof_b1.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b1 > $O/prof_b1.md 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -- python3 $R/bench.py --batch 8 --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/prof_b8.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b8 > $O/prof_b8.md 2>&1
exit 0
