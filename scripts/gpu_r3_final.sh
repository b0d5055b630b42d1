#!/bin/bash
# Round-3 closing checks: full GPU suite, smoke, the driver's bench command, a same-GPU TP2
# rehearsal through the self-launching bench, per-kernel profiles of decode and batch-8 decode.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3final}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
DL_BENCH_SAME_GPU=1 timeout -k 10 400 python -u $R/bench.py --gpus 2 --steps 16 --warmup 4 --no-prefill4k --long-ctx 0 --no-f32kv > $O/bench_tp2.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/prof_b1.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b1 > $O/prof_b1.md 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -- python3 $R/bench.py --batch 8 --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/prof_b8.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b8 > $O/prof_b8.md 2>&1
exit 0
