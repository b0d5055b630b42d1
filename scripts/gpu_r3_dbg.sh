#!/bin/bash
# Round-3 iteration: tensor-parallel batched rows all-reduced in the GEMM epilogues.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3dbg8}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_xgmi.py -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
for b in 1 0; do
  DL_TP_BATCHED=$b DL_BENCH_SAME_GPU=1 timeout -k 10 300 python -u $R/bench.py --gpus 2 --steps 16 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_tp2_b$b.log 2>&1 || exit $?
done
DL_BENCH_SAME_GPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tp2 -- python3 $R/bench.py --gpus 2 --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/prof_tp2.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_tp2 > $O/prof_tp2.md 2>&1
exit 0
