#!/bin/bash
# Wide-GEMM + MFMA decode attention iteration: numerics tests, attention microbench A/B, prefill
# points (A/B against the narrow kernel), headline bench, per-kernel profile of a 512-row prefill.
# usage (through gpurun): bash scripts/gpu_r3_wide.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3wide}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "gemm or batched or prefill or wide or outlier or slots or attention" > $O/tests.log 2>&1 || exit $?
DL_ATTN_MFMA=1 timeout -k 10 200 python -u $R/scripts/bench_attn.py > $O/attn_mfma.log 2>&1 || exit $?
DL_ATTN_MFMA=0 timeout -k 10 200 python -u $R/scripts/bench_attn.py > $O/attn_valu.log 2>&1 || exit $?
for c in 256 512 1024; do
  timeout -k 10 200 python -u $R/bench.py --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk $c > $O/bench_c$c.log 2>&1 || exit $?
done
DL_GEMM_WIDE=0 timeout -k 10 200 python -u $R/bench.py --steps 8 --warmup 2 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk 256 > $O/bench_narrow.log 2>&1 || exit $?
timeout -k 10 240 python -u $R/bench.py --steps 64 --warmup 8 > $O/bench.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_pf -- python3 $R/bench.py --steps 4 --warmup 1 --no-cli --long-ctx 0 --no-f32kv --prefill-chunk 512 > $O/prof_pf.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_pf > $O/prof_pf.md 2>&1
exit 0
