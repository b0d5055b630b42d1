#!/bin/bash
# Attention combine rework check + big-model shapes: attention / engine tests, long-context traces,
# attention micro-bench, then bench.py at the 70B and 405B shapes on one GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4c}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_engine.py $R/tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
case $rc in 0|1|4|5) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
for args in "8000 8192 1 1" "8000 8192 4 1" "8000 8192 1 8"; do
  timeout -k 10 120 python -u $R/scripts/trace_attention.py $args >> $O/trace_attn.log 2>&1 || exit $?
done
timeout -k 10 300 python -u $R/scripts/bench_attn.py > $O/bench_attn.log 2>&1 || exit $?
B="--no-cli --no-f32kv --no-prefill4k --no-cap128k"
timeout -k 10 500 python3 $R/bench.py $B --shape llama3_3_70b --steps 32 --warmup 4 --long-ctx 0 > $O/bench_70b.log 2>&1 || exit $?
timeout -k 10 700 python3 $R/bench.py $B --shape llama3_1_405b --steps 12 --warmup 3 --long-ctx 0 --prompt 32 > $O/bench_405b.log 2>&1 || exit $?
exit 0
