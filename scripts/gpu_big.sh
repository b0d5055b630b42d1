#!/bin/bash
# Big-model shapes on one GPU: shape tests against the CPU backend, then bench.py 70B / 405B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-big}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_engine.py -k "big_model or 8b_shape or attn_block" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
B="--no-cli --no-f32kv --no-prefill4k --no-cap128k --long-ctx 0"
timeout -k 10 500 python3 $R/bench.py $B --shape llama3_3_70b --steps 32 --warmup 4 > $O/bench_70b.log 2>&1 || exit $?
timeout -k 10 700 python3 $R/bench.py $B --shape llama3_1_405b --steps 12 --warmup 3 --prompt 32 > $O/bench_405b.log 2>&1 || exit $?
exit 0
