#!/bin/bash
# Head-major KV layout check: full GPU tests, attention micro-bench + timeline, decode bench with
# the long-context point.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-kvl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 300 python -u $R/scripts/bench_attn.py > $O/bench_attn.log 2>&1 || exit $?
timeout -k 10 120 python -u $R/scripts/trace_attention.py 8000 8192 1 1 > $O/trace.log 2>&1 || exit $?
timeout -k 10 400 python3 $R/bench.py --steps 32 --warmup 4 --no-cli --no-f32kv --no-prefill4k > $O/bench.log 2>&1 || exit $?
exit 0
