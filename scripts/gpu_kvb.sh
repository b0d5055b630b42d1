#!/bin/bash
# Blocked head-major KV check: full GPU tests, attention bench, decode bench (all points).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-kvb}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 300 python -u $R/scripts/bench_attn.py > $O/attn.log 2>&1 || exit $?
timeout -k 10 500 python3 $R/bench.py --steps 32 --warmup 4 --no-cli > $O/bench.log 2>&1 || exit $?
exit 0
