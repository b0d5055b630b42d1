#!/bin/bash
# Round-4 GPU session: full GPU suite, smoke, the driver's bench command and a per-kernel profile of
# batch-1 decode. usage: scripts/gpu_r4.sh <out-name> [skip-tests]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest $R/tests -m gpu -q -x --timeout 180 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
fi
timeout -k 10 300 python -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -- python3 $R/bench.py --steps 32 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k --no-cap128k > $O/prof_b1.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b1 > $O/prof_b1.md 2>&1
exit 0
