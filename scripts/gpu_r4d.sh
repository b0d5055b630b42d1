#!/bin/bash
# Paged-KV attention tests, then a per-kernel profile of the 70B decode.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4d}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_engine.py -k "paged or split or long" -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_70b -- python3 $R/bench.py --shape llama3_3_70b --steps 16 --warmup 3 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k --no-cap128k > $O/prof_70b.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_70b > $O/prof_70b.md 2>&1
exit 0
