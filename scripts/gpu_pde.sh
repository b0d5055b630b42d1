#!/bin/bash
# Decode-engine bring-up: its own tests first (stop on any crash / timeout), then the engine suite
# and the headline bench. usage: scripts/gpu_pde.sh <out-name>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pde}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_engine.py -k "decode_engine" -x -v --timeout 180 --timeout-method thread > $O/t_pde.log 2>&1
rc=$?; tail -5 $O/t_pde.log
case $rc in 0|1) ;; *) echo "pde tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_engine.py -q --timeout 180 --timeout-method thread > $O/t_engine.log 2>&1
rc=$?; tail -3 $O/t_engine.log
case $rc in 0|1) ;; *) echo "engine tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 500 python -u $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
DL_DECODE_ENGINE=0 timeout -k 10 300 python -u $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cli --no-prefill4k --no-f32kv > $O/bench_noengine.log 2>&1 || exit $?
tail -1 $O/bench_noengine.log
exit 0
