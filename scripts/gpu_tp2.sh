#!/bin/bash
# Tensor-parallel checks on one GPU: the xGMI / fused-exchange tests, the bench-harness tests (a
# same-GPU TP2 bench of the 1B shape), then bench.py --gpus 2 on the 8B shape (two ranks on one GPU
# over the xGMI comm). usage: scripts/gpu_tp2.sh <out-name>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tp2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_xgmi.py $R/tests/test_bench_harness.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
DL_BENCH_SAME_GPU=1 timeout -k 10 600 python3 -u $R/bench.py --gpus 2 --steps 16 --warmup 4 > $O/bench.log 2>&1 || exit $?
grep "self-test" $O/bench.log; tail -1 $O/bench.log
